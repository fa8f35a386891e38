"""Generate the golden fixtures in tests/golden/ by running the REFERENCE code.

Runs only in the survey container, where the read-only reference checkout is at
/root/reference (override with SVK_REFERENCE).  It never runs on the GPU box and
nothing in the product imports it.  Outputs are data only (inputs are regenerated
from seeds by oracle.inputs; the fixtures store input digests so a test can prove
that it regenerated the same inputs).

The reference imports third-party packages that are not installed here (timm,
mmcv, torchvision, bytecode) and two reference modules that are absent from the
snapshot (generate_LFB.py, transformer2_3_1.py).  They are replaced by the minimal
stand-ins below; only ``mmcv.cnn.ConvModule`` carries arithmetic (conv without
bias when a norm is configured -> BatchNorm2d named ``bn`` -> ReLU named
``activate``, mmcv's documented default order), every other stand-in is import-only
or an identity in eval mode.  ``Transformer2_3_1`` is replaced by a recorder that
captures the (enc_inputs, dec_inputs) it is called with, which pins the window
construction and the fc/tanh of adapter_transformer.py:329-347.

Usage:  python tests/golden/gen_golden.py        (writes tests/golden/*.npz)
"""
import os
import sys
import tempfile
import textwrap
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("SVK_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from oracle import inputs as I  # noqa: E402
from oracle import params as P  # noqa: E402

SHIMS = {
    "timm/__init__.py": "",
    "timm/layers/__init__.py": '''
        import torch, torch.nn as nn
        def to_2tuple(x):
            return tuple(x) if isinstance(x, (tuple, list)) else (x, x)
        def trunc_normal_(t, mean=0., std=1., a=-2., b=2.):
            return nn.init.trunc_normal_(t, mean, std, a, b)
        class DropPath(nn.Module):
            def __init__(self, drop_prob=0.):
                super().__init__(); self.drop_prob = drop_prob
            def forward(self, x):
                if self.drop_prob == 0. or not self.training:
                    return x
                keep = 1 - self.drop_prob
                m = x.new_empty((x.shape[0],) + (1,) * (x.ndim - 1)).bernoulli_(keep)
                return x * m / keep
    ''',
    "timm/models/__init__.py": "def register_model(f):\n    return f\n",
    "timm/models/vision_transformer.py": "def _cfg(**kw):\n    return kw\n",
    "torchvision/__init__.py": "from . import transforms, models\n",
    "torchvision/transforms/__init__.py": "",
    "torchvision/models/__init__.py": "",
    "mmcv/__init__.py": "",
    "mmcv/cnn/__init__.py": '''
        import torch.nn as nn
        class ConvModule(nn.Module):
            def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                         groups=1, bias="auto", conv_cfg=None, norm_cfg=None, act_cfg=dict(type="ReLU"),
                         inplace=True, **kw):
                super().__init__()
                with_norm = norm_cfg is not None
                if bias == "auto":
                    bias = not with_norm
                self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, bias)
                self.with_norm = with_norm
                if with_norm:
                    self.bn = nn.BatchNorm2d(out_channels)
                self.with_activation = act_cfg is not None
                if self.with_activation:
                    self.activate = nn.ReLU(inplace=inplace)
            def forward(self, x):
                x = self.conv(x)
                if self.with_norm:
                    x = self.bn(x)
                if self.with_activation:
                    x = self.activate(x)
                return x
        DepthwiseSeparableConvModule = ConvModule
    ''',
    "bytecode/__init__.py": "class Bytecode: pass\nclass Instr: pass\n",
    "generate_LFB.py": "device = 'cpu'\n",
}


def install_shims():
    d = tempfile.mkdtemp(prefix="svk_shims_")
    for rel, src in SHIMS.items():
        path = os.path.join(d, rel)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(textwrap.dedent(src))
    sys.path.insert(0, d)
    sys.path.insert(1, REF)            # top-level `visualizer` (mix_transformer_evp.py:69)
    pkg = types.ModuleType("refmodels")
    pkg.__path__ = [REF]               # so `from .segformer_head import ...` resolves (mix_transformer_evp.py:12)
    sys.modules["refmodels"] = pkg

    rec = types.ModuleType("refmodels.transformer2_3_1")

    class Transformer2_3_1(torch.nn.Module):
        calls = []

        def __init__(self, **kw):
            super().__init__()
            self.kw = kw

        def forward(self, enc_inputs, dec_inputs):
            Transformer2_3_1.calls.append((enc_inputs.detach().clone(), dec_inputs.detach().clone()))
            return dec_inputs

    rec.Transformer2_3_1 = Transformer2_3_1
    sys.modules["refmodels.transformer2_3_1"] = rec
    return Transformer2_3_1


def main():
    torch.set_num_threads(8)
    Recorder = install_shims()
    import importlib
    mte = importlib.import_module("refmodels.mix_transformer_evp")
    mstcn = importlib.import_module("refmodels.mstcn")
    at = importlib.import_module("refmodels.adapter_transformer")

    out = {}
    B = 2
    x, y, fl = I.frames(B, 0), I.segmaps(B, 0), I.flow(B, 0)
    out["in_digest_frames"] = I.digest(x)
    out["in_digest_segmaps"] = I.digest(y)
    out["in_digest_flow"] = I.digest(fl)

    for variant in ("mit_b0_evp", "mit_b2_evp", "mit_b3_evp"):
        m = getattr(mte, variant)()
        P.fill_module_(m, seed=0)
        m.eval()
        keys = sorted(m.state_dict().keys())
        out[f"{variant}_keys"] = np.array(keys)
        with torch.no_grad():
            out[f"{variant}_feat_flow"] = m(x, y, fl, return_features=True).numpy()
            if variant == "mit_b2_evp":
                out[f"{variant}_feat_noflow"] = m(x, y, None, return_features=True).numpy()
                yl, yant = m(x, y, fl)
                out[f"{variant}_logits_flow"] = yl.numpy()
                out[f"{variant}_logits_ant_flow"] = yant.numpy()
                outs = m.forward_features(x, y)
                for i, o in enumerate(outs):   # NCHW stage outputs (before flow fusion)
                    out[f"{variant}_stage{i + 1}_sum"] = o.double().sum(dim=(2, 3)).numpy()
                out[f"{variant}_stage4"] = outs[3].numpy()
                f3, f4 = m.flow_encoder(fl)
                out[f"{variant}_flow_s4"] = f4.numpy()
                hc = m.prompt_generator.init_prompts(y.view(-1, 3, 224, 224))
                out[f"{variant}_hc4"] = hc[3].numpy()
        print(variant, "params", sum(v.numel() for v in m.state_dict().values()), "keys", len(keys))

    # MS-TCN: the reference-logged config and the BASELINE config, causal; plus non-causal.
    T = 300
    for name, (S, L, Fm, D, causal) in {"mstcn_2_8_32_2048_c": (2, 8, 32, 2048, True),
                                        "mstcn_4_10_64_256_c": (4, 10, 64, 256, True),
                                        "mstcn_2_4_32_64_nc": (2, 4, 32, 64, False)}.items():
        m = mstcn.MultiStageModel_S(S, L, Fm, D, 14, causal)
        P.fill_module_(m, seed=1)
        m.eval()
        xin = I.lfb(T, D, seed=7).transpose(2, 1)          # [1, D, T] (trans_SV_output.py:276-279)
        with torch.no_grad():
            out[name] = m(xin).numpy()
        out[name + "_keys"] = np.array(sorted(m.state_dict().keys()))

    # Transformer.original_forward windowing + fc/tanh (Transformer2_3_1 recorded, not run).
    _cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self     # adapter_transformer.py:338 calls .cuda()
    try:
        m = at.Transformer(32, 2048, 14, 30)
        P.fill_module_(m, seed=2)
        m.eval()
        Tw = 75
        xg = torch.from_numpy(np.random.default_rng(8).standard_normal((1, 14, Tw)).astype(np.float32))
        lf = I.lfb(Tw, 2048, seed=9)
        Recorder.calls.clear()
        with torch.no_grad():
            m.original_forward(xg, lf)
        enc, dec = Recorder.calls[-1]
        out["trans_window_x"] = xg.numpy()
        out["trans_window_enc"] = enc.numpy()
        out["trans_window_dec"] = dec.numpy()
        out["trans_ctor"] = np.array([str(sorted(m.transformer.kw.items()))])
    finally:
        torch.Tensor.cuda = _cuda

    path = os.path.join(HERE, "reference_golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
