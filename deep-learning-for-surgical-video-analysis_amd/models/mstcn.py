"""MS-TCN temporal model — MI355X build (drop-in for the reference's models/mstcn.py).

``MultiStageModel_S`` / ``SingleStageModel`` / ``DilatedResidualLayer`` keep the
reference's constructor signatures, submodule names and ``state_dict`` keys
(mstcn.py:94-214).  Arithmetic: the video's feature sequence is consumed
time-major ([T, f_dim], the LFB row layout — the reference's ``[1, f_dim, T]`` input
is a transposed view of exactly that), the 1x1 convs are MFMA GEMMs, each dilated
residual layer (dilated k=3 conv + ReLU + 1x1 conv + residual) is ONE svk kernel, and
the inter-stage softmax over classes is one kernel.  Everything runs in f32 (the
reference path is f32; this model is HBM/launch-bound, not MFMA-bound).

Output: ``[stages, B, classes, T]`` like the reference, returned as a view of the
time-major [stages, B, T, classes] buffer the kernels write.
"""
import copy

import torch
import torch.nn as nn

from svk import ops
from svk.pack import get_packed
from ._common import check_inference

try:
    from mamba_ssm import Mamba
except ImportError:
    Mamba = None


def _w1x1(conv):
    return conv.weight.detach().float()[:, :, 0].contiguous(), conv.bias.detach().float().contiguous()


class DilatedResidualLayer(nn.Module):
    """(mstcn.py:181-214)."""

    def __init__(self, dilation, in_channels, out_channels, causal_conv=False, kernel_size=3):
        super().__init__()
        self.causal_conv = causal_conv
        self.dilation = dilation
        self.kernel_size = kernel_size
        pad = dilation * (kernel_size - 1) if causal_conv else dilation
        self.conv_dilated = nn.Conv1d(in_channels, out_channels, kernel_size, padding=pad, dilation=dilation)
        self.conv_1x1 = nn.Conv1d(out_channels, out_channels, 1)
        self.dropout = nn.Dropout()

    def _pack(self, dt):
        wd = self.conv_dilated.weight.detach().float().permute(2, 0, 1).contiguous()   # [3][F_out][F_in]
        w1, b1 = _w1x1(self.conv_1x1)
        return dict(wd=wd, bd=self.conv_dilated.bias.detach().float().contiguous(), w1=w1, b1=b1)

    def forward_tm(self, x):
        """x [T, F] time-major f32 -> [T, F]."""
        p = get_packed(self, torch.float32, self._pack)
        return ops.mstcn_layer(x, p["wd"], p["bd"], p["w1"], p["b1"], self.dilation, self.causal_conv)

    def forward(self, x):
        """Reference signature: x [B, F, T] -> [B, F, T]."""
        check_inference(self, x)
        return torch.stack([self.forward_tm(xb.t().float().contiguous()).t() for xb in x], 0)


class SingleStageModel(nn.Module):
    """(mstcn.py:153-178)."""

    def __init__(self, num_layers, num_f_maps, dim, num_classes, causal_conv=False):
        super().__init__()
        if num_layers > 0 and num_f_maps > 64:
            raise ValueError("SingleStageModel: the svk dilated-residual kernel supports num_f_maps <= 64")
        self.conv_1x1 = nn.Conv1d(dim, num_f_maps, 1)
        self.layers = nn.ModuleList([copy.deepcopy(DilatedResidualLayer(2 ** i, num_f_maps, num_f_maps,
                                                                        causal_conv=causal_conv))
                                     for i in range(num_layers)])
        self.conv_out_classes = nn.Conv1d(num_f_maps, num_classes, 1)

    def _pack(self, dt):
        wi, bi = _w1x1(self.conv_1x1)
        wo, bo = _w1x1(self.conv_out_classes)
        return dict(wi=wi, bi=bi, wo=wo, bo=bo)

    def forward_tm(self, x, out=None):
        """x [T, dim] time-major f32 -> class logits [T, classes] (written into ``out`` if given)."""
        p = get_packed(self, torch.float32, self._pack)
        h = ops.gemm(x, p["wi"], p["bi"])
        for layer in self.layers:
            h = layer.forward_tm(h)
        return ops.gemm(h, p["wo"], p["bo"], out=out)

    def forward(self, x):
        check_inference(self, x)
        return torch.stack([self.forward_tm(xb.t().float().contiguous()).t() for xb in x], 0)


class MultiStageModel_S(nn.Module):
    """(mstcn.py:94-130)."""

    def __init__(self, mstcn_stages, mstcn_layers, mstcn_f_maps, mstcn_f_dim, out_features, mstcn_causal_conv):
        self.num_stages = mstcn_stages
        self.num_layers = mstcn_layers
        self.num_f_maps = mstcn_f_maps
        self.dim = mstcn_f_dim
        self.num_classes = out_features
        self.causal_conv = mstcn_causal_conv
        print(f"num_stages_classification: {self.num_stages}, num_layers: {self.num_layers}, num_f_maps:"
              f" {self.num_f_maps}, dim: {self.dim}")
        super().__init__()
        self.stage1_phase = SingleStageModel(self.num_layers, self.num_f_maps, self.dim, self.num_classes,
                                             causal_conv=self.causal_conv)
        self.stages = nn.ModuleList([copy.deepcopy(SingleStageModel(self.num_layers, self.num_f_maps,
                                                                    self.num_classes, self.num_classes,
                                                                    causal_conv=self.causal_conv))
                                     for s in range(self.num_stages - 1)])
        self.smoothing = False

    def forward_tm(self, x):
        """x [T, f_dim] (f32, time-major) -> [stages, T, classes] time-major logits."""
        T = x.shape[0]
        out = torch.empty(self.num_stages, T, self.num_classes, device=x.device, dtype=torch.float32)
        self.stage1_phase.forward_tm(x, out=out[0])
        for s, stage in enumerate(self.stages):
            prob = ops.softmax_rows(out[s])                       # softmax over classes (mstcn.py:126)
            stage.forward_tm(prob, out=out[s + 1])
        return out

    def forward(self, x):
        """x [B, f_dim, T] -> [stages, B, classes, T] (mstcn.py:122-130)."""
        check_inference(self, x)
        per = []
        for xb in x:                                   # batch of videos (the reference uses B = 1)
            xt = xb.t()                                # [T, f_dim]; a view when x = lfb.transpose(2, 1)
            if xt.dtype != torch.float32 or xt.stride(1) != 1:
                xt = xt.float().contiguous()
            per.append(self.forward_tm(xt))
        out = torch.stack(per, dim=1) if len(per) > 1 else per[0].unsqueeze(1)   # [S, B, T, C]
        return out.permute(0, 1, 3, 2)

    @staticmethod
    def add_model_specific_args(parser):  # pragma: no cover
        g = parser.add_argument_group(title="mstcn reg specific args options")
        g.add_argument("--mstcn_stages", default=4, type=int)
        g.add_argument("--mstcn_layers", default=10, type=int)
        g.add_argument("--mstcn_f_maps", default=64, type=int)
        g.add_argument("--mstcn_f_dim", default=2048, type=int)
        g.add_argument("--mstcn_causal_conv", action="store_true")
        return parser


class CausalMambaModel(nn.Module):
    """(mstcn.py:282-343).  Needs the ``mamba_ssm`` selective-scan kernels; like the reference it
    raises ImportError when they are unavailable (mstcn.py:301-302).  An MI355X selective-scan
    kernel is the SURVEY §8(f) rank-2 "next" item."""

    def __init__(self, mstcn_stages, mstcn_layers, mstcn_f_maps, mstcn_f_dim, out_features, mstcn_causal_conv,
                 mamba_d_state=64, mamba_d_conv=4, mamba_expand=2, mamba_dropout=0.1):
        super().__init__()
        if Mamba is None:
            raise ImportError("mamba_ssm is not installed. Please run: pip install mamba-ssm")
        raise NotImplementedError("CausalMambaModel: svk selective-scan kernel not built yet (SURVEY §8(f) rank 2)")
