"""CPU-side tests of the build: C-ABI library exports, host-side module surface and weight
packing, refusal of CPU execution (no fallback), index helpers."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle import inputs as I, params as P, mit_evp as M, shapes as SH

HEADER = os.path.join(REPO, "include", "svk.h")


def _header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int|long|const char\*)\s+(svk_\w+)\s*\(([^)]*)\)\s*;", src):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(1)] = len(args)
    return out


def test_library_exports_every_header_symbol():
    from svk import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    funcs = _header_functions()
    assert len(funcs) >= 16
    for name, nargs in funcs.items():
        assert hasattr(lib, name), f"{name} declared in svk.h but not exported"
        if name in _lib.SIGNATURES:
            assert len(_lib.SIGNATURES[name]) == nargs, f"{name}: ctypes binding has wrong arity"
        elif name in _lib.LONG_FUNCS:
            assert len(_lib.LONG_FUNCS[name]) == nargs, f"{name}: ctypes binding has wrong arity"
        elif name in _lib.INT_QUERIES:
            assert len(_lib.INT_QUERIES[name]) == nargs, f"{name}: ctypes binding has wrong arity"
        else:
            assert name in _lib.STRING_FUNCS
    assert set(_lib.SIGNATURES) | set(_lib.STRING_FUNCS) | set(_lib.LONG_FUNCS) | set(_lib.INT_QUERIES) == set(funcs)


def test_mixffn_supported_query():
    """svk_mixffn_supported needs no GPU: the whole-MixFFN kernel covers the 224x224 stage-1 shapes."""
    from svk import _lib
    lib = _lib.load()
    assert lib.svk_mixffn_supported(56, 64) == 1 and lib.svk_mixffn_supported(56, 32) == 1
    assert lib.svk_mixffn_supported(28, 128) == 0 and lib.svk_mixffn_supported(14, 320) == 0


def test_fused_stem_supported_query():
    """svk_conv2d_s2d_ln_supported needs no GPU: the RGB stem (48-channel blocks -> 64) and the handcrafted prompt
    stem (48 -> 16 channels) are covered at the 224x224 width (OW = 56), other widths / channel counts are not."""
    from svk import _lib
    lib = _lib.load()
    BF16, F16 = 1, 2   # include/svk.h: SVK_F32 = 0, SVK_BF16 = 1, SVK_F16 = 2
    for dt in (F16, BF16):
        assert lib.svk_conv2d_s2d_ln_supported(dt, 48, 64, 56) == 1
        assert lib.svk_conv2d_s2d_ln_supported(dt, 48, 16, 56) == 1
        assert lib.svk_conv2d_s2d_ln_supported(dt, 32, 16, 56) == 1
        assert lib.svk_conv2d_s2d_ln_supported(dt, 48, 32, 56) == 0
        assert lib.svk_conv2d_s2d_ln_supported(dt, 48, 64, 65) == 0
        assert lib.svk_conv2d_s2d_ln_supported(dt, 64, 64, 56) == 0
    assert lib.svk_conv2d_s2d_ln_supported(0, 48, 64, 56) == 0   # f32: the stem runs unfused


def test_library_version_and_error_path():
    from svk import _lib
    lib = _lib.load()
    assert lib.svk_version().decode().startswith("svk")
    # argument validation happens on the host, before any HIP call: safe without a GPU
    rc = lib.svk_gemm(0, None, 0, None, 0, None, None, 0, None, 0, 4, 4, 4, 0, None)
    assert rc == -1 and b"svk_gemm" in lib.svk_last_error()
    rc = lib.svk_attention(0, None, 0, 0, None, 0, 0, None, 0, 0, None, 0, 0, 1, 1, 300, 1, 64, 1.0, None)
    assert rc == -1 and b"Nk" in lib.svk_last_error()


def test_tune_knobs_select_variants_only():
    """svk_tune accepts only variant-selecting knobs; the round-5 timing ablations that skipped stores or work
    ("pk_diag", "ffn_diag") exist only in a -DSVK_DIAG build, and the stream-K workspace
    registry is gone with the variant it served."""
    from svk import _lib
    lib = _lib.load()
    for knob in (b"pk_cfg", b"pk_elds", b"dw_lds", b"dw_rows", b"attn_cfg"):
        assert lib.svk_tune(knob, -1) == 0, knob
    for knob in (b"pk_diag", b"ffn_diag"):
        assert lib.svk_tune(knob, 2) == -1 and b"unknown knob" in lib.svk_last_error()
    assert not hasattr(lib, "svk_set_stream_workspace") and "svk_set_stream_workspace" not in _lib.SIGNATURES


def test_gemm_ln_requires_16_byte_outputs():
    """svk_gemm_ln stores X and H as 16-byte row chunks: an 8-byte-aligned X or H is rejected on the host before
    any launch (fake device addresses are never dereferenced)."""
    from svk import _lib
    lib = _lib.load()
    args = dict(A=0x10000, packed=0x20000, bias=0x30000, R=0x40008, gamma=0x50000, beta=0x60000, X=0x70000, H=0x80000)

    def run(**kw):
        a = dict(args, **kw)
        return lib.svk_gemm_ln(2, a["A"], 64, 320, a["packed"], a["bias"], a["R"], a["gamma"], a["beta"], 1e-6,
                               a["X"], a["H"], 320, None)
    assert run(X=0x70008) == -1 and b"misaligned" in lib.svk_last_error()
    assert run(H=0x80008) == -1 and b"misaligned" in lib.svk_last_error()
    assert run(A=0x10008) == -1


@pytest.mark.parametrize("variant", ["mit_b0_evp", "mit_b2_evp", "mit_b3_evp"])
def test_build_state_dict_matches_reference(golden, variant):
    from models import mix_transformer_evp as mte
    m = getattr(mte, variant)()
    sd = m.state_dict()
    assert sorted(sd) == list(golden[f"{variant}_keys"])
    shapes = SH.mit_evp_shapes(variant)
    for k, v in sd.items():
        assert tuple(v.shape) == tuple(shapes[k]), k
    m.load_state_dict(P.make_state_dict({k: v.shape for k, v in sd.items()}, 0), strict=True)


def test_mstcn_and_transformer_surface(golden):
    from models import mstcn, adapter_transformer
    m = mstcn.MultiStageModel_S(2, 8, 32, 2048, 14, True)
    assert sorted(m.state_dict()) == list(golden["mstcn_2_8_32_2048_c_keys"])
    assert len(m.state_dict()) == 72
    t = adapter_transformer.Transformer(32, 2048, 14, 30)
    assert sorted(t.state_dict()) == sorted(SH.transformer_shapes(32, 2048, 14))
    from oracle import mamba as OM
    mm = mstcn.CausalMambaModel(2, 8, 64, 2048, 14, True)      # tecno.py:153 (svk scan, no mamba_ssm)
    assert {k: tuple(v.shape) for k, v in mm.state_dict().items()} == OM.mamba_shapes(2048, 64, 8, 14)


def test_no_cpu_fallback():
    import svk
    from models import mix_transformer_evp as mte, mstcn
    m = mte.mit_b0_evp().eval()
    with pytest.raises(svk.SvkError, match="GPU"):
        m(I.frames(1), I.segmaps(1), None, return_features=True)
    with pytest.raises(svk.SvkError, match="train-mode"):
        mte.mit_b0_evp().train().flow_encoder.forward(torch.zeros(1, 2, 8, 8))
    ms = mstcn.MultiStageModel_S(1, 2, 8, 16, 14, True).eval()
    with pytest.raises(svk.SvkError):
        ms(torch.zeros(1, 16, 10))


def test_head_fold_is_exact_on_cpu():
    """Host-side weight folding of SegFormerHead (resize-first + linear_c*/fuse/BN -> one matrix)
    reproduces the reference op order (oracle) in fp64 on CPU."""
    from models import mix_transformer_evp as mte
    m = mte.mit_b2_evp()
    m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0))
    p = m.head._pack(torch.float64)
    sd = {k: v.double() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(0)
    dims = (64, 128, 320, 512)
    sides = (56, 28, 14, 7)
    outs = [(torch.randn(2, s * s, c, generator=g, dtype=torch.float64), s, s) for c, s in zip(dims, sides)]
    ref = M.segformer_head(outs, sd, return_features=True)
    r = []
    for t, H, W in (outs[3], outs[2], outs[1], outs[0]):
        nchw = t.transpose(1, 2).reshape(2, -1, H, W)
        if H != 7:
            nchw = torch.nn.functional.interpolate(nchw, (7, 7), None, "bilinear", False)
        r.append(nchw.flatten(2).transpose(1, 2))
    r = torch.cat(r, dim=2)
    y = torch.relu(r @ p["w"].t() + p["b"].double()).mean(dim=1)
    # the folded bias is stored f32 by design (kernel ABI: biases are f32) -> ~1e-8 absolute
    np.testing.assert_allclose(y.numpy(), ref.numpy(), rtol=0, atol=1e-6)


def test_flow_bn_fold_is_exact_on_cpu():
    from models import mix_transformer_evp as mte
    from svk.pack import fold_bn
    m = mte.mit_b0_evp()
    m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0))
    fe = m.flow_encoder.double().eval()
    x = torch.randn(2, 2, 32, 32, dtype=torch.float64)
    ref = fe.bn1(fe.conv1(x))
    w, b = fold_bn(fe.conv1.weight, fe.conv1.bias, fe.bn1)
    got = torch.nn.functional.conv2d(x, w, b, stride=4, padding=3)
    np.testing.assert_allclose(got.numpy(), ref.detach().numpy(), rtol=1e-10, atol=1e-10)


def test_conv_weight_packing_order():
    """[Cout, Cin, k, k] -> [Cout, (kh, kw, ci)] must match an NHWC im2col K order."""
    from svk.pack import conv_w
    w = torch.randn(5, 3, 7, 7, dtype=torch.float64)
    x = torch.randn(1, 3, 20, 20, dtype=torch.float64)
    ref = torch.nn.functional.conv2d(x, w, stride=4, padding=3)
    xn = torch.nn.functional.pad(x, (3, 3, 3, 3)).permute(0, 2, 3, 1)   # NHWC padded
    cols = xn.unfold(1, 7, 4).unfold(2, 7, 4)                            # [1, OH, OW, C, kh, kw]
    cols = cols.permute(0, 1, 2, 4, 5, 3).reshape(1, ref.shape[2], ref.shape[3], -1)
    got = cols @ conv_w(w, torch.float64).t()
    np.testing.assert_allclose(got.permute(0, 3, 1, 2).numpy(), ref.numpy(), atol=1e-10)


@pytest.mark.parametrize("C,H,W", [(3, 224, 224), (2, 20, 28), (3, 13, 9)])
def test_stem_s2d_layout_on_cpu(C, H, W):
    """The space-to-depth stem (svk_nchw_to_s2d's block layout, restated here in torch, + the 2x2 unpadded
    conv with svk.pack.conv_w_s2d's weights) == the k = 7 / stride-4 / pad-3 conv, in float64."""
    from svk.pack import conv_w_s2d
    w = torch.randn(6, C, 7, 7, dtype=torch.float64)
    x = torch.randn(2, C, H, W, dtype=torch.float64)
    ref = torch.nn.functional.conv2d(x, w, stride=4, padding=3)
    OH, OW = ref.shape[2:]
    # block (by, bx) = rows / columns 4*b - 3 .. 4*b, channel (dy, dx, c), zeros outside the image
    xp = torch.zeros(2, C, 4 * (OH + 1), 4 * (OW + 1), dtype=torch.float64)
    xp[:, :, 3:3 + H, 3:3 + W] = x
    blocks = xp.view(2, C, OH + 1, 4, OW + 1, 4).permute(0, 2, 4, 3, 5, 1).reshape(2, OH + 1, OW + 1, 16 * C)
    cols = blocks.unfold(1, 2, 1).unfold(2, 2, 1)                          # [2, OH, OW, 16C, by, bx]
    cols = cols.permute(0, 1, 2, 4, 5, 3).reshape(2, OH, OW, -1)          # K order (by, bx, dy, dx, c)
    got = cols @ conv_w_s2d(w, torch.float64, 4).t()
    np.testing.assert_allclose(got.permute(0, 3, 1, 2).numpy(), ref.numpy(), atol=1e-10)


def test_useful_start_idx():
    from models.data_process import get_useful_start_idx, get_useful_start_idx_LFB, SeqSampler
    # reference semantics (data_process.py:307-315): per video, starts count..count+len-seq
    assert get_useful_start_idx(3, [4, 5]) == [0, 1, 4, 5, 6]
    assert get_useful_start_idx_LFB(1, [2, 1]) == [0, 1, 2]
    assert list(SeqSampler(None, [3, 1, 2])) == [3, 1, 2]


def test_synthetic_dataset_contract():
    from models.data_process import SyntheticCholecFlowDataset
    ds = SyntheticCholecFlowDataset(3)
    img, seg, flow, ph, ant = ds[1]
    assert img.shape == (3, 224, 224) and seg.shape == (3, 224, 224) and flow.shape == (2, 224, 224)
    assert ph.dtype == np.int64 and ant.dtype == np.float64 and ant.shape == (7,)
    img2 = ds[1][0]
    assert torch.equal(img, img2)
