"""Torch-facing wrappers over the svk C ABI.

Every op takes CUDA (HIP) tensors, checks layout/dtype on the host, allocates its
output through the PyTorch caching allocator (the library never allocates) and
launches on the current stream.  There is deliberately no CPU path: a CPU tensor
is an error.
"""
import os

import torch

from . import _lib

F32, BF16 = 0, 1
ACT = {None: 0, "none": 0, "gelu": 1, "relu": 2, "tanh": 3}
_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dtype_code(dt):
    try:
        return _DT[dt]
    except KeyError:
        raise _lib.SvkError(f"svk: unsupported dtype {dt} (float32 / bfloat16 only)") from None


def _chk(t, name, dtype=None):
    if t is None:
        return
    if not t.is_cuda:
        raise _lib.SvkError(f"svk: {name} must be a GPU tensor (got {t.device}); there is no CPU path")
    if dtype is not None and t.dtype != dtype:
        raise _lib.SvkError(f"svk: {name} dtype {t.dtype} != {dtype}")


def _p(t):
    return None if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _rows(t, name):
    """View a tensor as a [rows, cols] matrix with unit column stride; returns (rows, cols, ld)."""
    if t.stride(-1) != 1:
        raise _lib.SvkError(f"svk: {name} must have unit stride in its last dim")
    cols = t.shape[-1]
    rows = t.numel() // cols if cols else 0
    if t.dim() == 1:
        return 1, cols, cols
    ld = t.stride(-2)
    # all leading dims must collapse onto a single row stride
    expect = ld
    for d in range(t.dim() - 2, -1, -1):
        if t.shape[d] != 1 and t.stride(d) != expect:
            raise _lib.SvkError(f"svk: {name} leading dims are not uniformly strided")
        expect *= t.shape[d]
    return rows, cols, max(ld, cols)


_PROF = None   # list receiving (kernel_name, flops, bytes, start_event, end_event) when profiling


def set_profiler(records):
    """Record HIP events around every MFMA GEMM / implicit-GEMM conv launch (bench.py roofline);
    ``None`` turns it off.  Events are recorded on the launch stream."""
    global _PROF
    _PROF = records


def _gemm_kernel_name(dt, M, N, vec, asrc):
    """Mirror of launch_gemm's tile choice (csrc/gemm.hip) -> the kernel symbol rocprof reports."""
    if N <= 64:
        bm, bn = (128, 64) if (M + 127) // 128 >= 512 else (64, 64)
    else:
        bm, bn = (128, 128) if ((M + 127) // 128) * ((N + 127) // 128) >= 512 else (64, 64)
    t = "float" if dt == F32 else "__bf16"
    return f"gemm_kernel<{t}, {bm}, {bn}, {'true' if vec else 'false'}, {asrc}>"


def _prof_begin():
    if _PROF is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _prof_end(start, name, flops, nbytes, shape=None):
    if start is None:
        return
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    _PROF.append((name, flops, nbytes, start, e, shape))


def gemm(a, w, bias=None, act=None, residual=None, out=None, n=None):
    """out = act(a @ w[:n].T + bias) + residual; a [..., K], w [N, K] (same dtype as a)."""
    _chk(a, "a"); _chk(w, "w", a.dtype); _chk(bias, "bias", torch.float32); _chk(residual, "residual", a.dtype)
    M, K, lda = _rows(a, "a")
    N = w.shape[0] if n is None else n
    if w.shape[1] != K or w.stride(1) != 1:
        raise _lib.SvkError(f"svk.gemm: weight {tuple(w.shape)} does not match K={K}")
    if out is None:
        out = torch.empty(*a.shape[:-1], N, device=a.device, dtype=a.dtype)
    _chk(out, "out", a.dtype)
    _, _, ldc = _rows(out, "out")
    ldr = 0
    if residual is not None:
        _, rc, ldr = _rows(residual, "residual")
        if rc != N:
            raise _lib.SvkError("svk.gemm: residual width mismatch")
    t0 = _prof_begin()
    _lib.call("svk_gemm", dtype_code(a.dtype), _p(a), lda, _p(w), w.stride(0), _p(bias), _p(residual), ldr,
              _p(out), ldc, M, N, K, ACT[act], _stream())
    if t0 is not None:
        es = a.element_size()
        vw = 16 // es
        vec = a.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0 and lda % vw == 0 and w.stride(0) % vw == 0
        nb = (M * K + N * K + M * N * (2 if residual is not None else 1)) * es
        _prof_end(t0, _gemm_kernel_name(dtype_code(a.dtype), M, N, vec, 0), 2.0 * M * N * K, nb, (M, N, K))
    return out


def conv2d_nhwc(x, w_packed, k, stride, pad, bias=None, act=None, residual=None):
    """x [B, H, W, Cin] NHWC; w_packed [Cout, k*k*Cin] (layout [Cout][kh][kw][Cin]) -> [B, OH, OW, Cout]."""
    _chk(x, "x"); _chk(w_packed, "w", x.dtype); _chk(bias, "bias", torch.float32)
    if not x.is_contiguous() or x.dim() != 4:
        raise _lib.SvkError("svk.conv2d_nhwc: x must be contiguous NHWC [B,H,W,C]")
    B, H, W, Cin = x.shape
    Cout = w_packed.shape[0]
    if w_packed.shape[1] != k * k * Cin or not w_packed.is_contiguous():
        raise _lib.SvkError("svk.conv2d_nhwc: packed weight shape mismatch")
    OH, OW = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    out = torch.empty(B, OH, OW, Cout, device=x.device, dtype=x.dtype)
    if residual is not None:
        _chk(residual, "residual", x.dtype)
        if residual.shape != out.shape or not residual.is_contiguous():
            raise _lib.SvkError("svk.conv2d_nhwc: residual shape mismatch")
    t0 = _prof_begin()
    _lib.call("svk_conv2d_nhwc", dtype_code(x.dtype), _p(x), B, H, W, Cin, _p(w_packed), _p(bias), _p(residual),
              _p(out), Cout, k, stride, pad, ACT[act], _stream())
    if t0 is not None:
        M, K = B * OH * OW, k * k * Cin
        vec = x.data_ptr() % 16 == 0 and w_packed.data_ptr() % 16 == 0 and Cin % 8 == 0
        nb = (x.numel() + Cout * K + M * Cout) * x.element_size()
        _prof_end(t0, _gemm_kernel_name(dtype_code(x.dtype), M, Cout, vec, 1), 2.0 * M * Cout * K, nb,
                  (M, Cout, K, f"conv{k}s{stride}"))
    return out


def layernorm(x, gamma, beta, eps, out=None):
    _chk(x, "x"); _chk(gamma, "gamma", torch.float32); _chk(beta, "beta", torch.float32)
    M, C, ldx = _rows(x, "x")
    if out is None:
        out = torch.empty(*x.shape, device=x.device, dtype=x.dtype)
    _, _, ldy = _rows(out, "out")
    _lib.call("svk_layernorm", dtype_code(x.dtype), _p(x), ldx, _p(out), ldy, _p(gamma), _p(beta), M, C,
              float(eps), _stream())
    return out


def attention(q, k, v, heads, scale, out=None):
    """q [B, Nq, heads*hd], k/v [B, Nk, heads*hd] (any row/batch strides, unit column stride)."""
    for t, nm in ((q, "q"), (k, "k"), (v, "v")):
        _chk(t, nm, q.dtype)
        if t.dim() != 3 or t.stride(2) != 1:
            raise _lib.SvkError(f"svk.attention: {nm} must be [B, N, C] with unit channel stride")
    B, Nq, C = q.shape
    Nk = k.shape[1]
    hd = C // heads
    if out is None:
        out = torch.empty(B, Nq, C, device=q.device, dtype=q.dtype)
    _lib.call("svk_attention", dtype_code(q.dtype), _p(q), q.stride(1), q.stride(0), _p(k), k.stride(1), k.stride(0),
              _p(v), v.stride(1), v.stride(0), _p(out), out.stride(1), out.stride(0), B, Nq, Nk, heads, hd,
              float(scale), _stream())
    return out


MIXFFN_CHANNELS = (32, 64, 128)
FUSED_MIXFFN = os.environ.get("SVK_FUSED_MIXFFN", "0") == "1"


def mixffn_fused(xn, x, w1, b1, taps, dbias, w2, b2):
    """x + fc2(GELU(dwconv3x3(fc1(xn)))) on NHWC [B, H, W, C] bf16 maps (hidden kept on chip)."""
    for t, nm in ((xn, "xn"), (x, "x"), (w1, "w1"), (w2, "w2")):
        _chk(t, nm, torch.bfloat16)
        if not t.is_contiguous():
            raise _lib.SvkError(f"svk.mixffn_fused: {nm} must be contiguous")
    for t, nm in ((b1, "b1"), (taps, "taps"), (dbias, "dbias"), (b2, "b2")):
        _chk(t, nm, torch.float32)
    B, H, W, C = xn.shape
    if x.shape != xn.shape or w1.shape != (4 * C, C) or w2.shape != (C, 4 * C) or taps.shape != (9, 4 * C):
        raise _lib.SvkError("svk.mixffn_fused: shape mismatch")
    out = torch.empty_like(x)
    t0 = _prof_begin()
    _lib.call("svk_mixffn_fused", BF16, _p(xn), _p(x), _p(w1), _p(b1), _p(taps), _p(dbias), _p(w2), _p(b2),
              _p(out), B, H, W, C, _stream())
    if t0 is not None:
        M = B * H * W
        _prof_end(t0, f"mixffn_bf16<{C}>", 2.0 * M * C * 4 * C * 2, (3 * M * C + 8 * C * C) * 2, (M, C, "mixffn"))
    return out


def dwconv3x3(x, taps, bias, act=None):
    """x [B, H, W, C] NHWC contiguous; taps [9, C] f32; bias [C] f32."""
    _chk(x, "x"); _chk(taps, "taps", torch.float32); _chk(bias, "bias", torch.float32)
    B, H, W, C = x.shape
    out = torch.empty_like(x)
    _lib.call("svk_dwconv3x3", dtype_code(x.dtype), _p(x), _p(taps), _p(bias), _p(out), B, H, W, C, ACT[act], _stream())
    return out


def nchw_to_nhwc(x, dtype, cpad=None):
    """[B, C, H, W] f32 -> [B, H, W, cpad] (channels >= C zero) in ``dtype``."""
    _chk(x, "x", torch.float32)
    x = x.contiguous()
    B, C, H, W = x.shape
    cpad = C if cpad is None else cpad
    out = torch.empty(B, H, W, cpad, device=x.device, dtype=dtype)
    _lib.call("svk_nchw_to_nhwc", dtype_code(dtype), _p(x), _p(out), B, C, H, W, cpad, _stream())
    return out


def gauss5x5_reflect(x, dtype, cpad=None):
    _chk(x, "x", torch.float32)
    x = x.contiguous()
    B, C, H, W = x.shape
    cpad = C if cpad is None else cpad
    out = torch.empty(B, H, W, cpad, device=x.device, dtype=dtype)
    _lib.call("svk_gauss5x5_reflect", dtype_code(dtype), _p(x), _p(out), B, C, H, W, cpad, _stream())
    return out


def resize_bilinear(x, H, W, OH, OW, out=None):
    """x [B, H*W, C] tokens (row stride any) -> [B, OH*OW, C] (written into ``out`` if given)."""
    _chk(x, "x")
    B = x.shape[0]
    C = x.shape[-1]
    if out is None:
        out = torch.empty(B, OH * OW, C, device=x.device, dtype=x.dtype)
    _lib.call("svk_resize_bilinear", dtype_code(x.dtype), _p(x), x.stride(-2), _p(out), out.stride(-2), B, H, W, C,
              OH, OW, _stream())
    return out


def mean_rows(x, R):
    """x [B*R, C] -> [B, C] f32 mean over each group of R consecutive rows."""
    _chk(x, "x")
    M, C, ldx = _rows(x, "x")
    B = M // R
    out = torch.empty(B, C, device=x.device, dtype=torch.float32)
    _lib.call("svk_mean_rows", dtype_code(x.dtype), _p(x), ldx, _p(out), B, R, C, _stream())
    return out


def softmax_rows(x, out=None):
    _chk(x, "x", torch.float32)
    M, C, ldx = _rows(x, "x")
    if out is None:
        out = torch.empty_like(x)
    _, _, ldy = _rows(out, "out")
    _lib.call("svk_softmax_rows", _p(x), ldx, _p(out), ldy, M, C, _stream())
    return out


def mstcn_layer(x, wd_packed, bd, w1, b1, dilation, causal, out=None):
    """x [T, F] f32 time-major; wd_packed [3, F, F]; w1 [F, F]."""
    for t, nm in ((x, "x"), (wd_packed, "wd"), (bd, "bd"), (w1, "w1"), (b1, "b1")):
        _chk(t, nm, torch.float32)
    T, F = x.shape
    if out is None:
        out = torch.empty_like(x)
    _lib.call("svk_mstcn_layer", _p(x), _p(wd_packed), _p(bd), _p(w1), _p(b1), _p(out), T, F, dilation,
              1 if causal else 0, _stream())
    return out


def window_unfold(x, length, pos=None):
    """x [T, C] -> [T, length, C] causal windows (zero left-pad) + pos[length, C]."""
    _chk(x, "x"); _chk(pos, "pos", torch.float32)
    T, C, ldx = _rows(x, "x")
    out = torch.empty(T, length, C, device=x.device, dtype=x.dtype)
    _lib.call("svk_window_unfold", dtype_code(x.dtype), _p(x), ldx, _p(pos), _p(out), T, C, length, _stream())
    return out


def cast(x, dtype):
    _chk(x, "x")
    x = x.contiguous()
    out = torch.empty(x.shape, device=x.device, dtype=dtype)
    _lib.call("svk_cast", dtype_code(x.dtype), _p(x), dtype_code(dtype), _p(out), x.numel(), _stream())
    return out


def add_bcast(x, table):
    """x [..., C] contiguous + table[r % period] for the rows r of x (table [period, C] f32)."""
    _chk(x, "x"); _chk(table, "table", torch.float32)
    x = x.contiguous()
    C = x.shape[-1]
    out = torch.empty_like(x)
    _lib.call("svk_add_bcast", dtype_code(x.dtype), _p(x), _p(table), _p(out), x.numel() // C, C, table.shape[0],
              _stream())
    return out
