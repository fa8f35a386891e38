"""Torch-facing wrappers over the svk C ABI.

Every op takes CUDA (HIP) tensors, checks layout/dtype on the host, allocates its
output through the PyTorch caching allocator (the library never allocates) and
launches on the current stream.  There is deliberately no CPU path: a CPU tensor
is an error.
"""
import collections
import ctypes
import os

import torch

from . import _lib

F32, BF16, F16 = 0, 1, 2
ACT = {None: 0, "none": 0, "gelu": 1, "relu": 2, "tanh": 3}
_DT = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16}
H16 = (torch.bfloat16, torch.float16)     # the 16-bit MFMA storage types


def dtype_code(dt):
    try:
        return _DT[dt]
    except KeyError:
        raise _lib.SvkError(f"svk: unsupported dtype {dt} (float32 / float16 / bfloat16 only)") from None


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


def tune(knob, value):
    """Set a kernel-selection knob (svk_tune: "pk_cfg", "pk_elds", "dw_lds", "dw_rows", "attn_cfg"; -1 = auto).
    Every value selects a complete, parity-tested variant: the product library has no work-skipping switch."""
    _lib.call("svk_tune", knob.encode(), int(value))


def _last_kernel():
    """The kernel instantiation the library launched last on this thread (svk_last_kernel)."""
    return _lib.load().svk_last_kernel().decode()


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


def gemm(a, w, bias=None, act=None, residual=None, out=None, n=None, row_scale=None, rows_per=1, dact=None,
         dact_src=None):
    """out = row_scale[m // rows_per] * act(a @ w[:n].T + bias) * dact'(dact_src) + residual; a [..., K],
    w [N, K] (same dtype as a); row_scale (f32, stochastic depth) and the activation-backward factor
    (dact in {"gelu", "relu", "tanh"} evaluated at dact_src [M, N]) are optional."""
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
    if (SKINNY and row_scale is None and a.dtype in H16 and N <= 64 and K <= 128 and M >= 2048
            and a.data_ptr() % 16 == 0 and (K % 8 or lda % 8 == 0)):
        return gemm_skinny(a, w, bias, act, residual, out, N, dact, dact_src)
    t0 = _prof_begin()
    if row_scale is None and dact is None:
        _lib.call("svk_gemm", dtype_code(a.dtype), _p(a), lda, _p(w), w.stride(0), _p(bias), _p(residual), ldr,
                  _p(out), ldc, M, N, K, ACT[act], _stream())
    else:
        _chk(row_scale, "row_scale", torch.float32)
        if row_scale is not None and row_scale.numel() * rows_per < M:
            raise _lib.SvkError("svk.gemm: row_scale too short")
        ldu = 0
        if dact is not None:
            _chk(dact_src, "dact_src", a.dtype)
            mu, nu, ldu = _rows(dact_src, "dact_src")
            if mu != M or nu != N:
                raise _lib.SvkError("svk.gemm: dact_src shape mismatch")
        _lib.call("svk_gemm_ex", dtype_code(a.dtype), _p(a), lda, _p(w), w.stride(0), _p(bias), _p(row_scale),
                  rows_per, _p(dact_src), ldu, ACT[dact], _p(residual), ldr, _p(out), ldc, M, N, K, ACT[act],
                  _stream())
    if t0 is not None:
        es = a.element_size()
        vw = 16 // es
        vec = a.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0 and lda % vw == 0 and w.stride(0) % vw == 0
        nb = (M * K + N * K + M * N * (1 + (residual is not None) + (dact is not None))) * es
        _prof_end(t0, _last_kernel(),
                  2.0 * M * N * K, nb, (M, N, K))
    return out


SKINNY = os.environ.get("SVK_SKINNY", "1") == "1"

def gemm_skinny(a, w, bias=None, act=None, residual=None, out=None, n=None, dact=None, dact_src=None):
    """svk_gemm_skinny (bf16 / f16, N <= 64, K <= 128): same contract as gemm() without row_scale."""
    _chk(a, "a")
    if a.dtype not in H16:
        raise _lib.SvkError("svk.gemm_skinny: bf16 / f16 only")
    _chk(w, "w", a.dtype); _chk(bias, "bias", torch.float32)
    _chk(residual, "residual", a.dtype); _chk(dact_src, "dact_src", a.dtype)
    M, K, lda = _rows(a, "a")
    N = w.shape[0] if n is None else n
    if w.shape[1] != K or w.stride(1) != 1:
        raise _lib.SvkError("svk.gemm_skinny: weight shape mismatch")
    if out is None:
        out = torch.empty(*a.shape[:-1], N, device=a.device, dtype=a.dtype)
    _, _, ldc = _rows(out, "out")
    ldr = _rows(residual, "residual")[2] if residual is not None else 0
    ldu = _rows(dact_src, "dact_src")[2] if dact_src is not None else 0
    t0 = _prof_begin()
    _lib.call("svk_gemm_skinny", dtype_code(a.dtype), _p(a), lda, _p(w), w.stride(0), _p(bias), _p(dact_src), ldu, ACT[dact],
              _p(residual), ldr, _p(out), ldc, M, N, K, ACT[act], _stream())
    _prof_end(t0, "skinny_gemm", 2.0 * M * N * K,
              (M * K + N * K + M * N * (1 + (residual is not None) + (dact is not None))) * 2, (M, N, K, "skinny"))
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
        _prof_end(t0, _last_kernel(), 2.0 * M * Cout * K, nb,
                  (M, Cout, K, f"conv{k}s{stride}"))
    return out


def conv2d_ln_nhwc(x, w_packed, k, stride, pad, bias, gamma, beta, eps):
    """LN(conv(x) + bias) over the output channels (Attention.sr + Attention.norm); long-K bf16
    patchify convs run split-K with an f32 workspace reduced inside the LayerNorm."""
    _chk(x, "x"); _chk(w_packed, "w", x.dtype)
    for t, nm in ((bias, "bias"), (gamma, "gamma"), (beta, "beta")):
        _chk(t, nm, torch.float32)
    if not x.is_contiguous() or x.dim() != 4:
        raise _lib.SvkError("svk.conv2d_ln_nhwc: x must be contiguous NHWC [B,H,W,C]")
    B, H, W, Cin = x.shape
    Cout = w_packed.shape[0]
    if w_packed.shape[1] != k * k * Cin or not w_packed.is_contiguous():
        raise _lib.SvkError("svk.conv2d_ln_nhwc: packed weight shape mismatch")
    OH, OW = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    out = torch.empty(B, OH, OW, Cout, device=x.device, dtype=x.dtype)
    lib = _lib.load()
    nbytes = lib.svk_conv2d_ln_workspace(dtype_code(x.dtype), B, H, W, Cin, Cout, k, stride, pad)
    ws = torch.empty((nbytes + 15) // 16 * 4, device=x.device, dtype=torch.float32) if nbytes > 0 else None
    t0 = _prof_begin()
    _lib.call("svk_conv2d_ln_nhwc", dtype_code(x.dtype), _p(x), B, H, W, Cin, _p(w_packed), _p(bias), _p(gamma),
              _p(beta), float(eps), _p(out), Cout, k, stride, pad, _p(ws), 0 if ws is None else ws.numel() * 4,
              _stream())
    if t0 is not None:
        M, K = B * OH * OW, k * k * Cin
        _prof_end(t0, _last_kernel(), 2.0 * M * Cout * K, (x.numel() + Cout * K + M * Cout) * x.element_size(),
                  (M, Cout, K, f"convln{k}s{stride}"))
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


# off by default: it does not beat the unfused pair yet (second form, A LDS-DMA ring + staged row stores: stage-3
# proj + norm2 52 us vs 35 + 15, shared MLP + norm1 47 vs 24 + 16; step 34.8k vs 35.7k same-box,
# profiles/r05/gemm_ln_v2.txt) — it is one tile per workgroup, where gemm_pk is persistent and overlaps a tile's
# epilogue with the next tile's loads; turning it on cuts the replayed step from 192 to 174 launches
# (profiles/r05/gemm_ln_mx28_ab.txt)
# "auto" (default): only where the fused kernel measured faster than GEMM + LayerNorm — the stage-4 prompt
# shared MLP + norm1 (N = 512, K = 128: 21.6 vs 24.8 us; the N = 320 and K = 512 shapes lose,
# profiles/r05/gemm_ln_v2.txt); "1": every instantiated shape; "0": off
GEMM_LN = os.environ.get("SVK_GEMM_LN", "auto")


def _gemm_ln_on(N, K):
    if GEMM_LN is True or GEMM_LN == "1":
        return True
    return GEMM_LN == "auto" and N == 512 and K <= 128


def gemm_ln_pack(w):
    """Packed weight fragments for gemm_ln (svk_gemm_ln_pack), or None where (dtype, N, K) has no gemm_ln
    instantiation (N in {320, 512}, 16-bit, K % 8 == 0).  Pack once per weight set."""
    if w.dtype not in H16 or not w.is_cuda or not _gemm_ln_on(*w.shape):
        return None
    N, K = w.shape
    nbytes = _lib.load().svk_gemm_ln_packed_bytes(dtype_code(w.dtype), int(N), int(K))
    if nbytes <= 0:
        return None
    _chk(w, "w")
    if not w.is_contiguous():
        raise _lib.SvkError("svk.gemm_ln_pack: w must be contiguous [N, K]")
    out = torch.empty(nbytes, device=w.device, dtype=torch.uint8)
    _lib.call("svk_gemm_ln_pack", dtype_code(w.dtype), _p(w), int(N), int(K), _p(out), _stream())
    return out


def gemm_ln(a, packed, n, bias, residual, gamma, beta, eps):
    """(x, h): x = a @ w.T + bias (+ residual), h = LayerNorm(x) over the full row (svk_gemm_ln: one kernel,
    the row statistics inside the workgroup); w from gemm_ln_pack.  a [..., K] 16-bit, n = N."""
    _chk(a, "a"); _chk(bias, "bias", torch.float32); _chk(residual, "residual", a.dtype)
    _chk(gamma, "gamma", torch.float32); _chk(beta, "beta", torch.float32)
    M, K, lda = _rows(a, "a")
    if lda != K:
        raise _lib.SvkError("svk.gemm_ln: a must be row-contiguous")
    shape = tuple(a.shape[:-1]) + (n,)
    if residual is not None and (tuple(residual.shape) != shape or not residual.is_contiguous()):
        raise _lib.SvkError("svk.gemm_ln: residual must be a contiguous [..., N] map")
    x = torch.empty(shape, device=a.device, dtype=a.dtype)
    h = torch.empty(shape, device=a.device, dtype=a.dtype)
    t0 = _prof_begin()
    _lib.call("svk_gemm_ln", dtype_code(a.dtype), _p(a), M, K, _p(packed), _p(bias), _p(residual), _p(gamma), _p(beta),
              float(eps), _p(x), _p(h), int(n), _stream())
    if t0 is not None:
        _prof_end(t0, _last_kernel(), 2.0 * M * n * K, (M * K + n * K + M * n * (3 if residual is not None else 2)) * 2,
                  (M, n, K, "gemm_ln"))
    return x, h


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


FUSED_MIXFFN = os.environ.get("SVK_FUSED_MIXFFN", "1") == "1"


def mixffn_supported(W, C):
    """True when svk_mixffn_fused has an instantiation for map width W and channels C."""
    return bool(_lib.load().svk_mixffn_supported(int(W), int(C)))


FUSED_ATTN_BLOCK = os.environ.get("SVK_FUSED_ATTN_BLOCK", "1") == "1"
# stage 4 (no sequence reduction): q and kv as one GEMM over the stacked weights
MERGED_QKV = os.environ.get("SVK_MERGED_QKV", "1") == "1"
FUSED_PROMPT_LN = os.environ.get("SVK_FUSED_PROMPT_LN", "1") == "1"
# C = 320 (stage 3) is available but off: at 256 VGPRs and 130 KB of LDS it runs one wave per SIMD and
# cost 11 % of the whole step in a same-box A/B
PROMPT_LN_C = tuple(int(c) for c in os.environ.get("SVK_PROMPT_LN_C", "64,128").split(",") if c)


def attn_block(hn, x, kv, wq, bq, wp, bp, gamma2, beta2, eps, scale):
    """Attention half of a MiT Block with 64-channel heads (C = 64 / 1 head, C = 128 / 2 heads; <= 64
    reduced keys) in one kernel: returns (y, h2) with y = x + proj(attn(q(hn), k, v)) and h2 = LayerNorm(y)
    (svk_attn_block).  hn, x [B, N, C] contiguous; kv [B, Nk, 2C] (k | v)."""
    if hn.dtype not in H16:
        raise _lib.SvkError("svk.attn_block: bf16 / f16 only")
    for t, nm in ((hn, "hn"), (x, "x"), (kv, "kv"), (wq, "wq"), (wp, "wp")):
        _chk(t, nm, hn.dtype)
    for t, nm in ((bq, "bq"), (bp, "bp"), (gamma2, "gamma2"), (beta2, "beta2")):
        _chk(t, nm, torch.float32)
    B, N, C = hn.shape
    Bk, Nk, C2 = kv.shape
    if (x.shape != hn.shape or Bk != B or C2 != 2 * C or not (hn.is_contiguous() and x.is_contiguous()
                                                               and kv.is_contiguous())):
        raise _lib.SvkError("svk.attn_block: shape / layout mismatch")
    y = torch.empty_like(x)
    h2 = torch.empty_like(x)
    t0 = _prof_begin()
    _lib.call("svk_attn_block", dtype_code(hn.dtype), _p(hn), _p(x), _p(kv), 2 * C, _p(wq), _p(bq), _p(wp), _p(bp),
              _p(gamma2), _p(beta2), float(eps), _p(y), _p(h2), B, N, Nk, C, float(scale), _stream())
    if t0 is not None:
        M = B * N
        _prof_end(t0, f"attn_block<{C}>", 2.0 * M * C * C * 2 + 4.0 * M * 64 * C, 4 * M * C * 2, (M, C, "attn_block"))
    return y, h2


def prompt_ln(x, summed, wl, bl, ws, bs, gamma1, beta1, eps):
    """(x + shared(GELU(light(summed))), norm1 of that) in one kernel (svk_prompt_ln; C in {64, 128, 320}):
    x [B, N, C], summed [B, N, C // 4] contiguous bf16 / f16 -> (x', h)."""
    if x.dtype not in H16:
        raise _lib.SvkError("svk.prompt_ln: bf16 / f16 only")
    for t, nm in ((x, "x"), (summed, "summed"), (wl, "wl"), (ws, "ws")):
        _chk(t, nm, x.dtype)
    for t, nm in ((bl, "bl"), (bs, "bs"), (gamma1, "gamma1"), (beta1, "beta1")):
        _chk(t, nm, torch.float32)
    C = x.shape[-1]
    M = x.numel() // C
    if (summed.numel() != M * (C // 4) or wl.shape != (C // 4, C // 4) or ws.shape != (C, C // 4)
            or not (x.is_contiguous() and summed.is_contiguous() and wl.is_contiguous() and ws.is_contiguous())):
        raise _lib.SvkError("svk.prompt_ln: shape / layout mismatch")
    xo = torch.empty_like(x)
    h = torch.empty_like(x)
    t0 = _prof_begin()
    _lib.call("svk_prompt_ln", dtype_code(x.dtype), _p(summed), _p(x), _p(wl), _p(bl), _p(ws), _p(bs), _p(gamma1),
              _p(beta1), float(eps), _p(xo), _p(h), M, C, _stream())
    if t0 is not None:
        _prof_end(t0, f"prompt_ln<{C}>", 2.0 * M * (C // 4) * (C // 4 + C), (3 * M * C + M * C // 4) * 2,
                  (M, C, "prompt_ln"))
    return xo, h


def mixffn_pack_taps(taps, dbias, dtype):
    """Depthwise taps [9, hid] f32 (row dy*3+dx) + bias [hid] f32 -> the packed form svk_mixffn_fused
    reads (include/svk.h): per channel quad q (channels 4q..4q+3) 13 16-byte records — 12 for
    (dy, c) = the dtype pairs (w1,w2), (w0,w1), (0,w0), (w2,0) of tap row dy of channel 4q + c — then the
    4 biases as f32; int32 [hid / 4 * 52]."""
    hid = taps.shape[1]
    w = taps.t().reshape(hid, 3, 3).to(dtype)                        # [ch][dy][dx]
    z = torch.zeros_like(w[..., 0])
    pairs = torch.stack([torch.stack([w[..., 1], w[..., 2]], -1), torch.stack([w[..., 0], w[..., 1]], -1),
                         torch.stack([z, w[..., 0]], -1), torch.stack([w[..., 2], z], -1)], 2)   # [ch, dy, 4, 2]
    rec = pairs.contiguous().view(torch.int32).reshape(hid // 4, 4, 3, 4)     # [q][c][dy][word]
    rec = rec.permute(0, 2, 1, 3).reshape(hid // 4, 48)                       # [q][dy][c][word]
    bias = dbias.float().contiguous().view(torch.int32).reshape(hid // 4, 4)
    return torch.cat([rec, bias], 1).contiguous().reshape(-1)


def mixffn_fused(xn, x, w1, b1, tpk, w2, b2, ln=None):
    """x + fc2(GELU(dwconv3x3(fc1(xn)))) on NHWC [B, H, W, C] bf16 / f16 maps, the 4C hidden kept on
    chip (svk_mixffn_fused); ``tpk`` from mixffn_pack_taps.  ``ln = (gamma, beta, eps)`` returns the
    LayerNorm of that sum instead (the stage norm fused into the epilogue; the sum is then not written)."""
    if xn.dtype not in H16:
        raise _lib.SvkError("svk.mixffn_fused: bf16 / f16 only")
    for t, nm in ((xn, "xn"), (x, "x"), (w1, "w1"), (w2, "w2")):
        _chk(t, nm, xn.dtype)
        if not t.is_contiguous():
            raise _lib.SvkError(f"svk.mixffn_fused: {nm} must be contiguous")
    for t, nm in ((b1, "b1"), (b2, "b2")):
        _chk(t, nm, torch.float32)
    _chk(tpk, "tpk", torch.int32)
    B, H, W, C = xn.shape
    if (x.shape != xn.shape or w1.shape != (4 * C, C) or w2.shape != (C, 4 * C) or tpk.shape != (52 * C,)
            or not tpk.is_contiguous()):
        raise _lib.SvkError("svk.mixffn_fused: shape mismatch")
    out = torch.empty_like(x)
    g = bt = None
    eps = 0.0
    if ln is not None:
        g, bt, eps = ln
        _chk(g, "gamma", torch.float32); _chk(bt, "beta", torch.float32)
    t0 = _prof_begin()
    _lib.call("svk_mixffn_fused", dtype_code(xn.dtype), _p(xn), _p(x), _p(w1), _p(b1), _p(tpk), _p(w2), _p(b2),
              None if ln is not None else _p(out), _p(out) if ln is not None else None, _p(g), _p(bt), float(eps),
              B, H, W, C, _stream())
    if t0 is not None:
        M = B * H * W
        _prof_end(t0, f"mixffn<{C}>", 2.0 * M * C * 4 * C * 2 + 2.0 * 9 * M * 4 * C,
                  (3 * M * C + 8 * C * C) * 2, (M, C, "mixffn"))
    return out


MIXFFN_RW = os.environ.get("SVK_MIXFFN_RW", "1") == "1"
# off by default: bit-identical to dwconv3x3 + gemm but measured no faster (stage 3 188.8 vs 186.8 us, stage 4
# 137.8 vs 99.6 us at B = 256, profiles/r04/dwfc2_bench.log): the per-tap LDS reads and masks of the G
# production are latency-bound at 2 waves per SIMD
DW_FC2 = os.environ.get("SVK_DW_FC2", "0") == "1"
DWFC2_MX = os.environ.get("SVK_DWFC2_MX", "1") == "1"
# map widths whose MixFFN back half the model runs in the matrix-core form (14: stage 3, 7: stage 4).  28 (stage 2)
# is instantiated but off: its fc1 then needs a GEMM of its own, and fc1 GEMM + dw_fc2_mx (196 us) loses to the
# register-window fc1dw_rw (fc1 + dwconv, 135 us) + fc2 GEMM (68 us): step 32.6k vs 34.2k frames/s same-box
# (profiles/r05/gemm_ln_mx28_ab.txt)
DWFC2_MX_WIDTHS = tuple(int(v) for v in os.environ.get("SVK_DWFC2_MX_WIDTHS", "14,7").split(",") if v)


def mixffn_dw_fc2_supported(dtype, W, N, K):
    """True when svk_mixffn_dw_fc2 (dwconv3x3 + GELU fused into fc2) has an instantiation for the map."""
    return dtype in H16 and bool(_lib.load().svk_mixffn_dw_fc2_supported(dtype_code(dtype), int(W), int(N), int(K)))


def mixffn_dw_fc2_pack(taps, dbias, w2, W):
    """The packed operand buffer of the matrix-core stage-3 form (svk_mixffn_dw_fc2_pack), or None where the
    map has no packed form.  Pack once per weight set (Mlp._pack does) and pass it to mixffn_dw_fc2."""
    N, K = w2.shape
    nbytes = _lib.load().svk_mixffn_dw_fc2_packed_bytes(dtype_code(w2.dtype), int(W), int(N), int(K))
    if nbytes <= 0:
        return None
    for t, nm in ((taps, "taps"), (dbias, "dbias")):
        _chk(t, nm, torch.float32)
    _chk(w2, "w2")
    if taps.shape != (9, K) or dbias.numel() != K or not (taps.is_contiguous() and w2.is_contiguous()):
        raise _lib.SvkError("svk.mixffn_dw_fc2_pack: taps [9, K] / dbias [K] / w2 [N, K] contiguous")
    out = torch.empty(nbytes, device=w2.device, dtype=torch.uint8)
    _lib.call("svk_mixffn_dw_fc2_pack", dtype_code(w2.dtype), _p(taps), _p(dbias), _p(w2), int(W), int(N), int(K),
              _p(out), _stream())
    return out


def mixffn_dw_fc2(h, taps, dbias, w2, b2, residual=None, packed=None, act="gelu", pre_out=None, row_scale=None,
                  rows_per=1):
    """fc2(GELU(dwconv3x3(h) + dbias)) + b2 (+ residual) with the GELU map kept on chip (svk_mixffn_dw_fc2):
    h [B, H, W, K] fc1 output (16-bit NHWC), taps [9, K] / dbias [K] f32 as DWConv packs them, w2 [N, K];
    returns [B, H * W, N].  Where the map has the matrix-core form (14 x 14 with N = 320, 7 x 7 with N = 512,
    28 x 28 with N = 128) it runs that,
    from ``packed`` (mixffn_dw_fc2_pack) or packing on the fly; ``SVK_DWFC2_MX=0`` keeps the LDS-tap form.
    When ``packed`` is given, the kernel reads the taps, dbias and W2 baked into it (``taps`` / ``dbias`` / ``w2``
    are then only shape-checked); its size is checked against svk_mixffn_dw_fc2_packed_bytes(dtype, W, N, K).
    Training forward (matrix-core form, GELU, 14 x 14 / 7 x 7): ``pre_out`` [B, H, W, K] receives the
    pre-activation dwconv3x3(h) + dbias (the GELU backward's source, as dwconv3x3(pre_out=) writes it), and
    ``row_scale`` [B * H * W / rows_per] f32 scales each token's fc2 output before the residual (DropPath).
    ``act="none"`` drops the GELU (matrix-core form only, 14 x 14 / 7 x 7): with flipped taps, zero dbias and
    w2 = W1ᵀ it is the data gradient through a frozen DWConv + fc1 (svk/train.py)."""
    if act not in ("gelu", "none"):
        raise _lib.SvkError("svk.mixffn_dw_fc2: act must be 'gelu' or 'none'")
    if h.dtype not in H16:
        raise _lib.SvkError("svk.mixffn_dw_fc2: bf16 / f16 only")
    _chk(h, "h"); _chk(w2, "w2", h.dtype); _chk(residual, "residual", h.dtype)
    for t, nm in ((taps, "taps"), (dbias, "dbias"), (b2, "b2")):
        _chk(t, nm, torch.float32)
    B, H, W, K = h.shape
    N = w2.shape[0]
    for t, nm in ((h, "h"), (w2, "w2"), (taps, "taps"), (dbias, "dbias"), (b2, "b2")):
        if not t.is_contiguous():
            raise _lib.SvkError(f"svk.mixffn_dw_fc2: {nm} must be contiguous")
    if w2.shape != (N, K) or taps.shape != (9, K) or dbias.numel() != K or b2.numel() != N:
        raise _lib.SvkError("svk.mixffn_dw_fc2: shape mismatch")
    if residual is not None and (residual.numel() != B * H * W * N or not residual.is_contiguous()):
        raise _lib.SvkError("svk.mixffn_dw_fc2: residual must be a contiguous [B, H*W, N] map")
    out = torch.empty(B, H * W, N, device=h.device, dtype=h.dtype)
    if (DWFC2_MX or act == "none") and packed is None:
        packed = mixffn_dw_fc2_pack(taps, dbias, w2, W)
    if act == "none" and packed is None:
        raise _lib.SvkError(f"svk.mixffn_dw_fc2: no identity-activation form for {W} x {W}, N = {N}")
    if packed is not None:
        # the packed buffer carries the taps, dbias and W2 (the arguments above are then unused by the kernel):
        # it must have been built for this (dtype, W, N, K), or the kernel would read past it
        want = int(_lib.load().svk_mixffn_dw_fc2_packed_bytes(dtype_code(h.dtype), int(W), int(N), int(K)))
        if (want == 0 or not packed.is_cuda or not packed.is_contiguous()
                or packed.numel() * packed.element_size() != want or packed.data_ptr() % 16):
            raise _lib.SvkError(f"svk.mixffn_dw_fc2: packed buffer is not the ({h.dtype}, W={W}, N={N}, K={K}) pack "
                                f"({packed.numel() * packed.element_size()} bytes, expected {want})")
    if pre_out is not None or row_scale is not None:
        if act != "gelu" or packed is None:
            raise _lib.SvkError("svk.mixffn_dw_fc2: pre_out / row_scale need the matrix-core GELU form")
        if pre_out is not None and (pre_out.dtype != h.dtype or pre_out.shape != h.shape or not pre_out.is_contiguous()):
            raise _lib.SvkError("svk.mixffn_dw_fc2: pre_out must be a contiguous map like h")
        if row_scale is not None and (row_scale.dtype != torch.float32 or not row_scale.is_contiguous()
                                      or row_scale.numel() * rows_per != B * H * W):
            raise _lib.SvkError("svk.mixffn_dw_fc2: row_scale must be f32 [tokens / rows_per]")
        t0 = _prof_begin()
        _lib.call("svk_mixffn_dw_fc2_packed_ex", dtype_code(h.dtype), _p(h), _p(packed), _p(b2), _p(residual),
                  _p(out), B, H, W, K, N, ACT["gelu"], _p(pre_out), _p(row_scale), int(rows_per), _stream())
        if t0 is not None:
            M = B * H * W
            _prof_end(t0, _last_kernel(), 2.0 * M * N * K + 2.0 * 9 * M * K,
                      (M * K * (2 if pre_out is not None else 1) + N * K + M * N * (2 if residual is not None else 1))
                      * h.element_size(), (M, N, K, "dw_fc2"))
        return out
    t0 = _prof_begin()
    if act == "none":
        _lib.call("svk_mixffn_dw_fc2_packed_act", dtype_code(h.dtype), _p(h), _p(packed), _p(b2), _p(residual),
                  _p(out), B, H, W, K, N, 0, _stream())
    elif DWFC2_MX and packed is not None:
        _lib.call("svk_mixffn_dw_fc2_packed", dtype_code(h.dtype), _p(h), _p(packed), _p(b2), _p(residual), _p(out),
                  B, H, W, K, N, _stream())
    else:
        _lib.call("svk_mixffn_dw_fc2", dtype_code(h.dtype), _p(h), _p(taps), _p(dbias), _p(w2), _p(b2), _p(residual),
                  _p(out), B, H, W, K, N, _stream())
    if t0 is not None:
        M = B * H * W
        _prof_end(t0, _last_kernel(), 2.0 * M * N * K + 2.0 * 9 * M * K,
                  (M * K + N * K + M * N * (2 if residual is not None else 1)) * h.element_size(), (M, N, K, "dw_fc2"))
    return out


def mixffn_rw_supported(dtype, W, C):
    """True when svk_mixffn_rw (the register-window whole MixFFN) has an instantiation for the map dtype,
    width W and channels C."""
    return dtype in H16 and bool(_lib.load().svk_mixffn_rw_supported(dtype_code(dtype), int(W), int(C)))


def mixffn_rw(xn, x, w1, b1, taps, dbias, w2, b2, ln=None):
    """x + fc2(GELU(dwconv3x3(fc1(xn)))) on NHWC [B, H, W, C] f16 maps with the depthwise window held in
    registers (svk_mixffn_rw); taps [9, 4C] / dbias [4C] f32 as DWConv packs them.  ``ln = (gamma, beta,
    eps)`` returns the LayerNorm of that sum instead (the sum is then not written)."""
    if xn.dtype not in H16:
        raise _lib.SvkError("svk.mixffn_rw: f16 only")
    for t, nm in ((xn, "xn"), (x, "x"), (w1, "w1"), (w2, "w2")):
        _chk(t, nm, xn.dtype)
        if not t.is_contiguous():
            raise _lib.SvkError(f"svk.mixffn_rw: {nm} must be contiguous")
    for t, nm in ((b1, "b1"), (b2, "b2"), (taps, "taps"), (dbias, "dbias")):
        _chk(t, nm, torch.float32)
        if not t.is_contiguous():
            raise _lib.SvkError(f"svk.mixffn_rw: {nm} must be contiguous")
    B, H, W, C = xn.shape
    if (x.shape != xn.shape or w1.shape != (4 * C, C) or w2.shape != (C, 4 * C) or taps.shape != (9, 4 * C)
            or b1.numel() != 4 * C or dbias.numel() != 4 * C or b2.numel() != C):
        raise _lib.SvkError("svk.mixffn_rw: shape mismatch")
    out = torch.empty_like(x)
    g = bt = None
    eps = 0.0
    if ln is not None:
        g, bt, eps = ln
        _chk(g, "gamma", torch.float32); _chk(bt, "beta", torch.float32)
    t0 = _prof_begin()
    _lib.call("svk_mixffn_rw", dtype_code(xn.dtype), _p(xn), _p(x), _p(w1), _p(b1), _p(taps), _p(dbias), _p(w2),
              _p(b2), None if ln is not None else _p(out), _p(out) if ln is not None else None, _p(g), _p(bt),
              float(eps), B, H, W, C, _stream())
    if t0 is not None:
        M = B * H * W
        _prof_end(t0, f"mixffn_rw<{C}>", 2.0 * M * C * 4 * C * 2 + 2.0 * 9 * M * 4 * C,
                  (3 * M * C + 8 * C * C) * 2, (M, C, "mixffn_rw"))
    return out


FC1_DWCONV = os.environ.get("SVK_FC1_DWCONV", "1") == "1"
# channel widths routed to it in inference (A/B knob; 320 / 512 are stages 3-4 of MiT-b1..b5)
FC1_DWCONV_C = tuple(int(c) for c in os.environ.get("SVK_FC1_DWCONV_C", "32,64,128").split(","))


def mixffn_fc1_dwconv(xn, w1, b1, taps, dbias, act="gelu", pre_out=None):
    """act(dwconv3x3(xn @ w1.T + b1) + dbias) on an NHWC [B, H, W, C] bf16 / f16 map -> [B, H, W, hidden];
    the hidden map never leaves the chip (svk_mixffn_fc1_dwconv_ex).  ``pre_out`` ([B, H, W, hidden], same
    dtype) also receives the pre-activation, as ``dwconv3x3(..., pre_out=)`` writes it."""
    _chk(xn, "xn"); _chk(w1, "w1", xn.dtype)
    if xn.dtype not in H16:
        raise _lib.SvkError("svk.mixffn_fc1_dwconv: bf16 / f16 only")
    for t, nm in ((b1, "b1"), (taps, "taps"), (dbias, "dbias")):
        _chk(t, nm, torch.float32)
    if not xn.is_contiguous() or xn.dim() != 4 or not w1.is_contiguous():
        raise _lib.SvkError("svk.mixffn_fc1_dwconv: xn must be contiguous NHWC, w1 contiguous")
    B, H, W, C = xn.shape
    hid = w1.shape[0]
    if w1.shape[1] != C or taps.shape != (9, hid) or b1.numel() != hid or dbias.numel() != hid:
        raise _lib.SvkError("svk.mixffn_fc1_dwconv: shape mismatch")
    out = torch.empty(B, H, W, hid, device=xn.device, dtype=xn.dtype)
    if pre_out is not None:
        _chk(pre_out, "pre_out", xn.dtype)
        if pre_out.shape != out.shape or not pre_out.is_contiguous():
            raise _lib.SvkError("svk.mixffn_fc1_dwconv: pre_out must be a contiguous [B, H, W, hidden] map")
    t0 = _prof_begin()
    _lib.call("svk_mixffn_fc1_dwconv_ex", dtype_code(xn.dtype), _p(xn), _p(w1), _p(b1), _p(taps), _p(dbias), _p(out),
              _p(pre_out), B, H, W, C, hid, ACT[act], _stream())
    if t0 is not None:
        M = B * H * W
        _prof_end(t0, "fc1_dwconv", 2.0 * M * C * hid,
                  (xn.numel() + out.numel() * (1 if pre_out is None else 2) + w1.numel()) * 2, (M, hid, C, "fc1dw"))
    return out


def dwconv3x3(x, taps, bias, act=None, pre_out=None):
    """x [B, H, W, C] NHWC contiguous; taps [9, C] f32; bias [C] f32.  ``pre_out`` (same shape)
    additionally receives the pre-activation map."""
    _chk(x, "x"); _chk(taps, "taps", torch.float32); _chk(bias, "bias", torch.float32); _chk(pre_out, "pre_out", x.dtype)
    B, H, W, C = x.shape
    out = torch.empty_like(x)
    if pre_out is None:
        _lib.call("svk_dwconv3x3", dtype_code(x.dtype), _p(x), _p(taps), _p(bias), _p(out), B, H, W, C, ACT[act],
                  _stream())
    else:
        if pre_out.shape != x.shape or not pre_out.is_contiguous():
            raise _lib.SvkError("svk.dwconv3x3: pre_out shape mismatch")
        _lib.call("svk_dwconv3x3_ex", dtype_code(x.dtype), _p(x), _p(taps), _p(bias), _p(out), _p(pre_out), B, H, W, C,
                  ACT[act], _stream())
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


# stem convs (k = 7, stride 4, 2/3 input channels) over space-to-depth blocks (A/B switch)
STEM_S2D = os.environ.get("SVK_STEM_S2D", "1") == "1"


def stem_s2d_ok(dtype, cin, k, stride):
    return STEM_S2D and dtype in H16 and cin in (2, 3) and stride == 4 and k <= 2 * stride


def nchw_to_s2d(x, dtype, s, pad, nbh, nbw):
    """[B, C, H, W] f32 -> space-to-depth blocks [B, nbh, nbw, s*s*C] in ``dtype`` (svk_nchw_to_s2d)."""
    _chk(x, "x", torch.float32)
    x = x.contiguous()
    B, C, H, W = x.shape
    out = torch.empty(B, nbh, nbw, s * s * C, device=x.device, dtype=dtype)
    _lib.call("svk_nchw_to_s2d", dtype_code(dtype), _p(x), _p(out), B, C, H, W, s, pad, nbh, nbw, _stream())
    return out


def gauss5x5_s2d(x, dtype, pad, nbh, nbw):
    """GaussianFilter.conv_gauss of an NCHW f32 map (C <= 3) -> space-to-depth blocks [B, nbh, nbw, 48]."""
    _chk(x, "x", torch.float32)
    x = x.contiguous()
    B, C, H, W = x.shape
    out = torch.empty(B, nbh, nbw, 48, device=x.device, dtype=dtype)
    _lib.call("svk_gauss5x5_s2d", dtype_code(dtype), _p(x), _p(out), B, C, H, W, pad, nbh, nbw, _stream())
    return out


def conv2d_stem_s2d(x, w_s2d, k, stride, pad, bias=None, act=None):
    """A k <= 2*stride, stride-4 conv of an NCHW f32 map with 2/3 channels, as the space-to-depth packing + a
    2x2 unpadded conv over the blocks -> NHWC [B, OH, OW, Cout]; w_s2d from svk.pack.conv_w_s2d."""
    B, C, H, W = x.shape
    OH, OW = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    xs = nchw_to_s2d(x if x.dtype == torch.float32 else x.float(), w_s2d.dtype, stride, pad, OH + 1, OW + 1)
    return conv2d_nhwc(xs, w_s2d, 2, 1, 0, bias=bias, act=act)


STEM_LN = os.environ.get("SVK_STEM_LN", "1") == "1"
STEM_LN16 = os.environ.get("SVK_STEM_LN16", "1") == "1"     # the 16-channel (handcrafted prompt) stem alone


def conv2d_s2d_ln_supported(dtype, cs, cout, ow):
    """True when svk_conv2d_s2d_ln (stage-1 patch embedding over s2d blocks + LayerNorm in one kernel) covers it."""
    return (STEM_LN and dtype in H16 and (int(cout) != 16 or STEM_LN16)
            and bool(_lib.load().svk_conv2d_s2d_ln_supported(dtype_code(dtype), int(cs), int(cout), int(ow))))


def conv2d_s2d_ln(xs, w_s2d, bias, gamma=None, beta=None, eps=1e-6):
    """xs [B, HB, WB, CS] space-to-depth blocks -> LN(conv2x2(xs) + bias) [B, HB-1, WB-1, Cout] (no LN when gamma
    is None); w_s2d [Cout, 4*CS] as svk.pack.conv_w_s2d packs it (svk_conv2d_s2d_ln)."""
    _chk(xs, "xs"); _chk(w_s2d, "w", xs.dtype); _chk(bias, "bias", torch.float32)
    _chk(gamma, "gamma", torch.float32); _chk(beta, "beta", torch.float32)
    B, HB, WB, CS = xs.shape
    Cout = w_s2d.shape[0]
    if not xs.is_contiguous() or not w_s2d.is_contiguous() or w_s2d.shape[1] != 4 * CS:
        raise _lib.SvkError("svk.conv2d_s2d_ln: layout mismatch")
    out = torch.empty(B, HB - 1, WB - 1, Cout, device=xs.device, dtype=xs.dtype)
    t0 = _prof_begin()
    _lib.call("svk_conv2d_s2d_ln", dtype_code(xs.dtype), _p(xs), B, HB, WB, CS, _p(w_s2d), _p(bias), _p(gamma),
              _p(beta), float(eps), _p(out), Cout, _stream())
    if t0 is not None:
        M = B * (HB - 1) * (WB - 1)
        _prof_end(t0, _last_kernel(), 2.0 * M * Cout * 4 * CS, (xs.numel() + M * Cout) * xs.element_size(),
                  (M, Cout, 4 * CS, "stem_s2d_ln"))
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


RESIZE_MULTI = os.environ.get("SVK_RESIZE_MULTI", "1") == "1"


def resize_bilinear_multi(levels, OH, OW, out):
    """levels: [(x [B, H*W, C] 16-bit, H, W)] (1-4, C % 8 == 0, unit channel stride) resized to OH x OW and
    written side by side along channels into out [B, OH*OW, >= sum C] (svk_resize_bilinear_multi, one
    launch; bit-identical to one resize_bilinear per level)."""
    n = len(levels)
    X = (ctypes.c_void_p * n)(*[_p(t) for t, _, _ in levels])
    ld = (ctypes.c_long * n)(*[t.stride(-2) for t, _, _ in levels])
    Hs = (ctypes.c_int * n)(*[h for _, h, _ in levels])
    Ws = (ctypes.c_int * n)(*[w for _, _, w in levels])
    Cs = (ctypes.c_int * n)(*[t.shape[-1] for t, _, _ in levels])
    for t, _, _ in levels:
        _chk(t, "x", out.dtype)
        if t.stride(-1) != 1:
            raise _lib.SvkError("svk.resize_bilinear_multi: unit channel stride required")
    _lib.call("svk_resize_bilinear_multi", dtype_code(out.dtype), n, X, ld, Hs, Ws, Cs, _p(out), out.stride(-2),
              out.shape[0], OH, OW, _stream())
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


class _LRU(collections.OrderedDict):
    """Bounded table cache (the ragged tables were keyed by every distinct batch of video
    lengths and never evicted, each entry holding device tensors)."""

    def __init__(self, cap):
        super().__init__()
        self.cap = cap

    def get(self, key, default=None):
        if key in self:
            self.move_to_end(key)
            return self[key]
        return default

    def __setitem__(self, key, value):
        super().__setitem__(key, value)
        self.move_to_end(key)
        while len(self) > self.cap:
            self.popitem(last=False)


_TILE_CACHE = _LRU(int(os.environ.get("SVK_TABLE_CACHE", "64")))


def mstcn_tiles(lengths, device):
    """Device tile table of svk_mstcn_layer_ragged for videos of the given lengths, concatenated
    time-major in that order: int32 [ntiles, 4] = {first row of the video, T_v, tile start, 0}."""
    key = (tuple(int(t) for t in lengths), str(device))
    tab = _TILE_CACHE.get(key)
    if tab is None:
        tt = _lib.load().svk_mstcn_tile_size()
        rows, start = [], 0
        for T in key[0]:
            if T < 0:
                raise _lib.SvkError("svk.mstcn_tiles: negative video length")
            rows += [(start, T, t0, 0) for t0 in range(0, T, tt)]
            start += T
        tab = torch.tensor(rows, dtype=torch.int32).reshape(-1, 4).to(device)
        _TILE_CACHE[key] = tab
    return tab


def mstcn_layer(x, wdT, bd, w1T, b1, dilation, causal, out=None, tiles=None):
    """x [T, F] f32 time-major; wdT [3, F_in, F_out]; w1T [F_in, F_out] (transposed packs).
    ``tiles`` (mstcn_tiles): x is a ragged batch of videos concatenated time-major, one launch for all."""
    for t, nm in ((x, "x"), (wdT, "wdT"), (bd, "bd"), (w1T, "w1T"), (b1, "b1")):
        _chk(t, nm, torch.float32)
    T, F = x.shape
    if out is None:
        out = torch.empty_like(x)
    t0 = _prof_begin()
    if tiles is not None:
        _chk(tiles, "tiles", torch.int32)
        if tiles.dim() != 2 or tiles.shape[1] != 4 or not tiles.is_contiguous():
            raise _lib.SvkError("svk.mstcn_layer: tiles must be a contiguous [ntiles, 4] int32 table")
        _lib.call("svk_mstcn_layer_ragged", _p(x), _p(wdT), _p(bd), _p(w1T), _p(b1), _p(out), _p(tiles),
                  tiles.shape[0], F, dilation, 1 if causal else 0, _stream())
    else:
        _lib.call("svk_mstcn_layer", _p(x), _p(wdT), _p(bd), _p(w1T), _p(b1), _p(out), T, F, dilation,
                  1 if causal else 0, _stream())
    _prof_end(t0, "mstcn_layer_kernel", 8.0 * T * F * F, 8 * T * F, (T, F, "mstcn"))
    return out


_MAMBA_RAGGED = _LRU(int(os.environ.get("SVK_TABLE_CACHE", "64")))
MAMBA_RAGGED_SEG = int(os.environ.get("SVK_MAMBA_RAGGED_SEG", "256"))


def mamba_ragged(lengths, device, seg_len=None):
    """Tables of the ragged Mamba kernels for videos of the given lengths, concatenated time-major:
    (tpos int32 [sum T] = time index inside the video, segs int32 [nseg, 4] = {first row, T_v, segment z,
    the video's first record}, seg_len)."""
    seg = MAMBA_RAGGED_SEG if seg_len is None else int(seg_len)
    key = (tuple(int(t) for t in lengths), str(device), seg)
    hit = _MAMBA_RAGGED.get(key)
    if hit is None:
        tpos, segs, start = [], [], 0
        for T in key[0]:
            if T < 0:
                raise _lib.SvkError("svk.mamba_ragged: negative video length")
            base = len(segs)
            segs += [(start, T, z, base) for z in range(-(-T // seg))]
            tpos.append(torch.arange(T, dtype=torch.int32))
            start += T
        tp = (torch.cat(tpos) if tpos else torch.zeros(0, dtype=torch.int32)).to(device)
        hit = (tp, torch.tensor(segs, dtype=torch.int32).reshape(-1, 4).to(device), seg)
        _MAMBA_RAGGED[key] = hit
    return hit


def mamba_conv_silu(x, w, bias, B, T, ragged=None):
    """x [B*T, Di] f32 (row stride may exceed Di: the x-half of in_proj's xz) -> silu(causal depthwise
    conv) [B*T, Di]; w [Di, K]."""
    _chk(x, "x", torch.float32); _chk(w, "w", torch.float32); _chk(bias, "bias", torch.float32)
    M, Di, ldx = _rows(x, "x")
    if ragged is not None:      # (tpos, segs, seg_len) of mamba_ragged: B, T unused
        tpos = ragged[0]
        if tpos.numel() != M or w.shape[0] != Di or not w.is_contiguous():
            raise _lib.SvkError("svk.mamba_conv_silu: ragged table does not match x")
        out = torch.empty(M, Di, device=x.device, dtype=torch.float32)
        _lib.call("svk_mamba_conv_silu_ragged", _p(x), ldx, _p(w), _p(bias), _p(out), _p(tpos), M, Di, w.shape[1],
                  _stream())
        return out
    if M != B * T or w.shape[0] != Di or not w.is_contiguous():
        raise _lib.SvkError(f"svk.mamba_conv_silu: x {tuple(x.shape)} / w {tuple(w.shape)} vs B={B} T={T}")
    out = torch.empty(M, Di, device=x.device, dtype=torch.float32)
    _lib.call("svk_mamba_conv_silu", _p(x), ldx, _p(w), _p(bias), _p(out), B, T, Di, w.shape[1], _stream())
    return out


MAMBA_GROUPS = int(os.environ.get("SVK_MAMBA_GROUPS", "512"))


def mamba_seg_len(B, T, Di, N, target_groups=None):
    """Time-segment length for the two-pass scan: enough (video, channel-group, segment) workgroups
    for ~2 per CU (256 CUs), segments a multiple of the 32-step chunk; >= T means one sequential pass."""
    target_groups = MAMBA_GROUPS if target_groups is None else target_groups
    groups = B * -(-Di // (4 * (64 // N)))
    S = max(1, min(target_groups // max(groups, 1), -(-T // 64)))
    if S <= 1:
        return max(T, 1)
    return -(-(-(-T // S)) // 32) * 32


def mamba_scan(u, xdbl, z, w_dt, b_dt, a_neg, d_skip, B, T, seg_len=None, ragged=None):
    """Selective scan with the dt projection, softplus, D skip and silu(z) gate fused:
    u [B*T, Di], xdbl [B*T, R+2N] (dt_low | B | C), z [B*T, Di] (may be strided), w_dt [Di, R],
    a_neg = -exp(A_log) [Di, N] -> y [B*T, Di] (f32)."""
    for t, nm in ((u, "u"), (xdbl, "xdbl"), (z, "z"), (w_dt, "w_dt"), (b_dt, "b_dt"), (a_neg, "A"),
                  (d_skip, "D")):
        _chk(t, nm, torch.float32)
    M, Di, ldu = _rows(u, "u")
    Mx, W, ldxd = _rows(xdbl, "xdbl")
    Mz, Dz, ldz = _rows(z, "z")
    Dn, N = a_neg.shape
    R = w_dt.shape[1]
    if ragged is not None:
        B, T = 1, M               # the tables carry the video boundaries
    if (M != B * T or Mx != M or Mz != M or Dz != Di or ldu != Di or Dn != Di or W != R + 2 * N
            or not (w_dt.is_contiguous() and a_neg.is_contiguous())):
        raise _lib.SvkError("svk.mamba_scan: shape mismatch")
    out = torch.empty(M, Di, device=u.device, dtype=torch.float32)
    if ragged is not None:
        tpos, segs, seg = ragged
        nseg = segs.shape[0]
        ws = torch.empty(max(1, _lib.load().svk_mamba_scan_ragged_workspace(nseg, Di, N) // 4), device=u.device,
                         dtype=torch.float32)
        t0 = _prof_begin()
        _lib.call("svk_mamba_scan_ragged", _p(u), _p(xdbl), ldxd, _p(z), ldz, _p(w_dt), _p(b_dt), _p(a_neg),
                  _p(d_skip), _p(out), _p(segs), nseg, Di, N, R, seg, _p(ws), _stream())
        _prof_end(t0, f"mamba_scan_kernel<{N}>", M * Di * (2 * R + 6 + 6 * N), 4 * M * (3 * Di + W), (M, Di, N))
        return out
    seg = mamba_seg_len(B, T, Di, N) if seg_len is None else int(seg_len)
    nws = _lib.load().svk_mamba_scan_workspace(B, T, Di, N, seg)
    ws = torch.empty(nws // 4, device=u.device, dtype=torch.float32) if nws > 0 else None
    t0 = _prof_begin()
    _lib.call("svk_mamba_scan", _p(u), _p(xdbl), ldxd, _p(z), ldz, _p(w_dt), _p(b_dt), _p(a_neg), _p(d_skip),
              _p(out), B, T, Di, N, R, seg, _p(ws), _stream())
    # algorithmic: u, z, dt_low|B|C in, y out (f32); per (row, channel): 2R + 6 FLOP, per state 6 FLOP
    _prof_end(t0, f"mamba_scan_kernel<{N}>", M * Di * (2 * R + 6 + 6 * N), 4 * M * (3 * Di + W), (M, Di, N))
    return out


# ---- temporal-model training (tecno.py:195-259) ------------------------------------------------------

def mstcn_layer_train(x, wdT, bd, w1T, b1, dilation, causal, mask, out=None, hidden=None):
    """DilatedResidualLayer train forward: out = x + mask * (w1 relu(dilated conv) + b1); ``hidden``
    [T, F] receives relu(pre) for the backward.  mask [T, F] f32 (0 or 1/keep)."""
    for t, nm in ((x, "x"), (wdT, "wdT"), (bd, "bd"), (w1T, "w1T"), (b1, "b1"), (mask, "mask")):
        _chk(t, nm, torch.float32)
    T, F = x.shape
    if mask.numel() != T * F or not (x.is_contiguous() and mask.is_contiguous()):
        raise _lib.SvkError("svk.mstcn_layer_train: x / mask must be contiguous [T, F]")
    out = torch.empty_like(x) if out is None else out
    hidden = torch.empty_like(x) if hidden is None else hidden
    t0 = _prof_begin()
    _lib.call("svk_mstcn_layer_train", _p(x), _p(wdT), _p(bd), _p(w1T), _p(b1), _p(mask), _p(out), _p(hidden),
              T, F, dilation, 1 if causal else 0, _stream())
    # algorithmic: x, mask in; y, h out (f32); 3 dilated taps + the 1x1 conv per (t, f_out, f_in)
    _prof_end(t0, "mstcn_layer_kernel<train>", 8.0 * T * F * F, 16 * T * F, (T, F, "mstcn_train"))
    return out, hidden


def mstcn_layer_bwd(x, hidden, mask, dy, wd_packed, w1, dwd, dbd, dw1, db1, dilation, causal, dx=None, scratch=None,
                    ws=None):
    """Backward of mstcn_layer_train: returns dx; dwd [F, F, 3] (nn.Conv1d layout) / dbd / dw1 [F, F] / db1 += (f32).
    wd_packed [3, F_out, F_in]; w1 [F_out, F_in]; ws: optional scratch of svk_mstcn_bwd_workspace bytes."""
    for t, nm in ((x, "x"), (hidden, "hidden"), (mask, "mask"), (dy, "dy"), (wd_packed, "wd"), (w1, "w1"),
                  (dwd, "dwd"), (dbd, "dbd"), (dw1, "dw1"), (db1, "db1")):
        _chk(t, nm, torch.float32)
        if not t.is_contiguous():
            raise _lib.SvkError(f"svk.mstcn_layer_bwd: {nm} must be contiguous")
    T, F = x.shape
    dx = torch.empty_like(x) if dx is None else dx
    scratch = torch.empty_like(x) if scratch is None else scratch
    nws = _lib.load().svk_mstcn_bwd_workspace(T, F)
    if ws is None or ws.numel() * 4 < nws:
        ws = torch.empty(max(nws // 4, 1), device=x.device, dtype=torch.float32)
    t0 = _prof_begin()
    _lib.call("svk_mstcn_layer_bwd", _p(x), _p(hidden), _p(mask), _p(dy), _p(wd_packed), _p(w1), _p(scratch), _p(dx),
              _p(dwd), _p(dbd), _p(dw1), _p(db1), _p(ws), T, F, dilation, 1 if causal else 0, _stream())
    # algorithmic: x, h, mask, dy in, dpre out (kernel A); dy, dpre in, dx out (kernel B); dh, 4 weight
    # gradients and the 3-tap transposed conv per (t, f, f')
    _prof_end(t0, "mstcn_bwd", 16.0 * T * F * F, 32 * T * F, (T, F, "mstcn_bwd"))
    return dx


def softmax_rows_bwd(p, dp, residual=None, out=None):
    """dX = P * (dP - rowsum(P * dP)) (+ residual) over [M, C] f32."""
    _chk(p, "p", torch.float32); _chk(dp, "dp", torch.float32); _chk(residual, "residual", torch.float32)
    M, C, ldp = _rows(p, "p")
    _, _, lddp = _rows(dp, "dp")
    ldr = _rows(residual, "residual")[2] if residual is not None else 0
    out = torch.empty(M, C, device=p.device, dtype=torch.float32) if out is None else out
    _, _, ldo = _rows(out, "out")
    _lib.call("svk_softmax_rows_bwd", _p(p), ldp, _p(dp), lddp, _p(residual), ldr, _p(out), ldo, M, C, _stream())
    return out


def neg_exp(x, out=None):
    _chk(x, "x", torch.float32)
    out = torch.empty_like(x) if out is None else out
    if not (x.is_contiguous() and out.is_contiguous()) or out.numel() != x.numel():
        raise _lib.SvkError("svk.neg_exp: contiguous equal-size tensors required")
    _lib.call("svk_neg_exp", _p(x), _p(out), x.numel(), _stream())
    return out


def mamba_scan_train(u, xdbl, z, w_dt, b_dt, a_neg, d_skip, B, T, seg_len=None):
    """mamba_scan that also returns the pre-gate output yss = sum_n C h + D u (for the backward)."""
    for t, nm in ((u, "u"), (xdbl, "xdbl"), (z, "z"), (w_dt, "w_dt"), (b_dt, "b_dt"), (a_neg, "A"),
                  (d_skip, "D")):
        _chk(t, nm, torch.float32)
    M, Di, ldu = _rows(u, "u")
    Mx, W, ldxd = _rows(xdbl, "xdbl")
    Mz, Dz, ldz = _rows(z, "z")
    Dn, N = a_neg.shape
    R = w_dt.shape[1]
    if (M != B * T or Mx != M or Mz != M or Dz != Di or ldu != Di or Dn != Di or W != R + 2 * N
            or not (w_dt.is_contiguous() and a_neg.is_contiguous())):
        raise _lib.SvkError("svk.mamba_scan_train: shape mismatch")
    out = torch.empty(M, Di, device=u.device, dtype=torch.float32)
    yss = torch.empty(M, Di, device=u.device, dtype=torch.float32)
    seg = mamba_seg_len(B, T, Di, N) if seg_len is None else int(seg_len)
    nws = _lib.load().svk_mamba_scan_workspace(B, T, Di, N, seg)
    ws = torch.empty(nws // 4, device=u.device, dtype=torch.float32) if nws > 0 else None
    t0 = _prof_begin()
    _lib.call("svk_mamba_scan_train", _p(u), _p(xdbl), ldxd, _p(z), ldz, _p(w_dt), _p(b_dt), _p(a_neg), _p(d_skip),
              _p(out), _p(yss), B, T, Di, N, R, seg, _p(ws), _stream())
    _prof_end(t0, f"mamba_scan_kernel<{N}, train>", M * Di * (2 * R + 6 + 6 * N), 4 * M * (4 * Di + W), (M, Di, N))
    return out, yss


def mamba_scan_bwd(u, xdbl, z, w_dt, b_dt, a_neg, d_skip, yss, dout, dz, dxdbl, da, dd, B, T):
    """Selective-scan backward.  Returns (du, ds) [B*T, Di]; writes dz (a [B*T, Di] view, any row stride);
    dxdbl[:, R:] (the dB | dC columns) += and da [Di, N] / dd [Di] += (zero them first)."""
    for t, nm in ((u, "u"), (xdbl, "xdbl"), (z, "z"), (w_dt, "w_dt"), (b_dt, "b_dt"), (a_neg, "A"),
                  (d_skip, "D"), (yss, "yss"), (dout, "dout"), (dz, "dz"), (dxdbl, "dxdbl"), (da, "da"), (dd, "dd")):
        _chk(t, nm, torch.float32)
    M, Di, ldu = _rows(u, "u")
    _, W, ldxd = _rows(xdbl, "xdbl")
    _, _, ldz = _rows(z, "z")
    _, _, lddz = _rows(dz, "dz")
    _, Wd, lddxd = _rows(dxdbl, "dxdbl")
    Dn, N = a_neg.shape
    R = w_dt.shape[1]
    if (M != B * T or ldu != Di or W != R + 2 * N or Wd != W or not (yss.is_contiguous() and dout.is_contiguous())
            or yss.numel() != M * Di or dout.numel() != M * Di or not (da.is_contiguous() and dd.is_contiguous())):
        raise _lib.SvkError("svk.mamba_scan_bwd: shape mismatch")
    du = torch.empty(M, Di, device=u.device, dtype=torch.float32)
    ds = torch.empty(M, Di, device=u.device, dtype=torch.float32)
    nws = _lib.load().svk_mamba_scan_bwd_workspace(B, T, Di, N)
    ws = torch.empty(max(nws // 4, 1), device=u.device, dtype=torch.float32)
    t0 = _prof_begin()
    _lib.call("svk_mamba_scan_bwd", _p(u), _p(xdbl), ldxd, _p(z), ldz, _p(w_dt), _p(b_dt), _p(a_neg), _p(d_skip),
              _p(yss), _p(dout), _p(du), _p(dz), lddz, _p(ds), _p(dxdbl), lddxd, _p(da), _p(dd), B, T, Di, N, R,
              _p(ws), _stream())
    # algorithmic: u, z, yss, dout, dt_low|B|C in; du, dz, ds out, dB|dC accumulated (f32); the
    # forward recurrence twice (checkpoint pass + recompute) and the reverse one, ~6 FLOP each per state
    _prof_end(t0, f"mamba_scan_bwd_kernel<{N}>", M * Di * (2 * R + 20 + 18 * N), 4 * M * (7 * Di + 3 * W), (M, Di, N))
    return du, ds


def mamba_conv_silu_bwd(x, w, bias, dy, dx, dw, db, B, T):
    """Backward of mamba_conv_silu: writes dx (a [B*T, Di] view, any row stride); dw [Di, K] / db += ."""
    for t, nm in ((x, "x"), (w, "w"), (bias, "bias"), (dy, "dy"), (dx, "dx"), (dw, "dw"), (db, "db")):
        _chk(t, nm, torch.float32)
    M, Di, ldx = _rows(x, "x")
    _, _, lddx = _rows(dx, "dx")
    if M != B * T or not (dy.is_contiguous() and w.is_contiguous() and dw.is_contiguous()) or dy.numel() != M * Di:
        raise _lib.SvkError("svk.mamba_conv_silu_bwd: shape mismatch")
    scratch = torch.empty(M, Di, device=x.device, dtype=torch.float32)
    _lib.call("svk_mamba_conv_silu_bwd", _p(x), ldx, _p(w), _p(bias), _p(dy), _p(scratch), _p(dx), lddx, _p(dw),
              _p(db), B, T, Di, w.shape[1], _stream())
    return dx


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


# ---- training step (train_evp.py:473-515) ----------------------------------------------------------

def _f32_rows(t, name):
    _chk(t, name, torch.float32)
    return _rows(t, name)


def gemm_wgrad(dy, x, dw, db=None):
    """dw [N, K] f32 (row stride any) += dy[M, N]^T @ x[M, K]; db [N] f32 += column sums of dy."""
    _chk(dy, "dy"); _chk(x, "x", dy.dtype)
    M, N, ldy = _rows(dy, "dy")
    Mx, K, ldx = _rows(x, "x")
    _, _, lddw = _f32_rows(dw, "dw")
    if Mx != M or dw.shape[-1] != K or dw.numel() // K != N:
        raise _lib.SvkError(f"svk.gemm_wgrad: shapes dy {tuple(dy.shape)} x {tuple(x.shape)} dw {tuple(dw.shape)}")
    _chk(db, "db", torch.float32)
    if db is not None and (db.numel() != N or not db.is_contiguous()):
        raise _lib.SvkError("svk.gemm_wgrad: db shape mismatch")
    t0 = _prof_begin()
    if SKINNY and _skinny_wgrad_ok(dy, x, M, N, K):
        _lib.call("svk_wgrad_skinny", _p(dy), ldy, _p(x), ldx, _p(dw), lddw, _p(db), M, N, K, _stream())
        name = "skinny_wgrad"
    else:
        _lib.call("svk_gemm_wgrad", dtype_code(dy.dtype), _p(dy), ldy, _p(x), ldx, _p(dw), lddw, _p(db), M, N, K,
                  _stream())
        name = "wgrad_pk" if dy.dtype in H16 else "wgrad_kernel"
    _prof_end(t0, name, 2.0 * M * N * K, (M * (N + K)) * dy.element_size() + N * K * 4, (M, N, K, "wgrad"))
    return dw


def _pow2_tiles(x):
    t = (x + 15) // 16
    return 1 if t <= 1 else 2 if t <= 2 else 4 if t <= 4 else 8 if t <= 8 else 99


def _skinny_wgrad_ok(dy, x, M, N, K):
    return (dy.dtype == torch.bfloat16 and M >= 2048 and _pow2_tiles(N) * _pow2_tiles(K) <= 16
            and dy.data_ptr() % 16 == 0 and x.data_ptr() % 16 == 0)


def conv2d_wgrad(x, dy, k, stride, pad, dw, db=None):
    """x [B, H, W, Cin] NHWC, dy [B, OH, OW, Cout]; dw [Cout, k*k*Cin] f32 += (packed like conv_w);
    db [Cout] f32 += column sums of dy."""
    _chk(x, "x"); _chk(dy, "dy", x.dtype); _chk(dw, "dw", torch.float32)
    B, H, W, Cin = x.shape
    Cout = dy.shape[-1]
    if not (x.is_contiguous() and dy.is_contiguous() and dw.is_contiguous()) or dw.numel() != Cout * k * k * Cin:
        raise _lib.SvkError("svk.conv2d_wgrad: layout mismatch")
    t0 = _prof_begin()
    _chk(db, "db", torch.float32)
    _lib.call("svk_conv2d_wgrad_nhwc", dtype_code(x.dtype), _p(x), B, H, W, Cin, _p(dy), Cout, k, stride, pad, _p(dw),
              _p(db), _stream())
    M = dy.numel() // Cout
    _prof_end(t0, _last_kernel(), 2.0 * M * Cout * k * k * Cin, (x.numel() + dy.numel()) * x.element_size(),
              (M, Cout, k * k * Cin, f"convwgrad{k}s{stride}"))
    return dw


def conv2d_dgrad(dy, wd_packed, H, W, Cin, k, stride, pad, residual=None, out=None):
    """dy [B, OH, OW, Cout]; wd_packed [Cin, k*k*Cout] -> dx [B, H, W, Cin] (+ residual)."""
    _chk(dy, "dy"); _chk(wd_packed, "wd", dy.dtype)
    B, OH, OW, Cout = dy.shape
    if not dy.is_contiguous() or wd_packed.shape != (Cin, k * k * Cout) or not wd_packed.is_contiguous():
        raise _lib.SvkError("svk.conv2d_dgrad: layout mismatch")
    if out is None:
        out = torch.empty(B, H, W, Cin, device=dy.device, dtype=dy.dtype)
    for t, nm in ((out, "out"), (residual, "residual")):
        if t is not None and (t.shape != (B, H, W, Cin) or not t.is_contiguous() or t.dtype != dy.dtype):
            raise _lib.SvkError(f"svk.conv2d_dgrad: {nm} mismatch")
    t0 = _prof_begin()
    _lib.call("svk_conv2d_dgrad_nhwc", dtype_code(dy.dtype), _p(dy), B, OH, OW, Cout, _p(wd_packed), _p(residual),
              _p(out), H, W, Cin, k, stride, pad, _stream())
    M = B * H * W
    vec = dy.data_ptr() % 16 == 0 and wd_packed.data_ptr() % 16 == 0 and Cout % 8 == 0
    _prof_end(t0, _last_kernel(), 2.0 * M * Cin * k * k * Cout / stride ** 2,
              (dy.numel() + out.numel()) * dy.element_size(), (M, Cin, k * k * Cout, f"convdgrad{k}s{stride}"))
    return out


def conv2d_dgrad_col2im(dy, wc, H, W, Cin, k, stride, pad, residual=None, out=None):
    """Conv data gradient as the per-tap product GEMM P = dy @ wc.T ([B*OH*OW, k*k*Cin], exactly the
    k*k*Cin*Cout MACs per output pixel) followed by the col2im gather (svk_col2im_nhwc) -> dx [B, H, W, Cin]
    (+ residual).  wc [(ky, kx, ci), co]; bf16 / f16, Cin % 8 == 0."""
    _chk(dy, "dy"); _chk(wc, "wc", dy.dtype)
    B, OH, OW, Cout = dy.shape
    if not dy.is_contiguous() or wc.shape != (k * k * Cin, Cout) or not wc.is_contiguous():
        raise _lib.SvkError("svk.conv2d_dgrad_col2im: layout mismatch")
    if out is None:
        out = torch.empty(B, H, W, Cin, device=dy.device, dtype=dy.dtype)
    for t, nm in ((out, "out"), (residual, "residual")):
        if t is not None and (t.shape != (B, H, W, Cin) or not t.is_contiguous() or t.dtype != dy.dtype):
            raise _lib.SvkError(f"svk.conv2d_dgrad_col2im: {nm} mismatch")
    p = gemm(dy.view(B * OH * OW, Cout), wc)
    t0 = _prof_begin()
    _lib.call("svk_col2im_nhwc", dtype_code(dy.dtype), _p(p), _p(residual), _p(out), B, H, W, Cin, OH, OW, k, stride,
              pad, _stream())
    _prof_end(t0, "col2im", 0.0, (p.numel() + out.numel() * (1 if residual is None else 2)) * dy.element_size(),
              (B * H * W, Cin, k * k, f"col2im{k}s{stride}"))
    return out


def gemm_unpatchify(a, w, out, s, residual=None):
    """out NHWC [B, H, W, C] = unpatchify(a [B*(H/s)*(W/s), K] @ w.T) + residual (adjoint of the k = s
    patchify conv; w [(i, j, ci), K]).  residual may alias out."""
    _chk(a, "a"); _chk(w, "w", a.dtype); _chk(out, "out", a.dtype); _chk(residual, "residual", a.dtype)
    M, K, lda = _rows(a, "a")
    B, H, W, C = out.shape
    if not out.is_contiguous() or w.shape != (s * s * C, K) or M != B * (H // s) * (W // s):
        raise _lib.SvkError("svk.gemm_unpatchify: shape mismatch")
    if residual is not None and (residual.shape != out.shape or not residual.is_contiguous()):
        raise _lib.SvkError("svk.gemm_unpatchify: residual mismatch")
    t0 = _prof_begin()
    _lib.call("svk_gemm_unpatchify", dtype_code(a.dtype), _p(a), lda, _p(w), w.stride(0), _p(residual), _p(out), B,
              H, W, s, C, K, _stream())
    _prof_end(t0, "gemm_kernel(unpatchify)", 2.0 * M * s * s * C * K, (a.numel() + w.numel() + out.numel()) *
              a.element_size(), (M, s * s * C, K, "unpatchify"))
    return out


def unpatchify(p, B, PH, PW, s, C, out, accumulate=False):
    """p [B*PH*PW, s*s*C] -> out NHWC [B, PH*s, PW*s, C] (written or accumulated)."""
    _chk(p, "p"); _chk(out, "out", p.dtype)
    if not (p.is_contiguous() and out.is_contiguous()) or p.numel() != B * PH * PW * s * s * C or out.numel() != p.numel():
        raise _lib.SvkError("svk.unpatchify: shape mismatch")
    _lib.call("svk_unpatchify", dtype_code(p.dtype), _p(p), _p(out), B, PH, PW, s, C, 1 if accumulate else 0, _stream())
    return out


def attention_bwd(q, k, v, o, do, heads, scale, dk=None, dv=None, dq=None):
    """Backward of attention(q, k, v) -> (dq, dk, dv) in the compute dtype.  dk / dv may be given as
    views with equal strides (e.g. the two halves of one [B, Nk, 2C] buffer)."""
    for t, nm in ((q, "q"), (k, "k"), (v, "v"), (o, "o"), (do, "do")):
        _chk(t, nm, q.dtype)
        if t.dim() != 3 or t.stride(2) != 1:
            raise _lib.SvkError(f"svk.attention_bwd: {nm} must be [B, N, C] with unit channel stride")
    B, Nq, C = q.shape
    Nk = k.shape[1]
    if dk is None:
        kv = torch.empty(B, Nk, 2 * C, device=q.device, dtype=q.dtype)
        dk, dv = kv[:, :, :C], kv[:, :, C:]
    for t, nm in ((dk, "dk"), (dv, "dv")):
        _chk(t, nm, q.dtype)
        if t.shape != (B, Nk, C) or t.stride(2) != 1 or t.stride() != dk.stride():
            raise _lib.SvkError(f"svk.attention_bwd: {nm} must be [B, Nk, C] (unit channel stride, dk/dv alike)")
    if dq is None:
        dq = torch.empty(B, Nq, C, device=q.device, dtype=q.dtype)
    hd = C // heads
    nbytes = _lib.load().svk_attention_bwd_workspace(dtype_code(q.dtype), B, Nq, Nk, heads, hd)
    ws = torch.empty((nbytes + 15) // 16 * 4, device=q.device, dtype=torch.float32)
    t0 = _prof_begin()
    _lib.call("svk_attention_bwd", dtype_code(q.dtype), _p(q), q.stride(1), q.stride(0), _p(k), k.stride(1),
              k.stride(0), _p(v), v.stride(1), v.stride(0), _p(o), o.stride(1), o.stride(0), _p(do), do.stride(1),
              do.stride(0), _p(dq), dq.stride(1), dq.stride(0), _p(dk), _p(dv), dk.stride(1), dk.stride(0), _p(ws),
              ws.numel() * 4, B, Nq, Nk, heads, hd, float(scale), _stream())
    _prof_end(t0, "attention_bwd", 2.0 * B * Nq * Nk * C * 4, 0, (B, Nq, Nk, C, "attn_bwd"))
    return dq, dk, dv


def layernorm_bwd(x, dy, gamma, eps, dres=None, out=None, dgamma=None, dbeta=None):
    """dx = LN'(x; gamma)^T dy (+ dres); dgamma/dbeta (f32) += when given."""
    _chk(x, "x"); _chk(dy, "dy", x.dtype); _chk(gamma, "gamma", torch.float32); _chk(dres, "dres", x.dtype)
    M, C, ldx = _rows(x, "x")
    _, _, ldy = _rows(dy, "dy")
    if out is None:
        out = torch.empty(*x.shape, device=x.device, dtype=x.dtype)
    _, _, ldo = _rows(out, "out")
    ldr = _rows(dres, "dres")[2] if dres is not None else 0
    _lib.call("svk_layernorm_bwd", dtype_code(x.dtype), _p(x), ldx, _p(dy), ldy, _p(gamma), _p(dres), ldr, _p(out),
              ldo, _p(dgamma), _p(dbeta), M, C, float(eps), _stream())
    return out


def act_bwd(u, dy, act, dres=None, out=None):
    _chk(u, "u"); _chk(dy, "dy", u.dtype); _chk(dres, "dres", u.dtype)
    for t in (u, dy, dres):
        if t is not None and not t.is_contiguous():
            raise _lib.SvkError("svk.act_bwd: contiguous tensors required")
    if out is None:
        out = torch.empty_like(u)
    _lib.call("svk_act_bwd", dtype_code(u.dtype), _p(u), _p(dy), _p(dres), _p(out), u.numel(), ACT[act], _stream())
    return out


def _stats_ws(M, C, device):
    """Workspace of the deterministic column reductions (svk_colstats / svk_bn_bwd): per-block partials."""
    n = _lib.load().svk_stats_ws_floats(M, C)
    if n < 0:
        raise _lib.SvkError(f"svk: bad statistics shape M={M} C={C}")
    return torch.empty(n, device=device, dtype=torch.float32)


def colstats(x, s, sq=None):
    """s (+ sq) f32 [C] += column sums (of squares) of x [M, C] (deterministic: fixed-order reduction)."""
    _chk(x, "x"); _chk(s, "sum", torch.float32); _chk(sq, "sumsq", torch.float32)
    M, C, ldx = _rows(x, "x")
    _lib.call("svk_colstats", dtype_code(x.dtype), _p(x), ldx, M, C, _p(s), _p(sq), _p(_stats_ws(M, C, x.device)),
              _stream())
    return s


def colstats_set(x, out=None):
    """f32 [2, C]: row 0 = column sums, row 1 = column sums of squares of x [M, C], written (not accumulated:
    no zero-fill launch), the same fixed-order reduction as colstats."""
    _chk(x, "x")
    M, C, ldx = _rows(x, "x")
    if out is None:
        out = torch.empty(2, C, device=x.device, dtype=torch.float32)
    _chk(out, "out", torch.float32)
    if tuple(out.shape) != (2, C) or not out.is_contiguous():
        raise _lib.SvkError(f"svk.colstats_set: out must be a contiguous f32 [2, {C}] tensor, got {tuple(out.shape)}")
    _lib.call("svk_colstats_set", dtype_code(x.dtype), _p(x), ldx, M, C, _p(out), _p(_stats_ws(M, C, x.device)),
              _stream())
    return out


def bn_apply(x, s, sq, gamma, beta, eps, act=None, out=None):
    _chk(x, "x")
    C = x.shape[-1]
    M = x.numel() // C
    if out is None:
        out = torch.empty_like(x)
    _lib.call("svk_bn_apply", dtype_code(x.dtype), _p(x), _p(s), _p(sq), _p(gamma), _p(beta), _p(out), M, C,
              float(eps), ACT[act], _stream())
    return out


def bn_bwd(x, dy, s, sq, gamma, beta, eps, dgamma, dbeta, relu=True, out=None):
    _chk(x, "x"); _chk(dy, "dy", x.dtype)
    C = x.shape[-1]
    M = x.numel() // C
    if out is None:
        out = torch.empty_like(x)
    _lib.call("svk_bn_bwd", dtype_code(x.dtype), _p(x), _p(dy), _p(s), _p(sq), _p(gamma), _p(beta), _p(out),
              _p(dgamma), _p(dbeta), M, C, float(eps), 1 if relu else 0, _p(_stats_ws(M, C, x.device)), _stream())
    return out


def bn_update_running(s, sq, M, running_mean, running_var, momentum):
    _lib.call("svk_bn_update_running", _p(s), _p(sq), M, s.numel(), float(momentum), _p(running_mean),
              _p(running_var), _stream())


def resize_bilinear_bwd(dy, H, W, OH, OW, dx):
    """dx f32 [B, H*W, C] += adjoint of resize_bilinear applied to dy [B, OH*OW, C]."""
    _chk(dy, "dy"); _chk(dx, "dx", torch.float32)
    B, C = dy.shape[0], dy.shape[-1]
    if not dx.is_contiguous() or dx.numel() != B * H * W * C:
        raise _lib.SvkError("svk.resize_bilinear_bwd: dx shape mismatch")
    _lib.call("svk_resize_bilinear_bwd", dtype_code(dy.dtype), _p(dy), dy.stride(-2), _p(dx), B, H, W, C, OH, OW,
              _stream())
    return dx


def bcast_rows(df, R, dtype, scale=1.0, mask=None):
    """df f32 [B, C] -> [B*R, C] (dtype) rows df[b] * mask[b] * scale."""
    _chk(df, "df", torch.float32); _chk(mask, "mask", torch.float32)
    B, C = df.shape
    out = torch.empty(B * R, C, device=df.device, dtype=dtype)
    _lib.call("svk_bcast_rows", dtype_code(dtype), _p(df.contiguous()), _p(mask), float(scale), _p(out), B, R, C,
              _stream())
    return out


def mul_f32(a, b, out=None):
    _chk(a, "a", torch.float32); _chk(b, "b", torch.float32)
    out = torch.empty_like(a) if out is None else out
    if not (a.is_contiguous() and b.is_contiguous() and out.is_contiguous()) or not (a.numel() == b.numel() == out.numel()):
        raise _lib.SvkError("svk.mul_f32: contiguous equal-size tensors required")
    _lib.call("svk_mul_f32", _p(a), _p(b), _p(out), a.numel(), _stream())
    return out


def keep_mask(n, keep, seed, device, counter=None):
    """Bernoulli(keep)/keep mask of n floats; ``counter`` (device int64 tensor) is mixed in at run time."""
    _chk(counter, "counter", torch.int64)
    out = torch.empty(n, device=device, dtype=torch.float32)
    _lib.call("svk_keep_mask", _p(out), n, float(keep), int(seed) & 0xFFFFFFFF, _p(counter), _stream())
    return out


def keep_mask_multi(n, keeps, seeds, counter=None):
    """[len(keeps), n] f32: row m = keep_mask(n, keep, seed) for the m-th (keep, seed), bit for bit, in one
    launch.  keeps: device f32 [nm] (the float32 values keep_mask would receive), seeds: device int32 [nm]
    (the low 32 bits of the seeds)."""
    _chk(keeps, "keeps", torch.float32); _chk(seeds, "seeds", torch.int32); _chk(counter, "counter", torch.int64)
    nm = keeps.numel()
    if seeds.numel() != nm or not (keeps.is_contiguous() and seeds.is_contiguous()):
        raise _lib.SvkError("svk.keep_mask_multi: keeps / seeds must be contiguous [nm]")
    out = torch.empty(nm, n, device=keeps.device, dtype=torch.float32)
    _lib.call("svk_keep_mask_multi", _p(out), n, nm, _p(keeps), _p(seeds), _p(counter), _stream())
    return out


def phase_loss(logits, ant, labels, ant_targets):
    """CE(sum) + SmoothL1(sum) -> (loss f32 [2], dlogits, dant)."""
    for t, nm in ((logits, "logits"), (ant, "ant"), (ant_targets, "ant_targets")):
        _chk(t, nm, torch.float32)
    _chk(labels, "labels", torch.int64)
    B, K = logits.shape
    loss = torch.zeros(2, device=logits.device, dtype=torch.float32)
    dl = torch.empty_like(logits)
    da = torch.empty_like(ant)
    _lib.call("svk_phase_loss", _p(logits.contiguous()), _p(ant.contiguous()), _p(labels.contiguous()),
              _p(ant_targets.contiguous()), B, K, _p(loss), _p(dl), _p(da), _stream())
    return loss, dl, da


def sgd(p, g, buf, lr, momentum, dampening, wd, nesterov, first):
    _lib.call("svk_sgd", _p(p), _p(g), _p(buf), p.numel(), float(lr), float(momentum), float(dampening), float(wd),
              1 if nesterov else 0, 1 if first else 0, _stream())


def pack_params(desc, ndesc, total, src, dst):
    _lib.call("svk_pack_params", dtype_code(dst.dtype), _p(desc), ndesc, total, _p(src), _p(dst), _stream())


def pack_params8(desc, ndesc, total, src, dst):
    """svk_pack_params8: descriptor starts and packed offsets 8-aligned, total % 8 == 0."""
    _lib.call("svk_pack_params8", dtype_code(dst.dtype), _p(desc), ndesc, total, _p(src), _p(dst), _stream())


def pack_transpose(tiles, ntiles, src, dst):
    _lib.call("svk_pack_transpose", dtype_code(dst.dtype), _p(tiles), ntiles, _p(src), _p(dst), _stream())


def tecno_loss(logits, labels, ant_targets, class_w=None, out=None, dlogits=None):
    """tecno.py:237-254 loss over time-major logits [S, T, 2P] -> (loss f32 [3] = (clc, ant, #correct
    of the last stage), dlogits [S, T, 2P] = d(clc + ant))."""
    _chk(logits, "logits", torch.float32); _chk(labels, "labels", torch.int64)
    _chk(ant_targets, "ant_targets", torch.float32); _chk(class_w, "class_w", torch.float32)
    if logits.dim() != 3 or logits.stride(2) != 1:
        raise _lib.SvkError("svk.tecno_loss: logits must be [S, T, 2P] with unit column stride")
    S, T, C = logits.shape
    P = C // 2
    if C != 2 * P or labels.numel() != T or ant_targets.shape != (T, P) or not ant_targets.is_contiguous():
        raise _lib.SvkError("svk.tecno_loss: shape mismatch")
    out = torch.empty(3, device=logits.device, dtype=torch.float32) if out is None else out
    dlogits = torch.empty_like(logits) if dlogits is None else dlogits
    if dlogits.stride() != logits.stride():
        raise _lib.SvkError("svk.tecno_loss: dlogits must share the logits layout")
    _lib.call("svk_tecno_loss", _p(logits), logits.stride(1), logits.stride(0), S, T, P, _p(labels.contiguous()),
              _p(ant_targets), _p(class_w), _p(out), _p(dlogits), _stream())
    return out, dlogits


NORM_PARTS = 256   # csrc/tecno_train.hip NORM_PARTS (svk_norm_parts())


def grad_sqnorm(g, partials, step=None):
    _chk(g, "g", torch.float32); _chk(partials, "partials", torch.float32); _chk(step, "step", torch.int64)
    if partials.numel() < NORM_PARTS or not g.is_contiguous():
        raise _lib.SvkError("svk.grad_sqnorm: partials must hold svk_norm_parts() floats, g contiguous")
    _lib.call("svk_grad_sqnorm", _p(g), g.numel(), _p(partials), _p(step), _stream())


def adamw(p, g, m, v, lr, step, partials=None, max_norm=0.0, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=1e-2):
    """clip_grad_norm_(max_norm) (when partials from grad_sqnorm are given) + torch.optim.AdamW step over
    flat f32 buffers; lr (f32 [1]) and step (int64 [1], already advanced) live on the device."""
    for t, nm in ((p, "p"), (g, "g"), (m, "m"), (v, "v"), (lr, "lr"), (partials, "partials")):
        _chk(t, nm, torch.float32)
    _chk(step, "step", torch.int64)
    n = p.numel()
    if any(t.numel() != n or not t.is_contiguous() for t in (g, m, v)) or not p.is_contiguous():
        raise _lib.SvkError("svk.adamw: p / g / m / v must be contiguous and equally sized")
    _lib.call("svk_adamw", _p(p), _p(g), _p(m), _p(v), n, _p(partials), float(max_norm), _p(lr), float(beta1),
              float(beta2), float(eps), float(weight_decay), _p(step), _stream())


def mstcn_bwd_floats(T, F):
    """f32 count of the svk_mstcn_layer_bwd workspace for a [T, F] layer."""
    return _lib.load().svk_mstcn_bwd_workspace(T, F) // 4
