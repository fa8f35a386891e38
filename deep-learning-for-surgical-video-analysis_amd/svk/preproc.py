"""GPU frame preprocessing: the extraction transform of generate_evp_LFB.py:243-247
(``Resize((250, 250))`` -> ``CenterCrop(224)`` -> ``ToTensor()`` -> ``Normalize(mean, std)``) on decoded
uint8 RGB frames, bit-exact to Pillow + torch.

The resampling windows and fixed-point coefficients are computed here on the host exactly as Pillow's
``libImaging/Resample.c`` does (``precompute_coeffs`` with the bilinear filter, support 1, widened by the
downscale factor; ``normalize_coeffs_8bpc`` with 22 fractional bits — the Pillow in this image is 12.2.0),
uploaded once per (input size, output size) and consumed by ``svk_frame_preproc``.
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib
from .ops import _chk, _p, _prof_begin, _prof_end, _stream

CHOLEC80_MEAN = (0.41757566, 0.26098573, 0.25888634)     # generate_evp_LFB.py:247 / train_evp.py:152
CHOLEC80_STD = (0.21938758, 0.1983, 0.19342837)
PRECISION_BITS = 32 - 8 - 2


def pillow_bilinear_coeffs(in_size, out_size):
    """(bounds [out, 2] = (first tap, tap count), fixed-point coefficients [out, ksize], ksize) for a
    Pillow BILINEAR resize of one axis from ``in_size`` to ``out_size`` (box = the whole axis)."""
    scale = float(in_size) / out_size          # (double)(in1 - in0) / outSize, in0 = 0, in1 = in_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    coef = np.zeros((out_size, ksize), np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w.append(1.0 - t if t < 1.0 else 0.0)
        ww = 0.0
        for v in w:
            ww += v
        for x, v in enumerate(w):
            k = v / ww if ww != 0.0 else v
            coef[xx, x] = int(-0.5 + k * (1 << PRECISION_BITS)) if k < 0 else int(0.5 + k * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, xmax)
    return bounds, coef, ksize


_COEF_CACHE = {}


def _coeffs(in_size, out_size, device):
    key = (in_size, out_size, device)
    if key not in _COEF_CACHE:
        b, c, k = pillow_bilinear_coeffs(in_size, out_size)
        _COEF_CACHE[key] = (torch.from_numpy(b).to(device), torch.from_numpy(c).to(device), k)
    return _COEF_CACHE[key]


def center_crop_offsets(size, crop):
    """torchvision CenterCrop: top/left = int(round((size - crop) / 2.0))."""
    if crop > size:
        raise _lib.SvkError(f"svk.frame_transform: crop {crop} larger than the resized frame {size}")
    return int(round((size - crop) / 2.0))


def frame_transform(frames, size=(250, 250), crop=224, mean=CHOLEC80_MEAN, std=CHOLEC80_STD, out=None):
    """frames [B, H, W, 3] uint8 (decoded RGB, on the GPU) -> [B, 3, crop, crop] f32, equal to
    ``Normalize(mean, std)(ToTensor()(CenterCrop(crop)(Resize(size)(PIL frame))))`` stacked over B."""
    _chk(frames, "frames", torch.uint8)
    if frames.dim() != 4 or frames.shape[-1] != 3 or not frames.is_contiguous():
        raise _lib.SvkError(f"svk.frame_transform: frames must be contiguous [B, H, W, 3] uint8, got "
                            f"{tuple(frames.shape)}")
    B, H, W, _ = frames.shape
    OH, OW = size
    CH = CW = crop
    cy0, cx0 = center_crop_offsets(OH, CH), center_crop_offsets(OW, CW)
    xb, xk, ksx = _coeffs(W, OW, frames.device)
    yb, yk, ksy = _coeffs(H, OH, frames.device)
    tmp = torch.empty(B, H, CW, 3, device=frames.device, dtype=torch.uint8)
    if out is None:
        out = torch.empty(B, 3, CH, CW, device=frames.device, dtype=torch.float32)
    _chk(out, "out", torch.float32)
    if tuple(out.shape) != (B, 3, CH, CW) or not out.is_contiguous():
        raise _lib.SvkError("svk.frame_transform: out must be contiguous [B, 3, crop, crop] f32")
    m, sd = (ctypes.c_float * 3)(*mean), (ctypes.c_float * 3)(*std)     # host arrays, read at launch
    t0 = _prof_begin()
    _lib.call("svk_frame_preproc", _p(frames), _p(tmp), _p(out), _p(xb), _p(xk), ksx, _p(yb), _p(yk), ksy, B, H, W,
              cy0, cx0, CH, CW, ctypes.addressof(m), ctypes.addressof(sd), _stream())
    # algorithmic bytes: the decoded frames in, the f32 crop out (the uint8 horizontal-pass scratch is extra)
    _prof_end(t0, "frame_preproc", B * (CW * H * ksx + CH * CW * ksy) * 3 * 2, B * (H * W * 3 + 3 * CH * CW * 4),
              (B, H, W))
    return out


def cv2_linear_table(in_size, out_size):
    """cv2.resize INTER_LINEAR (float images) per-axis table: source index and (1 - f, f) float32 weights,
    fx = (float)((dx + 0.5) * scale - 0.5), scale = 1 / (out / in) in double, clamped at both edges."""
    scale = 1.0 / (float(out_size) / in_size)
    ofs = np.zeros(out_size, np.int32)
    alpha = np.zeros((out_size, 2), np.float32)
    for dx in range(out_size):
        fx = np.float32((dx + 0.5) * scale - 0.5)
        sx = int(math.floor(fx))
        fx = np.float32(fx - np.float32(sx))
        if sx < 0:
            fx, sx = np.float32(0.0), 0
        if sx >= in_size - 1:
            fx, sx = np.float32(0.0), in_size - 1
        ofs[dx] = sx
        alpha[dx] = (np.float32(1.0) - fx, fx)
    return ofs, alpha


_CV_CACHE = {}


def flow_transform(flow, size=(250, 250), crop=224, out=None):
    """flow [B, H, W, 2] f32 (the RAFT .npy fields, on the GPU) -> [B, 2, crop, crop] f32: CholecFlowDataset's
    cv2 resize + displacement rescale (data_process.py:425-447) and the transform's CenterCrop."""
    _chk(flow, "flow", torch.float32)
    if flow.dim() != 4 or flow.shape[-1] != 2 or not flow.is_contiguous():
        raise _lib.SvkError(f"svk.flow_transform: flow must be contiguous [B, H, W, 2] f32, got {tuple(flow.shape)}")
    B, H, W, _ = flow.shape
    OH, OW = size
    cy0, cx0 = center_crop_offsets(OH, crop), center_crop_offsets(OW, crop)
    key = (H, W, OH, OW, flow.device)
    if key not in _CV_CACHE:
        xo, xa = cv2_linear_table(W, OW)
        yo, ya = cv2_linear_table(H, OH)
        d = flow.device
        _CV_CACHE[key] = tuple(torch.from_numpy(a).to(d) for a in (xo, xa, yo, ya))
    xo, xa, yo, ya = _CV_CACHE[key]
    if out is None:
        out = torch.empty(B, 2, crop, crop, device=flow.device, dtype=torch.float32)
    _chk(out, "out", torch.float32)
    if tuple(out.shape) != (B, 2, crop, crop) or not out.is_contiguous():
        raise _lib.SvkError("svk.flow_transform: out must be contiguous [B, 2, crop, crop] f32")
    su, sv = float(np.float32(OW / W)), float(np.float32(OH / H))     # numpy: f32 array *= python float
    _lib.call("svk_flow_preproc", _p(flow), _p(out), _p(xo), _p(xa), _p(yo), _p(ya), B, H, W, cy0, cx0, crop, crop,
              su, sv, _stream())
    return out
