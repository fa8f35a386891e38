"""CPU restatement of the extraction frame transform (oracle / test infrastructure only).

generate_evp_LFB.py:243-247: ``transforms.Compose([Resize((250, 250)), CenterCrop(224), ToTensor(),
Normalize(mean, std)])`` applied to ``pil_loader(path, mode='RGB')`` frames (data_process.py) — and to the
RGB segmaps (data_process.py:455-462).  The resize is Pillow's (torchvision's PIL path calls
``Image.resize(size[::-1], BILINEAR)``): restated here from Pillow's libImaging/Resample.c (Pillow 12.2.0 is
the version in this image): per-axis windows/weights from ``precompute_coeffs`` (bilinear filter, support
widened by the downscale factor), ``normalize_coeffs_8bpc`` (22-bit fixed point), horizontal pass then
vertical pass, each ``+2^21``, ``>> 22``, clip to [0, 255].  torchvision is absent here: CenterCrop offset =
``int(round((size - crop) / 2.0))``, ToTensor = ``u8.float().div(255)``, Normalize = ``sub_(mean).div_(std)``
(f32).  Pinned by tests/test_preproc_cpu.py against Pillow itself (bit-exact).
"""
import math

import numpy as np
import torch

PREC = 22


def _axis(in_size, out_size):
    scale = in_size / out_size
    fs = max(scale, 1.0)
    support = fs
    ksize = int(math.ceil(support)) * 2 + 1
    idx = np.zeros((out_size, ksize), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        n = min(int(center + support + 0.5), in_size) - xmin
        w = [max(0.0, 1.0 - abs((x + xmin - center + 0.5) * (1.0 / fs))) for x in range(n)]
        ww = 0.0
        for v in w:
            ww += v
        for x in range(n):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + k * (1 << PREC)) if k < 0 else int(0.5 + k * (1 << PREC))
            idx[xx, x] = xmin + x
        idx[xx, n:] = xmin
    return idx, kk


def _pass(img, idx, kk, axis):
    """One 8-bit resampling pass along ``axis`` of an int64 [H, W, C] image."""
    taps = np.take(img, idx, axis=axis)                  # axis expanded to [out, ksize]
    if axis == 1:
        acc = (taps * kk[None, :, :, None]).sum(2)
    else:
        acc = (taps * kk[:, :, None, None]).sum(1)
    return np.clip((acc + (1 << (PREC - 1))) >> PREC, 0, 255)


def pil_resize_bilinear(img_u8, out_hw):
    """img [H, W, 3] uint8 -> Pillow BILINEAR resize to (OH, OW), uint8."""
    H, W, _ = img_u8.shape
    OH, OW = out_hw
    x = img_u8.astype(np.int64)
    xi, xk = _axis(W, OW)
    x = _pass(x, xi, xk, 1)
    yi, yk = _axis(H, OH)
    x = _pass(x, yi, yk, 0)
    return x.astype(np.uint8)


def frame_transform(img_u8, size=(250, 250), crop=224, mean=(0.41757566, 0.26098573, 0.25888634),
                    std=(0.21938758, 0.1983, 0.19342837)):
    """[H, W, 3] uint8 -> [3, crop, crop] f32 (the DataLoader's per-frame tensor)."""
    r = pil_resize_bilinear(img_u8, size)
    t = int(round((size[0] - crop) / 2.0))
    l = int(round((size[1] - crop) / 2.0))
    c = torch.from_numpy(np.ascontiguousarray(r[t:t + crop, l:l + crop])).permute(2, 0, 1).contiguous()
    x = c.to(torch.float32).div(255)
    m = torch.as_tensor(mean, dtype=torch.float32)[:, None, None]
    s = torch.as_tensor(std, dtype=torch.float32)[:, None, None]
    return x.sub_(m).div_(s)


# ---- optical flow (data_process.py:425-447): cv2.resize INTER_LINEAR on float32, displacement rescale, crop ----
# cv2 (opencv-python) is absent from this image: the restatement follows OpenCV's resizeGeneric_ for
# INTER_LINEAR on CV_32F (HResizeLinear + VResizeLinear): fx = (float)((dx + 0.5) * scale - 0.5),
# sx = floor(fx), fx -= sx, clamped to (0, 0) below and (size - 1, 0) above; horizontal blend per source row,
# then vertical blend, each as f32 multiply + add.  **Parity against cv2 unpinned** (OpenCV's SIMD vertical
# blend may use FMA, a <= 1-ulp difference); the GPU kernel is checked against this restatement.

def _cv_axis(in_size, out_size):
    scale = 1.0 / (float(out_size) / in_size)
    i0 = np.zeros(out_size, np.int64)
    w = np.zeros((out_size, 2), np.float32)
    for d in range(out_size):
        f = np.float32((d + 0.5) * scale - 0.5)
        sidx = int(np.floor(f))
        f = np.float32(f - np.float32(sidx))
        if sidx < 0:
            sidx, f = 0, np.float32(0)
        if sidx >= in_size - 1:
            sidx, f = in_size - 1, np.float32(0)
        i0[d] = sidx
        w[d] = (np.float32(1) - f, f)
    return i0, np.minimum(i0 + 1, in_size - 1), w


def cv2_resize_linear(img, out_hw):
    """img [H, W, C] float32 -> [OH, OW, C] float32 (cv2.resize(img, (OW, OH), interpolation=INTER_LINEAR))."""
    H, W, _ = img.shape
    OH, OW = out_hw
    x0, x1, wx = _cv_axis(W, OW)
    y0, y1, wy = _cv_axis(H, OH)
    hr = img[:, x0, :] * wx[None, :, 0:1] + img[:, x1, :] * wx[None, :, 1:2]      # f32 mul, f32 add
    return (hr[y0] * wy[:, 0:1, None] + hr[y1] * wy[:, 1:2, None]).astype(np.float32)


def flow_transform(flow, size=(250, 250), crop=224):
    """flow [H, W, 2] float32 -> [2, crop, crop] f32 as CholecFlowDataset + CenterCrop produce it."""
    H, W, _ = flow.shape
    r = cv2_resize_linear(flow.astype(np.float32), size)
    r[:, :, 0] *= size[1] / W                  # numpy 2: python float is weak -> f32 multiply
    r[:, :, 1] *= size[0] / H
    t = int(round((size[0] - crop) / 2.0))
    l = int(round((size[1] - crop) / 2.0))
    return torch.from_numpy(np.ascontiguousarray(r[t:t + crop, l:l + crop])).permute(2, 0, 1).contiguous()
