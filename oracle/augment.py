"""CPU restatement of the TRAINING-time augmentations (oracle / test infrastructure only).

train_evp.py:146-163 builds ``transforms.Compose([Resize((250, 250)), RandomCrop(224), [ColorJitter(0.1, 0.1, 0.1,
0.05)], RandomHorizontalFlip(), [RandomRotation(5)], ToTensor(), Normalize(mean, std)])`` (the bracketed steps
only with ``use_flip == 1``) from the synced classes of data_process.py:53-186, and CholecFlowDataset
(data_process.py:425-487) applies it to the decoded RGB frame, to the RGB segmap, and — its geometric steps only
(Resize, RandomCrop, RandomHorizontalFlip, RandomRotation) — to the RAFT flow tensor.

The PIL-image arithmetic is restated from Pillow 12.2.0 (the version in this image; torchvision, which only
forwards to it for PIL inputs, is absent) and pinned bit-exactly against Pillow itself by
tests/test_augment_cpu.py:

* ``Image.blend(im1, im2, alpha)`` (libImaging/Blend.c; ImageEnhance.Brightness / Contrast / Color call it):
  ``in1 + alpha * (in2 - in1)`` in C float (alpha narrowed to float, multiply then add, each rounded), truncated
  to uint8 for 0 <= alpha <= 1, clipped to [0, 255] then truncated otherwise.
* ``convert("L")`` (libImaging/Convert.c): ``(R * 19595 + G * 38470 + B * 7471 + 0x8000) >> 16``.
* ImageEnhance.Contrast: degenerate = ``int(mean(L) + 0.5)`` (ImageStat's histogram mean, a double).
* ImageEnhance.Color: degenerate = the L image replicated to RGB.
* torchvision's PIL ``adjust_hue``: ``convert("HSV")``, ``h += uint8(hue * 255)`` (wrapping), back to RGB —
  Pillow's rgb2hsv / hsv2rgb (Convert.c) restated with their float / double promotions; pinned over all 2^24
  RGB and all 2^24 HSV triples.
* ``Image.rotate(angle, NEAREST, expand=False)``: the inverse matrix Image.rotate builds (cos / sin rounded to
  15 digits, centred), then ImagingTransformAffine's nearest path in 16.16 fixed point: ``FIX(v) =
  floor(v * 65536 + 0.5)``, the pixel-centre offset folded into the constant terms, source = ``(x*a0 + y*a1 +
  a2) >> 16`` (arithmetic shift), outside -> fill 0.  Pinned for every angle RandomRotation(5) draws.

The flow (tensor) path follows torchvision's tensor ops (absent here, so **parity unpinned**): crop = slicing,
flip = ``flip(-1)`` with u negated, rotate = ``_apply_grid_transform`` over the affine grid of
``_gen_affine_grid`` (base grid ``linspace(-w/2 + 0.5, w/2 - 0.5)``, theta = the inverse rotation, rescaled by
(w/2, h/2)) with ``grid_sample(mode="nearest", padding_mode="zeros", align_corners=False)``, then the vector
rotation of data_process.py:145-156 (f32 tensor times Python float).  The grid here is formed with explicit f32
operations in a fixed order (x * t0 + y * t1 + t2); the GPU kernel uses the same order.
"""
import math

import numpy as np
import torch

from . import preproc as PP

F32 = np.float32


def pil_blend(a, b, alpha):
    """Image.blend(a, b, alpha) on uint8 arrays of one shape."""
    af = F32(alpha)
    ai = a.astype(np.int64)
    t = ai.astype(F32) + af * (b.astype(np.int64) - ai).astype(F32)       # float * float, float + float
    if 0.0 <= alpha <= 1.0:
        return t.astype(np.int64).astype(np.uint8)                        # (UINT8) truncation, in range
    return np.where(t <= 0, 0, np.where(t >= 255, 255, np.trunc(t))).astype(np.uint8)


def pil_luma(rgb):
    """[..., 3] uint8 -> [...] uint8: Pillow's RGB -> L."""
    i = rgb.astype(np.int64)
    return ((i[..., 0] * 19595 + i[..., 1] * 38470 + i[..., 2] * 7471 + 0x8000) >> 16).astype(np.uint8)


def rgb_to_hsv(rgb):
    """Pillow's rgb2hsv_row over [..., 3] uint8."""
    r, g, b = (rgb[..., k].astype(np.int64) for k in range(3))
    maxc = np.maximum(r, np.maximum(g, b))
    minc = np.minimum(r, np.minimum(g, b))
    cr = (maxc - minc).astype(F32)
    with np.errstate(divide="ignore", invalid="ignore"):
        s = cr / maxc.astype(F32)
        rc, gc, bc = ((maxc - c).astype(F32) / cr for c in (r, g, b))
        h = np.where(r == maxc, (bc - gc).astype(F32),
                     np.where(g == maxc, (2.0 + rc.astype(np.float64) - bc.astype(np.float64)).astype(F32),
                              (4.0 + gc.astype(np.float64) - rc.astype(np.float64)).astype(F32)))
        h = np.fmod(h.astype(np.float64) / 6.0 + 1.0, 1.0).astype(F32)
        uh = np.clip(np.nan_to_num(h.astype(np.float64) * 255.0).astype(np.int64), 0, 255)
        us = np.clip(np.nan_to_num(s.astype(np.float64) * 255.0).astype(np.int64), 0, 255)
    eq = maxc == minc
    return np.stack([np.where(eq, 0, uh), np.where(eq, 0, us), maxc], -1).astype(np.uint8)


def hsv_to_rgb(hsv):
    """Pillow's hsv2rgb over [..., 3] uint8."""
    H, S, V = (hsv[..., k].astype(np.int64) for k in range(3))
    hd = H.astype(F32).astype(np.float64) * 6.0 / 255.0
    i = np.floor(hd).astype(np.int64)
    f = (hd - i.astype(F32).astype(np.float64)).astype(F32).astype(np.float64)
    fs = (S.astype(F32).astype(np.float64) / 255.0).astype(F32).astype(np.float64)
    v = V.astype(F32).astype(np.float64)
    cround = lambda x: np.floor(x + 0.5)                                   # C round(), x >= 0 here
    p = np.clip(cround(v * (1.0 - fs)).astype(np.int64), 0, 255)
    q = np.clip(cround(v * (1.0 - fs * f)).astype(np.int64), 0, 255)
    t = np.clip(cround(v * (1.0 - fs * (1.0 - f))).astype(np.int64), 0, 255)
    sel = [(V, t, p), (q, V, p), (p, V, t), (p, q, V), (t, p, V), (V, p, q)]
    out = np.zeros(H.shape + (3,), np.int64)
    k6 = i % 6
    for k in range(6):
        m = k6 == k
        for c in range(3):
            out[..., c] = np.where(m, sel[k][c], out[..., c])
    out = np.where((S == 0)[..., None], V[..., None], out)
    return out.astype(np.uint8)


def hue_shift_u8(hue_factor):
    """torchvision adjust_hue's ``np.array(hue_factor * 255).astype(np.uint8)`` (negative: truncate, wrap)."""
    return int(np.array(hue_factor * 255).astype(np.int64).astype(np.uint8))


def color_jitter(img, b, c, s, h):
    """ColorJitter.__call__ (data_process.py:177-186) on a [H, W, 3] uint8 PIL-layout image."""
    img = pil_blend(np.zeros_like(img), img, b)                          # brightness
    mean = int(pil_luma(img).astype(np.int64).sum() / (img.shape[0] * img.shape[1]) + 0.5)
    img = pil_blend(np.full_like(img, mean), img, c)                     # contrast
    img = pil_blend(np.repeat(pil_luma(img)[..., None], 3, -1), img, s)  # colour (saturation)
    hsv = rgb_to_hsv(img)
    hsv[..., 0] = ((hsv[..., 0].astype(np.int64) + hue_shift_u8(h)) % 256).astype(np.uint8)
    return hsv_to_rgb(hsv)


def rotate_matrix_fixed(angle, w, h):
    """Image.rotate's inverse matrix for (angle, expand=False, centre) and ImagingTransformAffine's 16.16
    fixed-point terms (a0, a1, a2, a3, a4, a5) with the pixel-centre offsets folded into a2 / a5."""
    angle = angle % 360.0
    cx, cy = w / 2.0, h / 2.0
    r = -math.radians(angle)
    m = [round(math.cos(r), 15), round(math.sin(r), 15), 0.0, round(-math.sin(r), 15), round(math.cos(r), 15), 0.0]
    m[2], m[5] = m[0] * -cx + m[1] * -cy + m[2], m[3] * -cx + m[4] * -cy + m[5]
    m[2] += cx
    m[5] += cy
    fix = lambda v: int(math.floor(v * 65536.0 + 0.5))
    return (fix(m[0]), fix(m[1]), fix(m[2] + m[0] * 0.5 + m[1] * 0.5), fix(m[3]), fix(m[4]),
            fix(m[5] + m[3] * 0.5 + m[4] * 0.5))


def pil_rotate_nearest(img, angle):
    """Image.rotate(angle, NEAREST, expand=False) of an [H, W, C] uint8 array, fill 0."""
    h, w = img.shape[:2]
    if angle % 360.0 == 0:
        return img.copy()
    a0, a1, a2, a3, a4, a5 = rotate_matrix_fixed(angle, w, h)
    ys, xs = np.mgrid[0:h, 0:w].astype(np.int64)
    xi = (a2 + a1 * ys + a0 * xs) >> 16
    yi = (a5 + a4 * ys + a3 * xs) >> 16
    ok = (xi >= 0) & (xi < w) & (yi >= 0) & (yi < h)
    out = np.zeros_like(img)
    out[ok] = img[yi[ok], xi[ok]]
    return out


def train_image_transform(img_u8, crop_xy, jitter=None, flip=False, angle=None, size=(250, 250), crop=224,
                          mean=(0.41757566, 0.26098573, 0.25888634), std=(0.21938758, 0.1983, 0.19342837)):
    """[H, W, 3] uint8 decoded frame (or RGB segmap) -> [3, crop, crop] f32: Resize -> RandomCrop(x1, y1) ->
    [ColorJitter(b, c, s, h)] -> [flip] -> [rotate(angle)] -> ToTensor -> Normalize."""
    r = PP.pil_resize_bilinear(img_u8, size)
    x1, y1 = crop_xy
    r = r[y1:y1 + crop, x1:x1 + crop]
    if jitter is not None:
        r = color_jitter(r, *jitter)
    if flip:
        r = r[:, ::-1]
    if angle is not None:
        r = pil_rotate_nearest(np.ascontiguousarray(r), angle)
    t = torch.from_numpy(np.ascontiguousarray(r)).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    m = torch.as_tensor(mean, dtype=torch.float32)[:, None, None]
    s = torch.as_tensor(std, dtype=torch.float32)[:, None, None]
    return t.sub_(m).div_(s)


def rotate_grid_params(angle, w, h):
    """torchvision F.rotate (tensor) -> _get_inverse_affine_matrix(center 0, -angle) rescaled by (w/2, h/2):
    the f32 coefficients (t00, t01, t02, t10, t11, t12) with grid_x = x_b * t00 + y_b * t01 + t02 etc. for the base
    grid point (x_b, y_b) = (x - w/2 + 0.5, y - h/2 + 0.5)."""
    rot = math.radians(-angle)
    a, b, c, d = math.cos(rot), -math.sin(rot), math.sin(rot), math.cos(rot)
    m = [d, -b, 0.0, -c, a, 0.0]                       # inverse of [[a, b], [c, d]] (det 1), no translation
    sx, sy = 0.5 * w, 0.5 * h
    return (F32(F32(m[0]) / F32(sx)), F32(F32(m[1]) / F32(sx)), F32(F32(m[2]) / F32(sx)),
            F32(F32(m[3]) / F32(sy)), F32(F32(m[4]) / F32(sy)), F32(F32(m[5]) / F32(sy)))


def tensor_rotate_nearest(img, angle):
    """[C, H, W] f32 numpy -> rotated (nearest, zero fill): the affine grid in explicit f32 ops, then grid_sample's
    align_corners=False unnormalisation ((g + 1) * size - 1) / 2 and round-half-to-even."""
    c, h, w = img.shape
    t = rotate_grid_params(angle, w, h)
    xb = (np.arange(w, dtype=F32) - F32(w * 0.5) + F32(0.5)).astype(F32)
    yb = (np.arange(h, dtype=F32) - F32(h * 0.5) + F32(0.5)).astype(F32)
    X, Y = np.meshgrid(xb, yb)
    gx = (X * t[0] + Y * t[1]).astype(F32) + t[2]
    gy = (X * t[3] + Y * t[4]).astype(F32) + t[5]
    ix = np.rint(((gx + F32(1)) * F32(w) - F32(1)) / F32(2)).astype(np.int64)
    iy = np.rint(((gy + F32(1)) * F32(h) - F32(1)) / F32(2)).astype(np.int64)
    ok = (ix >= 0) & (ix < w) & (iy >= 0) & (iy < h)
    out = np.zeros_like(img)
    out[:, ok] = img[:, iy[ok], ix[ok]]
    return out


def train_flow_transform(flow, crop_xy, flip=False, angle=None, size=(250, 250), crop=224):
    """[H, W, 2] f32 RAFT field -> [2, crop, crop] f32: CholecFlowDataset's cv2 resize + displacement rescale,
    then RandomCrop(x1, y1) -> [flip: u negated] -> [rotate(angle) + vector rotation]."""
    H, W, _ = flow.shape
    r = PP.cv2_resize_linear(flow.astype(F32), size)
    r[:, :, 0] *= size[1] / W
    r[:, :, 1] *= size[0] / H
    x1, y1 = crop_xy
    t = np.ascontiguousarray(r[y1:y1 + crop, x1:x1 + crop].transpose(2, 0, 1))
    if flip:
        t = np.ascontiguousarray(t[:, :, ::-1])
        t[0] = -t[0]
    if angle is not None:
        t = tensor_rotate_nearest(t, angle)
        rad = math.radians(angle)
        ca, sa = F32(math.cos(rad)), F32(math.sin(rad))
        u, v = t[0].copy(), t[1].copy()
        t[0] = u * ca - v * sa
        t[1] = u * sa + v * ca
    return torch.from_numpy(np.ascontiguousarray(t))
