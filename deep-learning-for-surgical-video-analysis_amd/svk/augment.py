"""GPU training augmentations: train_evp.py:146-163's ``train_transforms`` as CholecFlowDataset applies them
(data_process.py:455-487) — to the decoded RGB frame, to the RGB segmap, and (geometric steps only) to the RAFT
flow — on a whole batch at once.

The random draws stay exactly the reference's: the drop-in classes of ``models.data_process`` (RandomCrop,
ColorJitter, RandomHorizontalFlip, RandomRotation — each reseeding Python's ``random`` with ``count // 30``) are
asked for their parameters in the order CholecFlowDataset.__getitem__ calls them, sample by sample (frame: crop,
[jitter], flip, [rotation]; segmap: the same; flow: crop, flip, [rotation]), i.e. the single-process
(``num_workers=0``) DataLoader semantics.  The pixel work runs in ``svk_train_augment`` /
``svk_train_augment_flow``: bit-exact to Pillow 12.2.0 for the images (tests/test_augment_gpu.py against
oracle/augment.py, which tests/test_augment_cpu.py pins against Pillow itself); the flow path follows
torchvision's tensor ops (absent in this image: parity vs the restatement only).

Host-side parameter math (per sample, tiny): Image.rotate's inverse matrix in ImagingTransformAffine's 16.16 fixed
point, torchvision's rescaled inverse affine grid for the tensor rotation, the ColorJitter factors as f32 bits and
adjust_hue's ``np.uint8(hue * 255)`` shift.
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib
from .ops import _chk, _p, _prof_begin, _prof_end, _stream
from .preproc import CHOLEC80_MEAN, CHOLEC80_STD, _coeffs, _CV_CACHE, cv2_linear_table

NP = 16          # int32 parameters per sample (include/svk.h)


def _f32_bits(v):
    return int(np.array(v, dtype=np.float32).view(np.int32))


def rotate_fixed(angle, w, h):
    """Image.rotate(angle, expand=False) inverse matrix -> ImagingTransformAffine's nearest-path 16.16 terms."""
    angle = angle % 360.0
    cx, cy = w / 2.0, h / 2.0
    r = -math.radians(angle)
    m = [round(math.cos(r), 15), round(math.sin(r), 15), 0.0, round(-math.sin(r), 15), round(math.cos(r), 15), 0.0]
    m[2], m[5] = m[0] * -cx + m[1] * -cy + m[2] + cx, m[3] * -cx + m[4] * -cy + m[5] + cy
    fix = lambda v: int(math.floor(v * 65536.0 + 0.5))
    return [fix(m[0]), fix(m[1]), fix(m[2] + m[0] * 0.5 + m[1] * 0.5), fix(m[3]), fix(m[4]),
            fix(m[5] + m[3] * 0.5 + m[4] * 0.5)]


def tensor_rotate_grid(angle, w, h):
    """torchvision's tensor rotate: _get_inverse_affine_matrix(centre 0, -angle) divided by (w/2, h/2), f32."""
    rot = math.radians(-angle)
    a, b, c, d = math.cos(rot), -math.sin(rot), math.sin(rot), math.cos(rot)
    m = [d, -b, 0.0, -c, a, 0.0]
    f = np.float32
    sx, sy = f(0.5 * w), f(0.5 * h)
    return [f(f(m[0]) / sx), f(f(m[1]) / sx), f(f(m[2]) / sx), f(f(m[3]) / sy), f(f(m[4]) / sy), f(f(m[5]) / sy)]


class TrainAugment:
    """The batch twin of ``transforms.Compose([Resize((250, 250)), RandomCrop(224), [ColorJitter(0.1, 0.1, 0.1,
    0.05)], RandomHorizontalFlip(), [RandomRotation(5)], ToTensor(), Normalize(mean, std)])`` (train_evp.py:146-163;
    ``use_flip`` selects the bracketed steps as the script's flag does).  ``crop``, ``flip``, ``rotation``,
    ``jitter`` are the drop-in synced transform objects; pass your own to continue their counts."""

    def __init__(self, use_flip=1, size=(250, 250), crop=224, mean=CHOLEC80_MEAN, std=CHOLEC80_STD, transforms=None):
        from models.data_process import RandomCrop, RandomHorizontalFlip, RandomRotation, ColorJitter
        self.size, self.crop_size, self.mean, self.std = tuple(size), int(crop), tuple(mean), tuple(std)
        if transforms is None:
            transforms = (RandomCrop(crop), ColorJitter(0.1, 0.1, 0.1, 0.05) if use_flip else None,
                          RandomHorizontalFlip(), RandomRotation(5) if use_flip else None)
        self.crop, self.jitter, self.flip, self.rotation = transforms
        if getattr(self.crop, "padding", 0):
            # the GPU pass crops the resized image itself (train_evp.py:146-163 uses RandomCrop(224), no padding)
            raise _lib.SvkError("svk.augment: RandomCrop(padding > 0) is not implemented by the GPU pass")
        self._ws = {}

    # ---- parameter draws, in CholecFlowDataset.__getitem__'s order ---------------------------------------
    def _image_params(self):
        OH, OW = self.size
        xy = self.crop.draw(OW, OH)
        x1, y1 = xy if xy is not None else (0, 0)
        row = [x1, y1, 0, 0, 65536, 0, 0, 0, 65536, 0, 0, 0, 0, 0, 0, 0]
        if self.jitter is not None:
            b, c, s, h = self.jitter.factors()
            row[10:15] = [1, _f32_bits(b), _f32_bits(c), _f32_bits(s),
                          int(np.array(h * 255).astype(np.int64).astype(np.uint8))]
        row[2] = int(self.flip.draw())
        if self.rotation is not None:
            ang = self.rotation.draw()
            if ang % 360 != 0:
                row[3] = 1
                row[4:10] = rotate_fixed(ang, self.crop_size, self.crop_size)
        return row

    def _flow_params(self):
        OH, OW = self.size
        xy = self.crop.draw(OW, OH)
        x1, y1 = xy if xy is not None else (0, 0)
        row = [x1, y1, int(self.flip.draw())] + [0] * 13
        if self.rotation is not None:
            ang = self.rotation.draw()
            if ang % 360 != 0:
                row[3] = 1
                row[4:10] = [_f32_bits(v) for v in tensor_rotate_grid(ang, self.crop_size, self.crop_size)]
                rad = math.radians(ang)
                row[10:12] = [_f32_bits(math.cos(rad)), _f32_bits(math.sin(rad))]
        return row

    def draw(self, n, with_segmaps=True, with_flow=True):
        """Parameters of n samples: (frames [n, 16], segmaps [n, 16], flows [n, 16]) int32."""
        img, seg, fl = [], [], []
        for _ in range(n):
            img.append(self._image_params())
            if with_segmaps:
                seg.append(self._image_params())
            if with_flow:
                fl.append(self._flow_params())
        t = lambda rows: torch.tensor(rows, dtype=torch.int32) if rows else None
        return t(img), t(seg), t(fl)

    def _check_params(self, prm, flow):
        """Host-side validation of per-sample parameters (the kernels trust them): crop offsets inside the resized
        image, flag fields 0 / 1.  A device tensor is copied to the host for the check."""
        OH, OW = self.size
        C = self.crop_size
        q = prm.cpu() if prm.is_cuda else prm
        if q.numel() == 0:
            return
        x1, y1 = q[:, 0], q[:, 1]
        if bool(((x1 < 0) | (x1 > OW - C) | (y1 < 0) | (y1 > OH - C)).any()):
            raise _lib.SvkError(f"svk.augment: crop offsets must lie in [0, {OW - C}] x [0, {OH - C}]")
        flags = (2, 3) if flow else (2, 3, 10)
        if bool(((q[:, list(flags)] != 0) & (q[:, list(flags)] != 1)).any()):
            raise _lib.SvkError("svk.augment: flip / rotation / jitter flags must be 0 or 1")

    # ---- GPU passes ---------------------------------------------------------------------------------------
    def images(self, frames, params, out=None):
        """frames [B, H, W, 3] uint8 (GPU), params [B, 16] int32 -> [B, 3, 224, 224] f32."""
        _chk(frames, "frames", torch.uint8)
        if frames.dim() != 4 or frames.shape[-1] != 3 or not frames.is_contiguous():
            raise _lib.SvkError(f"svk.augment: frames must be contiguous [B, H, W, 3] uint8, got {tuple(frames.shape)}")
        B, H, W, _ = frames.shape
        OH, OW = self.size
        C = self.crop_size
        prm = params.to(frames.device, torch.int32).contiguous()
        if tuple(prm.shape) != (B, NP):
            raise _lib.SvkError(f"svk.augment: params must be [{B}, {NP}] int32")
        self._check_params(params, flow=False)
        xb, xk, ksx = _coeffs(W, OW, frames.device)
        yb, yk, ksy = _coeffs(H, OH, frames.device)
        key = (B, H, frames.device)
        if key not in self._ws:
            self._ws[key] = (torch.empty(B, H, C, 3, device=frames.device, dtype=torch.uint8),
                             torch.empty(B, C, C, 3, device=frames.device, dtype=torch.uint8),
                             torch.empty(B, device=frames.device, dtype=torch.int64))
        tmp, crop, sums = self._ws[key]
        if out is None:
            out = torch.empty(B, 3, C, C, device=frames.device, dtype=torch.float32)
        m, sd = (ctypes.c_float * 3)(*self.mean), (ctypes.c_float * 3)(*self.std)
        t0 = _prof_begin()
        _lib.call("svk_train_augment", _p(frames), _p(tmp), _p(crop), _p(sums), _p(out), _p(xb), _p(xk), ksx, _p(yb),
                  _p(yk), ksy, _p(prm), B, H, W, OH, OW, C, C, ctypes.addressof(m), ctypes.addressof(sd), _stream())
        # algorithmic bytes: the decoded frames in, the f32 tensor out (the uint8 crop round trips are extra)
        _prof_end(t0, "train_augment", 0, B * (H * W * 3 + 3 * C * C * 4), (B, H, W))
        return out

    def flows(self, flow, params, out=None):
        """flow [B, H, W, 2] f32 (GPU, raw RAFT fields), params [B, 16] -> [B, 2, 224, 224] f32."""
        _chk(flow, "flow", torch.float32)
        if flow.dim() != 4 or flow.shape[-1] != 2 or not flow.is_contiguous():
            raise _lib.SvkError(f"svk.augment: flow must be contiguous [B, H, W, 2] f32, got {tuple(flow.shape)}")
        B, H, W, _ = flow.shape
        OH, OW = self.size
        C = self.crop_size
        prm = params.to(flow.device, torch.int32).contiguous()
        if tuple(prm.shape) != (B, NP):
            raise _lib.SvkError(f"svk.augment: params must be [{B}, {NP}] int32")
        self._check_params(params, flow=True)
        key = (H, W, OH, OW, flow.device)
        if key not in _CV_CACHE:
            xo, xa = cv2_linear_table(W, OW)
            yo, ya = cv2_linear_table(H, OH)
            _CV_CACHE[key] = tuple(torch.from_numpy(a).to(flow.device) for a in (xo, xa, yo, ya))
        xo, xa, yo, ya = _CV_CACHE[key]
        if out is None:
            out = torch.empty(B, 2, C, C, device=flow.device, dtype=torch.float32)
        su, sv = float(np.float32(OW / W)), float(np.float32(OH / H))
        t0 = _prof_begin()
        _lib.call("svk_train_augment_flow", _p(flow), _p(out), _p(xo), _p(xa), _p(yo), _p(ya), _p(prm), B, H, W, C, C,
                  su, sv, _stream())
        _prof_end(t0, "train_augment_flow", 0, B * (H * W * 8 + 2 * C * C * 4), (B, H, W))
        return out

    def __call__(self, frames, segmaps=None, flow=None):
        """One training batch: draws every sample's parameters (reference order), then the GPU passes ->
        (frames [B, 3, 224, 224], segmaps or None, flow [B, 2, 224, 224] or None)."""
        pi, ps, pf = self.draw(frames.shape[0], segmaps is not None, flow is not None)
        return (self.images(frames, pi), None if segmaps is None else self.images(segmaps, ps),
                None if flow is None else self.flows(flow, pf))
