"""Diagnostics for svk_train_augment: per-stage mismatch counts against oracle/augment.py (GPU box)."""
import os
import sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "deep-learning-for-surgical-video-analysis_amd"), REPO]
from oracle import augment as AU, preproc as PP
from svk.augment import TrainAugment, rotate_fixed, _f32_bits

dev = torch.device("cuda:0")
H, W = 480, 854
fr = np.random.default_rng(5).integers(0, 256, (1, H, W, 3), dtype=np.uint8)
aug = TrainAugment()
x1, y1 = 7, 13
r = PP.pil_resize_bilinear(fr[0], (250, 250))[y1:y1 + 224, x1:x1 + 224]
for name, jit, flip, ang in [("crop", None, False, None), ("flip", None, True, None), ("rot-5", None, False, -5),
                             ("rot3", None, False, 3), ("bright", (0.9, 1.0, 1.0, 0.0), False, None),
                             ("contrast", (1.0, 1.1, 1.0, 0.0), False, None), ("color", (1.0, 1.0, 0.9, 0.0), False, None),
                             ("hue", (1.0, 1.0, 1.0, -0.05), False, None), ("all", (0.9, 1.1, 0.9, -0.05), True, -5)]:
    row = [x1, y1, int(flip), int(ang is not None)] + (rotate_fixed(ang, 224, 224) if ang else [65536, 0, 0, 0, 65536, 0])
    row += ([1, _f32_bits(jit[0]), _f32_bits(jit[1]), _f32_bits(jit[2]),
             int(np.array(jit[3] * 255).astype(np.int64).astype(np.uint8))] if jit else [0] * 5) + [0]
    got = aug.images(torch.from_numpy(fr).to(dev), torch.tensor([row], dtype=torch.int32))
    torch.cuda.synchronize()
    crop = aug._ws[(1, H, dev)][1].cpu().numpy()[0]
    tmp = aug._ws[(1, H, dev)][0].cpu().numpy()[0]                      # horizontal pass [H, 224, 3]
    xi, xk = PP._axis(W, 250)
    href = PP._pass(fr[0].astype(np.int64), xi, xk, 1)[:, x1:x1 + 224]
    if name == "crop":
        hb = np.nonzero(tmp != href)
        print("h-pass mismatches:", len(hb[0]), list(zip(*[h[:6] for h in hb])))
    ref = AU.train_image_transform(fr[0], (x1, y1), jit, flip, ang)
    d = (got[0].cpu() != ref)
    print(f"{name:9s} crop-mismatch {(crop != r).sum():6d}  out-mismatch {int(d.sum()):6d}  "
          f"max|d| {float((got[0].cpu() - ref).abs().max()):.4f}", flush=True)
    if name == "crop" and (crop != r).any():
        yy, xx, cc = np.nonzero(crop != r)
        print("first crop diffs:", list(zip(yy[:5], xx[:5], cc[:5])), crop[yy[0], xx[0]], r[yy[0], xx[0]])
