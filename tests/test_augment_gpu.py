"""GPU training augmentations (svk.augment, svk_train_augment / svk_train_augment_flow) against the oracle
(oracle/augment.py, pinned to Pillow by tests/test_augment_cpu.py) — bit-exact — and end to end against the
drop-in host transforms run on Pillow itself with the same synced draws."""
import numpy as np
import pytest
import torch
from PIL import Image

from oracle import augment as AU

pytestmark = pytest.mark.gpu

MEAN = (0.41757566, 0.26098573, 0.25888634)
STD = (0.21938758, 0.1983, 0.19342837)


def _frames(B, H, W, seed):
    return np.random.default_rng(seed).integers(0, 256, (B, H, W, 3), dtype=np.uint8)


@pytest.mark.parametrize("H,W", [(480, 854), (250, 250), (300, 404)])
def test_train_images_vs_oracle(cuda, H, W):
    """Per-sample crops, jitter factors (incl. the range ends and negative hue), flips and angles -5..5."""
    from svk.augment import TrainAugment, rotate_fixed, _f32_bits
    B = 11
    fr = _frames(B, H, W, 5)
    rng = np.random.default_rng(6)
    aug = TrainAugment()
    rows, expect = [], []
    for i in range(B):
        x1, y1 = int(rng.integers(0, 27)), int(rng.integers(0, 27))
        jit = None if i % 4 == 3 else tuple(float(v) for v in (rng.uniform(0.9, 1.1), rng.uniform(0.9, 1.1),
                                                                  rng.uniform(0.9, 1.1), rng.uniform(-0.05, 0.05)))
        if i == 0:
            jit = (0.9, 1.1, 0.9, -0.05)
        flip = bool(i % 2)
        ang = i - 5
        row = [x1, y1, int(flip), int(ang != 0)] + (rotate_fixed(ang, 224, 224) if ang else [65536, 0, 0, 0, 65536, 0])
        row += ([1, _f32_bits(jit[0]), _f32_bits(jit[1]), _f32_bits(jit[2]),
                 int(np.array(jit[3] * 255).astype(np.int64).astype(np.uint8))] if jit else [0] * 5) + [0]
        rows.append(row)
        expect.append(AU.train_image_transform(fr[i], (x1, y1), jit, flip, ang if ang else None))
    got = aug.images(torch.from_numpy(fr).to(cuda), torch.tensor(rows, dtype=torch.int32))
    torch.cuda.synchronize()
    for i in range(B):
        assert torch.equal(got[i].cpu(), expect[i]), f"sample {i}: {(got[i].cpu() != expect[i]).sum().item()} values differ"


def test_train_flows_vs_oracle(cuda):
    from svk.augment import TrainAugment, tensor_rotate_grid, _f32_bits
    import math
    B, H, W = 9, 480, 854
    fl = (np.random.default_rng(8).normal(size=(B, H, W, 2)) * 5).astype(np.float32)
    rng = np.random.default_rng(9)
    rows, expect = [], []
    for i in range(B):
        x1, y1, flip, ang = int(rng.integers(0, 27)), int(rng.integers(0, 27)), bool(i % 2), i - 4
        row = [x1, y1, int(flip), int(ang != 0)]
        row += [_f32_bits(v) for v in tensor_rotate_grid(ang, 224, 224)] if ang else [0] * 6
        row += [_f32_bits(math.cos(math.radians(ang))), _f32_bits(math.sin(math.radians(ang)))] + [0] * 4
        rows.append(row)
        expect.append(AU.train_flow_transform(fl[i], (x1, y1), flip, ang if ang else None))
    got = TrainAugment().flows(torch.from_numpy(fl).to(cuda), torch.tensor(rows, dtype=torch.int32))
    torch.cuda.synchronize()
    for i in range(B):
        torch.testing.assert_close(got[i].cpu(), expect[i], rtol=0, atol=0)


@pytest.mark.parametrize("use_flip", [1, 0])
def test_train_augment_end_to_end_vs_host_pillow(cuda, use_flip):
    """TrainAugment(frames, segmaps, flow) == the drop-in classes of models/data_process.py applied per sample
    in CholecFlowDataset.__getitem__'s order on PIL images (Pillow does the pixel work) and on the flow tensor,
    both sides starting from the same counts (clip boundaries inside the batch: counts 25.. cross 30 and 60)."""
    import random
    from models import data_process as DP
    from oracle import preproc as PP
    from svk.augment import TrainAugment
    B, H, W = 12, 480, 854
    fr, sg = _frames(B, H, W, 21), _frames(B, H, W, 22)
    fl = (np.random.default_rng(23).normal(size=(B, H, W, 2)) * 3).astype(np.float32)

    def objs():
        t = (DP.RandomCrop(224), DP.ColorJitter(0.1, 0.1, 0.1, 0.05) if use_flip else None, DP.RandomHorizontalFlip(),
             DP.RandomRotation(5) if use_flip else None)
        for o in t:
            if o is not None:
                o.count = 25
        return t

    aug = TrainAugment(use_flip, transforms=objs())
    gi, gs, gf = aug(torch.from_numpy(fr).to(cuda), torch.from_numpy(sg).to(cuda), torch.from_numpy(fl).to(cuda))
    torch.cuda.synchronize()
    crop, jit, flip, rot = objs()
    pipe = [t for t in (crop, jit, flip, rot) if t is not None]
    m, s = torch.tensor(MEAN)[:, None, None], torch.tensor(STD)[:, None, None]

    def pil_path(img):
        im = Image.fromarray(img).resize((250, 250), Image.BILINEAR)
        for t in pipe:
            im = t(im)
        return torch.from_numpy(np.array(im)).permute(2, 0, 1).float().div(255).sub_(m).div_(s)

    for i in range(B):
        ri, rs = pil_path(fr[i]), pil_path(sg[i])
        r = PP.cv2_resize_linear(fl[i], (250, 250))
        r[:, :, 0] *= 250 / W
        r[:, :, 1] *= 250 / H
        t = torch.from_numpy(np.ascontiguousarray(r.transpose(2, 0, 1)))
        for tr in (crop, flip, rot):
            if tr is not None:
                t = tr(t)
        assert torch.equal(gi[i].cpu(), ri), f"frame {i}"
        assert torch.equal(gs[i].cpu(), rs), f"segmap {i}"
        torch.testing.assert_close(gf[i].cpu(), t, rtol=0, atol=0)
    assert aug.crop.count == crop.count and aug.flip.count == flip.count
