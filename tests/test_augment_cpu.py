"""The training-augmentation oracle (oracle/augment.py) pinned against Pillow 12.2.0 itself (bit-exact), and its
flow-tensor path against the drop-in host transforms (models/data_process.py, torch grid_sample)."""
import math
import os
import sys

import numpy as np
import pytest
import torch
from PIL import Image, ImageEnhance

from oracle import augment as AU, preproc as PP

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "deep-learning-for-surgical-video-analysis_amd"))


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)


def test_luma_and_hsv_exhaustive_subset():
    """convert("L"), convert("HSV") and HSV -> RGB over every 16th of all 2^24 triples (the oracle was checked
    on all of them when it was written)."""
    v = np.arange(0, 1 << 24, 16, dtype=np.uint32)
    trip = np.stack([(v >> 16) & 255, (v >> 8) & 255, v & 255], -1).astype(np.uint8).reshape(1024, 1024, 3)
    im = Image.fromarray(trip)
    assert np.array_equal(AU.pil_luma(trip), np.array(im.convert("L")))
    assert np.array_equal(AU.rgb_to_hsv(trip), np.array(im.convert("HSV")))
    assert np.array_equal(AU.hsv_to_rgb(trip), np.array(Image.fromarray(trip, "HSV").convert("RGB")))


@pytest.mark.parametrize("seed", range(6))
def test_color_jitter_vs_pillow(seed):
    """ColorJitter's four PIL steps (ImageEnhance Brightness / Contrast / Color, torchvision's HSV hue shift) at
    the factors data_process.py draws (incl. the extremes and a negative hue)."""
    rng = np.random.default_rng(100 + seed)
    img = _img(224, 224, seed)
    b, c, s = (float(rng.uniform(0.9, 1.1)) for _ in range(3))
    h = float(rng.uniform(-0.05, 0.05)) if seed < 4 else (-0.05, 0.05)[seed - 4]
    im = ImageEnhance.Brightness(Image.fromarray(img)).enhance(b)
    im = ImageEnhance.Contrast(im).enhance(c)
    im = ImageEnhance.Color(im).enhance(s)
    hh, ss, vv = im.convert("HSV").split()
    nh = np.array(hh, dtype=np.uint8)
    nh += np.array(h * 255).astype(np.uint8)
    ref = np.array(Image.merge("HSV", (Image.fromarray(nh, "L"), ss, vv)).convert("RGB"))
    assert np.array_equal(AU.color_jitter(img, b, c, s, h), ref)


@pytest.mark.parametrize("hw", [(224, 224), (250, 250), (37, 53)])
def test_rotate_nearest_vs_pillow(hw):
    img = _img(*hw, 7)
    for ang in range(-5, 6):
        ref = np.array(Image.fromarray(img).rotate(ang, resample=Image.NEAREST, expand=False))
        assert np.array_equal(AU.pil_rotate_nearest(img, ang), ref), ang


@pytest.mark.parametrize("shape,jit,flip,ang", [((480, 854), True, True, -5), ((480, 854), True, False, 3),
                                                ((250, 250), False, True, None), ((300, 400), True, True, 0)])
def test_train_image_transform_vs_pillow_chain(shape, jit, flip, ang):
    """The whole use_flip == 1 / 0 image transform against the PIL chain it stands for."""
    img = _img(*shape, 11)
    x1, y1 = 17, 5
    jitter = (1.07, 0.93, 1.02, -0.031) if jit else None
    got = AU.train_image_transform(img, (x1, y1), jitter, flip, ang)
    im = Image.fromarray(img).resize((250, 250), Image.BILINEAR).crop((x1, y1, x1 + 224, y1 + 224))
    if jit:
        im = ImageEnhance.Color(ImageEnhance.Contrast(ImageEnhance.Brightness(im).enhance(1.07)).enhance(0.93)).enhance(1.02)
        hh, ss, vv = im.convert("HSV").split()
        nh = np.array(hh, dtype=np.uint8)
        nh += np.array(-0.031 * 255).astype(np.uint8)
        im = Image.merge("HSV", (Image.fromarray(nh, "L"), ss, vv)).convert("RGB")
    if flip:
        im = im.transpose(Image.FLIP_LEFT_RIGHT)
    if ang is not None:
        im = im.rotate(ang, resample=Image.NEAREST, expand=False)
    t = torch.from_numpy(np.array(im)).permute(2, 0, 1).float().div(255)
    ref = t.sub_(torch.tensor(PP_MEAN)[:, None, None]).div_(torch.tensor(PP_STD)[:, None, None])
    assert torch.equal(got, ref)


PP_MEAN = (0.41757566, 0.26098573, 0.25888634)
PP_STD = (0.21938758, 0.1983, 0.19342837)


@pytest.mark.parametrize("ang", [-5, -2, 0, 1, 4])
def test_tensor_rotate_matches_host_grid_sample(ang):
    """The oracle's explicit-f32 affine grid + nearest sampling == the drop-in host transform
    (models/data_process.py: torch affine grid @ theta + F.grid_sample nearest) on a flow-shaped tensor."""
    from models.data_process import _rotate_tensor_nearest
    t = torch.randn(2, 224, 224, generator=torch.Generator().manual_seed(ang + 10))
    got = AU.tensor_rotate_nearest(t.numpy(), ang)
    ref = _rotate_tensor_nearest(t.clone(), ang).numpy()
    diff = (got != ref).any(0).mean()
    assert diff == 0.0, f"{diff:.2e} of the pixels sample a different source"


def test_train_flow_transform_matches_host_classes():
    """The flow path (cv2 resize + rescale, crop, flip with u negated, rotation + vector rotation) == the drop-in
    RandomCrop / RandomHorizontalFlip / RandomRotation applied to the same tensor with the same draws."""
    import random
    from models import data_process as DP
    flow = np.random.default_rng(3).normal(size=(480, 854, 2)).astype(np.float32) * 4
    r = PP.cv2_resize_linear(flow, (250, 250))
    r[:, :, 0] *= 250 / 854
    r[:, :, 1] *= 250 / 480
    t = torch.from_numpy(np.ascontiguousarray(r.transpose(2, 0, 1)))
    crop, fl, rot = DP.RandomCrop(224), DP.RandomHorizontalFlip(), DP.RandomRotation(5)
    for c in range(0, 95, 31):                  # four clips: different draws
        crop.count = fl.count = rot.count = c
        random.seed(c // 30)
        x1, y1 = random.randint(0, 26), random.randint(0, 26)
        random.seed(c // 30)
        do_flip = random.random() < 0.5
        random.seed(c // 30)
        ang = random.randint(-5, 5)
        ref = rot(fl(crop(t.clone())))
        got = AU.train_flow_transform(flow, (x1, y1), do_flip, ang)
        torch.testing.assert_close(got, ref, rtol=0, atol=0)


def test_train_augment_rejects_bad_params():
    """the GPU passes trust the per-sample parameters, so TrainAugment validates them on the host —
    crop offsets inside the 250 x 250 resized image, 0 / 1 flags — and refuses a padded RandomCrop it does not
    implement."""
    from models import data_process as DP
    from svk import SvkError
    from svk.augment import TrainAugment, NP
    ta = TrainAugment()
    ok = torch.zeros(2, NP, dtype=torch.int32)
    ok[:, 0], ok[:, 1] = 26, 3
    ta._check_params(ok, flow=False)
    ta._check_params(ok, flow=True)
    for col, v in ((0, 27), (1, -1), (2, 2), (3, 5), (10, 3)):
        bad = ok.clone()
        bad[1, col] = v
        with pytest.raises(SvkError):
            ta._check_params(bad, flow=False)
    with pytest.raises(SvkError):
        TrainAugment(transforms=(DP.RandomCrop(224, padding=4), None, DP.RandomHorizontalFlip(), None))
