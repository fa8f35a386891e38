"""Frame preprocessing oracle (oracle/preproc.py) pinned against Pillow itself (the reference's resize
implementation; bit-exact), and the product's host-side coefficient builder (svk/preproc.py) against it."""
import numpy as np
import pytest
import torch
from PIL import Image

from oracle import preproc as OP

SIZES = [(480, 854), (250, 250), (200, 300), (251, 249), (90, 120), (1080, 1920)]


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, size=(h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("hw", SIZES)
def test_resize_matches_pillow(hw):
    img = _img(*hw, seed=hw[0] + hw[1])
    ref = np.asarray(Image.fromarray(img, "RGB").resize((250, 250), Image.BILINEAR))
    np.testing.assert_array_equal(OP.pil_resize_bilinear(img, (250, 250)), ref)


def test_transform_matches_pillow_and_torch_ops():
    img = _img(480, 854, 1)
    pil = Image.fromarray(img, "RGB").resize((250, 250), Image.BILINEAR).crop((13, 13, 237, 237))
    t = torch.from_numpy(np.asarray(pil).copy()).permute(2, 0, 1).contiguous().float().div(255)
    t = t.sub_(torch.tensor(OP.frame_transform.__defaults__[2])[:, None, None]).div_(
        torch.tensor(OP.frame_transform.__defaults__[3])[:, None, None])
    assert torch.equal(OP.frame_transform(img), t)


@pytest.mark.parametrize("n_in,n_out", [(854, 250), (480, 250), (250, 250), (200, 250), (1920, 250)])
def test_host_coefficients_match_oracle(n_in, n_out):
    from svk.preproc import pillow_bilinear_coeffs
    b, c, k = pillow_bilinear_coeffs(n_in, n_out)
    idx, kk = OP._axis(n_in, n_out)
    assert c.shape == kk.shape
    np.testing.assert_array_equal(c, kk)
    np.testing.assert_array_equal(b[:, 0], idx[:, 0])


def test_flow_oracle_identity_size_is_a_crop():
    f = np.random.default_rng(0).standard_normal((250, 250, 2)).astype(np.float32)
    out = OP.flow_transform(f)
    assert torch.equal(out, torch.from_numpy(f[13:237, 13:237].copy()).permute(2, 0, 1))


def test_flow_oracle_constant_and_ramp():
    const = np.empty((480, 854, 2), np.float32)
    const[..., 0], const[..., 1] = 3.0, -2.0
    out = OP.flow_transform(const)
    assert torch.allclose(out[0], torch.tensor(3.0 * 250 / 854)) and torch.allclose(out[1], torch.tensor(-2.0 * 250 / 480))
    # a linear ramp along x is reproduced by bilinear interpolation at the half-pixel-centred sample points
    W = 500
    ramp = np.broadcast_to(np.arange(W, dtype=np.float32)[None, :, None], (100, W, 2)).copy()
    r = OP.cv2_resize_linear(ramp, (250, 250))
    expect = (np.arange(250) + 0.5) * (W / 250) - 0.5
    np.testing.assert_allclose(r[0, :, 0], np.clip(expect, 0, W - 1), rtol=0, atol=1e-4)


def test_host_cv2_tables_match_oracle():
    from svk.preproc import cv2_linear_table
    for n_in in (854, 480, 250, 200):
        o, a = cv2_linear_table(n_in, 250)
        i0, _, w = OP._cv_axis(n_in, 250)
        np.testing.assert_array_equal(o, i0)
        np.testing.assert_array_equal(a, w)
