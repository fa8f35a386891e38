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
