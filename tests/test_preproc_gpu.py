"""svk_frame_preproc (generate_evp_LFB.py:243-247 transform on the GPU) against Pillow + torch's CPU ops —
the reference DataLoader's own pipeline — bit-exact (torch.equal on the f32 tensors)."""
import numpy as np
import pytest
import torch
from PIL import Image

from oracle import preproc as OP

pytestmark = pytest.mark.gpu


def _frames(B, h, w, seed, mask=False):
    r = np.random.default_rng(seed)
    if not mask:
        return r.integers(0, 256, size=(B, h, w, 3), dtype=np.uint8)
    yy, xx = np.mgrid[0:h, 0:w]                          # binary ellipse masks replicated to RGB (segmaps)
    out = np.zeros((B, h, w, 3), np.uint8)
    for b in range(B):
        cy, cx, ry, rx = r.uniform(0.2, 0.8) * h, r.uniform(0.2, 0.8) * w, r.uniform(0.1, 0.4) * h, r.uniform(0.1, 0.4) * w
        out[b][((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1] = 255
    return out


def _reference(frames):
    """Resize((250, 250)) -> CenterCrop(224) -> ToTensor -> Normalize exactly as the reference's workers do
    it, with Pillow doing the resize (torchvision's PIL path) and torch's CPU ops the rest."""
    mean = torch.tensor(OP.frame_transform.__defaults__[2], dtype=torch.float32)[:, None, None]
    std = torch.tensor(OP.frame_transform.__defaults__[3], dtype=torch.float32)[:, None, None]
    outs = []
    for f in frames:
        pil = Image.fromarray(f, "RGB").resize((250, 250), Image.BILINEAR).crop((13, 13, 237, 237))
        t = torch.from_numpy(np.asarray(pil).copy()).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
        outs.append(t.sub_(mean).div_(std))
    return torch.stack(outs)


@pytest.mark.parametrize("hw", [(480, 854), (250, 250), (200, 300), (251, 249), (1080, 1920)])
def test_frame_transform_bit_exact(cuda, hw):
    from svk.preproc import frame_transform
    fr = _frames(3, *hw, seed=hw[0])
    out = frame_transform(torch.from_numpy(fr).to(cuda))
    torch.cuda.synchronize()
    assert out.shape == (3, 3, 224, 224)
    ref = _reference(fr)
    assert torch.equal(out.cpu(), ref), float((out.cpu() - ref).abs().max())


def test_segmap_transform_bit_exact(cuda):
    from svk.preproc import frame_transform
    fr = _frames(4, 480, 854, 7, mask=True)
    out = frame_transform(torch.from_numpy(fr).to(cuda))
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), _reference(fr))


def test_frame_transform_feeds_the_extractor(cuda):
    """The preprocessed batch is what MixVisionTransformerEVP.forward consumes ([B, 1, 3, 224, 224])."""
    from svk.preproc import frame_transform
    fr = torch.from_numpy(_frames(2, 480, 854, 3)).to(cuda)
    x = frame_transform(fr).view(2, 1, 3, 224, 224)
    assert x.is_contiguous() and torch.isfinite(x).all()


def test_frame_transform_rejects_bad_input(cuda):
    import svk
    from svk.preproc import frame_transform
    with pytest.raises(svk.SvkError):
        frame_transform(torch.zeros(1, 100, 100, 4, dtype=torch.uint8, device=cuda))
    with pytest.raises(svk.SvkError):
        frame_transform(torch.zeros(1, 100, 100, 3, dtype=torch.float32, device=cuda))
    with pytest.raises(svk.SvkError):
        frame_transform(torch.zeros(1, 100, 100, 3, dtype=torch.uint8, device=cuda), size=(200, 200), crop=224)


@pytest.mark.parametrize("hw", [(480, 854), (250, 250), (200, 300)])
def test_flow_transform_vs_oracle(cuda, hw):
    """GPU flow transform vs the cv2 INTER_LINEAR restatement (both f32 multiply + add, no FMA): bit-exact.
    Parity against cv2 itself is unpinned (cv2 absent here; see oracle/preproc.py)."""
    from svk.preproc import flow_transform
    fl = (np.random.default_rng(hw[1]).standard_normal((2, *hw, 2)) * 2.0).astype(np.float32)   # N(0, 2 px)
    out = flow_transform(torch.from_numpy(fl).to(cuda))
    torch.cuda.synchronize()
    ref = torch.stack([OP.flow_transform(f) for f in fl])
    assert out.shape == (2, 2, 224, 224)
    assert torch.equal(out.cpu(), ref), float((out.cpu() - ref).abs().max())
