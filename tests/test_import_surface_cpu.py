"""The drop-in import surface: every name the reference's callers import from the
``models`` package and the top-level helper modules resolves from this build (written as a name list,
not as script text), plus the host-side semantics of the data-pipeline pieces that run without a GPU:
synced augmentations, the datasets' item contracts and CholecFlowDataset's cv2-equivalent flow resize."""
import importlib
import os

import numpy as np
import pytest
import torch
from PIL import Image

# (module, names) exactly as the reference scripts import them
IMPORTS = [
    # generate_evp_LFB.py:21, 23
    ("models.mix_transformer_evp", ["mit_b2_evp", "mit_b5_evp", "mit_b3_evp", "mit_b4_evp", "mit_b1_evp"]),
    ("models.data_process", ["CholecSegmapDataset", "M2caiSegmapDataset", "RandomCrop", "RandomHorizontalFlip",
                             "RandomRotation", "ColorJitter", "CholecDataset", "SeqSampler", "get_useful_start_idx",
                             "get_useful_start_idx_LFB", "CholecFlowDataset"]),
    # train_evp.py:18-20
    ("models.mix_transformer_evp", ["mit_b0_evp"]),
    # trans_SV_output.py:11-16, tecno_trans.py:9-12, tecno.py:5
    ("models", ["mstcn"]),
    ("models.mstcn", ["MultiStageModel_S", "CausalMambaModel"]),
    ("models.transformer2_3_1", ["Transformer2_3_1"]),
    ("generate_phase_anticipation", ["plot_phase_anticipation", "generate_anticipation_gt"]),
    ("models.adapter_transformer", ["Transformer"]),
    ("models.modules", ["OverlapPatchEmbed", "PromptGenerator", "GaussianFilter", "SRMFilter"]),
    # mix_transformer_evp.py:12, 69
    ("models.segformer_head", ["SegFormerHead"]),
    ("visualizer", ["get_local"]),
]


@pytest.mark.parametrize("mod,names", IMPORTS)
def test_caller_imports_resolve(mod, names):
    m = importlib.import_module(mod)
    for n in names:                                  # `from mod import n` semantics (attribute or submodule)
        if not hasattr(m, n):
            importlib.import_module(f"{mod}.{n}")
        assert hasattr(m, n), f"{mod}.{n}"


def test_star_import_of_models_modules():
    ns = {}
    exec("from models.modules import *", ns)                 # trans_SV_output.py:16 / tecno_trans.py:12
    for n in ("OverlapPatchEmbed", "PromptGenerator", "GaussianFilter", "SRMFilter"):
        assert n in ns
    srm = ns["SRMFilter"]()
    assert srm.srm_layer.weight.shape == (3, 3, 5, 5) and not srm.srm_layer.weight.requires_grad
    assert abs(float(srm.srm_layer.weight[0, 0, 2, 2]) + 1.0) < 1e-7


def test_anticipation_requires_gpu_and_plot_writes(tmp_path):
    import svk
    from generate_phase_anticipation import generate_anticipation_gt, plot_phase_anticipation
    phases = torch.zeros(7, 50, dtype=torch.int64)
    phases[2, 10:20] = 1
    if not torch.cuda.is_available():
        with pytest.raises(svk.SvkError):
            generate_anticipation_gt(phases, 5)
    gt = torch.rand(50, 7)
    p = tmp_path / "ant.png"
    plot_phase_anticipation(str(p), gt * 5, gt)
    assert p.exists() and p.stat().st_size > 1000


# ---- synced augmentations -------------------------------------------------------------------------
def _pil(seed, size=(260, 250)):
    a = np.random.default_rng(seed).integers(0, 256, size=(size[1], size[0], 3), dtype=np.uint8)
    return Image.fromarray(a, "RGB")


def test_random_crop_is_synced_per_clip():
    from models.data_process import RandomCrop, sequence_length
    rc = RandomCrop(224)
    boxes = []
    for i in range(2 * sequence_length):
        img = _pil(i)
        out = rc(img)
        assert out.size == (224, 224)
        a, b = np.asarray(img), np.asarray(out)
        # locate the crop offset
        found = [(y, x) for y in range(img.size[1] - 223) for x in range(img.size[0] - 223)
                 if np.array_equal(a[y, x], b[0, 0]) and np.array_equal(a[y:y + 224, x:x + 224], b)]
        boxes.append(found[0])
    assert len(set(boxes[:sequence_length])) == 1 and len(set(boxes[sequence_length:])) == 1


def test_crop_tensor_and_pil_paths_agree():
    from models.data_process import RandomCrop
    img = _pil(3)
    t = torch.from_numpy(np.asarray(img).copy()).permute(2, 0, 1)
    a, b = RandomCrop(224), RandomCrop(224)
    out_pil = np.asarray(a(img))
    out_t = b(t).permute(1, 2, 0).numpy()
    np.testing.assert_array_equal(out_pil, out_t)


def test_flip_negates_flow_u_and_rotation_rotates_vectors():
    from models.data_process import RandomHorizontalFlip, RandomRotation
    import random
    flip = RandomHorizontalFlip()
    # find a clip index whose draw flips
    k = next(c for c in range(50) if (random.seed(c), random.random())[1] < 0.5)
    flip.count = k * 30
    flow = torch.randn(2, 8, 9)
    out = flip(flow.clone())
    torch.testing.assert_close(out[0], -flow[0].flip(-1))
    torch.testing.assert_close(out[1], flow[1].flip(-1))
    rot = RandomRotation(0)                                    # angle 0: identity grid, identity vectors
    torch.testing.assert_close(rot(flow.clone()), flow)
    rot = RandomRotation(90)
    rot.count = 0
    random.seed(0)
    ang = random.randint(-90, 90)
    rot.count = 0
    const = torch.zeros(2, 33, 33)
    const[0] = 1.0                                             # uniform field (1, 0)
    r = rot(const.clone())
    c, s = np.cos(np.radians(ang)), np.sin(np.radians(ang))
    np.testing.assert_allclose(r[:, 16, 16].numpy(), [c, s], atol=1e-5)


def test_color_jitter_synced_factors_and_identity():
    from models.data_process import ColorJitter
    cj = ColorJitter(0, 0, 0, 0)
    img = _pil(5, (64, 48))
    # factors 1 and hue 0: what remains is the hue op's HSV round trip (torchvision's adjust_hue does it too)
    np.testing.assert_array_equal(np.asarray(cj(img)), np.asarray(img.convert("HSV").convert("RGB")))
    a, b = ColorJitter(), ColorJitter()
    fa = [a.factors() for _ in range(31)]
    fb = [b.factors() for _ in range(31)]
    assert fa == fb and len(set(fa[:30])) == 1 and fa[30] != fa[0]
    out = ColorJitter()(img)
    assert out.size == img.size and out.mode == "RGB"


def test_index_plumbing():
    from models.data_process import get_useful_start_idx, get_useful_start_idx_LFB, SeqSampler
    idx = get_useful_start_idx(3, [5, 4])
    assert idx == [0, 1, 2, 5, 6]
    assert get_useful_start_idx_LFB(1, [2, 2]) == [0, 1, 2, 3]
    assert list(SeqSampler(None, idx)) == idx and len(SeqSampler(None, idx)) == 5


# ---- datasets ---------------------------------------------------------------------------------------
def _write_clip(root, n=3, hw=(120, 160)):
    os.makedirs(root / "cutMargin" / "v1", exist_ok=True)
    os.makedirs(root / "SegMap" / "v1", exist_ok=True)
    os.makedirs(root / "raft_flow_npy" / "v1", exist_ok=True)
    paths, segs = [], []
    rng = np.random.default_rng(0)
    for i in range(n):
        p = root / "cutMargin" / "v1" / f"{i}.jpg"
        s = root / "SegMap" / "v1" / f"{i}.jpg"
        Image.fromarray(rng.integers(0, 256, (hw[0], hw[1], 3), dtype=np.uint8)).save(p, format="PNG")
        Image.fromarray((rng.random((hw[0], hw[1])) > 0.5).astype(np.uint8) * 255).convert("RGB").save(s, format="PNG")
        if i != 1:                                             # frame 1 has no flow file -> zeros
            np.save(root / "raft_flow_npy" / "v1" / f"{i}.npy", rng.standard_normal((hw[0], hw[1], 2)).astype(np.float32))
        paths.append(str(p))
        segs.append(str(s))
    labels = np.zeros((n, 15))
    labels[:, 0] = [1, 2, 3]
    labels[:, 8:15] = rng.random((n, 7))
    return np.array(paths), np.array(segs), labels


def test_cholec_flow_dataset_item_contract(tmp_path):
    from models.data_process import CholecFlowDataset, RandomCrop, RandomHorizontalFlip
    from oracle import preproc as OP

    class Compose:                                             # a torchvision-Compose-shaped container
        def __init__(self, transforms):
            self.transforms = transforms

        def __call__(self, img):
            for t in self.transforms:
                img = t(img)
            return img

    class Resize:                                              # torchvision.transforms.Resize((250, 250)) stand-in
        def __call__(self, img):
            if isinstance(img, torch.Tensor):
                assert img.shape[-2:] == (250, 250)            # the flow is already at the resize size
                return img
            return img.resize((250, 250), Image.BILINEAR)

    class ToTensor:
        def __call__(self, img):
            return torch.from_numpy(np.asarray(img).copy()).permute(2, 0, 1).float() / 255.

    paths, segs, labels = _write_clip(tmp_path)
    raw = CholecFlowDataset(paths, segs, labels, transform=None)
    img, seg, flow, ph, ant = raw[0]
    assert isinstance(img, Image.Image) and flow.shape == (2, 250, 250) and ph.dtype == np.int64
    assert ant.dtype == np.float64 and ant.shape == (7,)
    src = np.load(str(paths[0]).replace("cutMargin", "raft_flow_npy").replace(".jpg", ".npy"))
    ref = OP.cv2_resize_linear(src, (250, 250))
    ref[:, :, 0] *= np.float32(250 / 160)
    ref[:, :, 1] *= np.float32(250 / 120)
    np.testing.assert_allclose(flow.permute(1, 2, 0).numpy(), ref, rtol=1e-6, atol=1e-6)
    assert torch.count_nonzero(raw[1][2]) == 0                 # missing flow file -> zero field
    tf = Compose([Resize(), RandomCrop(200), RandomHorizontalFlip(), ToTensor()])
    ds = CholecFlowDataset(paths, segs, labels, transform=tf)
    img, seg, flow, ph, ant = ds[2]
    assert img.shape == (3, 200, 200) and seg.shape == (3, 200, 200) and flow.shape == (2, 200, 200)
    dec = CholecFlowDataset(paths, segs, labels, decoded=True)[0]
    assert dec[0].dtype == np.uint8 and dec[0].shape == (120, 160, 3) and dec[2].shape == (120, 160, 2)


def test_segmap_datasets_label_columns(tmp_path):
    from models.data_process import CholecSegmapDataset, M2caiSegmapDataset, CholecDataset
    paths, segs, labels = _write_clip(tmp_path)
    it = CholecSegmapDataset(paths, segs, labels)[1]
    assert it[2] == 2 and np.array_equal(it[3], labels[1, 8:15])
    it = M2caiSegmapDataset(paths, segs, labels)[1]
    assert np.array_equal(it[3], labels[1, 1:9])
    it = CholecDataset(paths, labels)[0]
    assert it[1] == 1 and len(it) == 3
