"""Drop-in for the reference's ``models/data_process.py``: every name train_evp.py:19-20 and
generate_evp_LFB.py:23 import from it.

* index plumbing: ``SeqSampler``, ``get_useful_start_idx``, ``get_useful_start_idx_LFB``
  (data_process.py:189-200, 307-324);
* the synced training augmentations ``RandomCrop``, ``RandomHorizontalFlip``, ``RandomRotation``,
  ``ColorJitter`` (data_process.py:53-186): every instance reseeds Python's ``random`` with
  ``count // sequence_length`` per call, so the frames, segmaps and flows of one 30-frame clip share
  the same crop / flip / angle / colour factors; PIL images and tensors (flow: the u component is
  negated by a flip, (u, v) is rotated with the grid) like the reference;
* the datasets ``CholecDataset``, ``CholecSegmapDataset``, ``M2caiSegmapDataset`` and
  ``CholecFlowDataset`` with the reference's per-item contracts (data_process.py:203-304, 396-490);
  ``CholecFlowDataset`` resizes the RAFT ``.npy`` flow to 250x250 exactly like its ``cv2.resize``
  (INTER_LINEAR) call and rescales the displacements.

torchvision and OpenCV are used when they are importable (deployment boxes — the reference's scripts
import torchvision themselves); without them (this image) the PIL / torch restatements below carry the
same arithmetic: torchvision's PIL colour ops are ``ImageEnhance`` + an HSV hue shift, its rotation is
``Image.rotate(NEAREST)`` on PIL and a nearest-neighbour affine grid on tensors, cv2's INTER_LINEAR
is the separable two-tap float blend of ``svk.preproc.cv2_linear_table``.  These are data-loader
(host, worker-process) steps of the reference's pipeline, not the GPU hot path; the batched GPU
transforms (``svk.preproc.frame_transform`` / ``flow_transform``) are the fast path for extraction:
construct ``CholecFlowDataset(..., transform=None, decoded=True)`` to get the decoded uint8 frames and
raw flows for them.

``SyntheticCholecFlowDataset`` fills CholecFlowDataset's item contract with seeded synthetic data
(benchmarks and tests; no Cholec80 data ships with the container).
"""
import math
import numbers
import os
import random

import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image, ImageEnhance, ImageOps
from torch.utils.data import Dataset, Sampler

try:                                    # exact reference behaviour where the reference's deps exist
    import torchvision.transforms.functional as TF
    from torchvision import transforms as _tv_transforms
except ImportError:                     # this image: PIL / torch restatements below
    TF, _tv_transforms = None, None
try:
    import cv2
except ImportError:
    cv2 = None

device = torch.device("cuda:0")          # module global of the reference (data_process.py:30)
sequence_length = 30
MEAN = (0.41757566, 0.26098573, 0.25888634)   # train_evp.py:152
STD = (0.21938758, 0.1983, 0.19342837)


def pil_loader(path, mode="RGB"):
    """Open an image file and convert it (data_process.py:34-49)."""
    with open(path, "rb") as f:
        with Image.open(f) as img:
            return img.convert(mode)


# ---- synced augmentations (data_process.py:53-186) ----------------------------------------------
def _rotate_tensor_nearest(img, angle):
    """torchvision.transforms.functional.rotate on a [C, H, W] tensor: nearest-neighbour affine grid
    about the image centre, zero fill, no expansion (angle in degrees, counter-clockwise)."""
    if TF is not None:
        return TF.rotate(img, angle)
    c, h, w = img.shape[-3:]
    rot = math.radians(-angle)
    # inverse affine matrix of a pure rotation about the centre (output -> input coordinates)
    a, b, cc, d = math.cos(rot), -math.sin(rot), math.sin(rot), math.cos(rot)
    m = [d, -b, 0.0, -cc, a, 0.0]
    theta = torch.tensor([[m[0], m[1], m[2]], [m[3], m[4], m[5]]], dtype=torch.float32)
    xs = torch.linspace(-w * 0.5 + 0.5, w * 0.5 + 0.5 - 1, steps=w)
    ys = torch.linspace(-h * 0.5 + 0.5, h * 0.5 + 0.5 - 1, steps=h)
    base = torch.ones(h, w, 3)
    base[..., 0] = xs
    base[..., 1] = ys[:, None]
    grid = (base.view(1, h * w, 3) @ (theta.t() / torch.tensor([0.5 * w, 0.5 * h]))).view(1, h, w, 2)
    out = F.grid_sample(img.reshape(1, -1, h, w).float(), grid.to(img.device), mode="nearest",
                        padding_mode="zeros", align_corners=False)
    return out.view(img.shape).to(img.dtype)


def _rotate_pil(img, angle):
    return TF.rotate(img, angle) if TF is not None else img.rotate(angle, resample=Image.NEAREST, expand=False)


def _adjust_hue_pil(img, hue_factor):
    if img.mode in {"L", "1", "I", "F"}:
        return img
    h, s, v = img.convert("HSV").split()
    np_h = np.array(h, dtype=np.uint8)
    shift = int(hue_factor * 255)                     # np.array(hue_factor * 255).astype(uint8): truncate, wrap
    np_h = ((np_h.astype(np.int16) + shift) % 256).astype(np.uint8)
    return Image.merge("HSV", (Image.fromarray(np_h, "L"), s, v)).convert(img.mode)


class RandomCrop(object):
    """Synced random crop (data_process.py:53-97): the offset is drawn after random.seed(count // 30)."""

    def __init__(self, size, padding=0):
        self.size = (int(size), int(size)) if isinstance(size, numbers.Number) else size
        self.padding = padding
        self.count = 0

    def draw(self, w, h):
        """The offset __call__ draws for a (padded) w x h input — (x1, y1), count advanced — or None when the
        input already has the crop size (no draw, no count: data_process.py:71-72)."""
        th, tw = self.size
        if w == tw and h == th:
            return None
        random.seed(self.count // sequence_length)
        x1 = random.randint(0, w - tw)
        y1 = random.randint(0, h - th)
        self.count += 1
        return x1, y1

    def __call__(self, img):
        th, tw = self.size
        if isinstance(img, torch.Tensor):
            if self.padding > 0:
                img = F.pad(img, (self.padding,) * 4, value=0)
            xy = self.draw(img.shape[-1], img.shape[-2])
            return img if xy is None else img[..., xy[1]:xy[1] + th, xy[0]:xy[0] + tw]
        if self.padding > 0:
            img = ImageOps.expand(img, border=self.padding, fill=0)
        xy = self.draw(*img.size)
        return img if xy is None else img.crop((xy[0], xy[1], xy[0] + tw, xy[1] + th))


class RandomHorizontalFlip(object):
    """Synced horizontal flip with p = 0.5 (data_process.py:100-123); a 2-channel tensor is a flow
    field and its u component changes sign."""

    def __init__(self):
        self.count = 0

    def draw(self):
        """True when this call flips (count advanced)."""
        random.seed(self.count // sequence_length)
        prob = random.random()
        self.count += 1
        return prob < 0.5

    def __call__(self, img):
        if not self.draw():
            return img
        if isinstance(img, torch.Tensor):
            img = img.flip(-1)
            if img.shape[0] == 2:
                img[0] = -img[0]
            return img
        return img.transpose(Image.FLIP_LEFT_RIGHT)


class RandomRotation(object):
    """Synced rotation by an integer angle in [-degrees, degrees] (data_process.py:126-160); flow
    vectors are rotated with the grid."""

    def __init__(self, degrees):
        self.degrees = degrees
        self.count = 0

    def draw(self):
        """The integer angle of this call (count advanced)."""
        random.seed(self.count // sequence_length)
        self.count += 1
        return random.randint(-self.degrees, self.degrees)

    def __call__(self, img):
        angle = self.draw()
        if isinstance(img, torch.Tensor):
            img = _rotate_tensor_nearest(img, angle)
            if img.shape[0] == 2:
                rad = math.radians(angle)
                cos_a, sin_a = math.cos(rad), math.sin(rad)
                u, v = img[0].clone(), img[1].clone()
                img[0] = u * cos_a - v * sin_a
                img[1] = u * sin_a + v * cos_a
            return img
        return _rotate_pil(img, angle)


class ColorJitter(object):
    """Synced brightness / contrast / saturation / hue jitter (data_process.py:163-186)."""

    def __init__(self, brightness=0.1, contrast=0.1, saturation=0.1, hue=0.1):
        self.brightness, self.contrast, self.saturation, self.hue = brightness, contrast, saturation, hue
        self.count = 0

    def factors(self):
        random.seed(self.count // sequence_length)
        self.count += 1
        return (random.uniform(1 - self.brightness, 1 + self.brightness),
                random.uniform(1 - self.contrast, 1 + self.contrast),
                random.uniform(1 - self.saturation, 1 + self.saturation),
                random.uniform(-self.hue, self.hue))

    def __call__(self, img):
        b, c, s, h = self.factors()
        if TF is not None:
            return TF.adjust_hue(TF.adjust_saturation(TF.adjust_contrast(TF.adjust_brightness(img, b), c), s), h)
        img = ImageEnhance.Brightness(img).enhance(b)
        img = ImageEnhance.Contrast(img).enhance(c)
        img = ImageEnhance.Color(img).enhance(s)
        return _adjust_hue_pil(img, h)


# ---- index plumbing (data_process.py:189-200, 307-324) ------------------------------------------
class SeqSampler(Sampler):
    def __init__(self, data_source, idx):
        super().__init__()
        self.data_source = data_source
        self.idx = idx

    def __iter__(self):
        return iter(self.idx)

    def __len__(self):
        return len(self.idx)


def get_useful_start_idx(sequence_length, list_each_length):
    """All start indices whose window of ``sequence_length`` frames stays inside one video."""
    idx, count = [], 0
    for n in list_each_length:
        idx.extend(range(count, count + (n + 1 - sequence_length)))
        count += n
    return idx


def get_useful_start_idx_LFB(sequence_length, list_each_length):
    return get_useful_start_idx(sequence_length, list_each_length)


# ---- datasets (data_process.py:203-304, 396-490) -------------------------------------------------
class CholecDataset(Dataset):
    """Frames + phase label (column 0) + anticipation targets (columns 8..14)."""

    def __init__(self, file_paths, file_labels, transform=None, loader=pil_loader):
        self.file_paths = file_paths
        self.file_labels_phase = file_labels[:, 0]
        self.file_labels_phase_ant = file_labels[:, 8:15]
        self.transform = transform
        self.loader = loader

    def __getitem__(self, index):
        imgs = self.loader(self.file_paths[index])
        if self.transform is not None:
            imgs = self.transform(imgs)
        return (imgs, self.file_labels_phase[index].astype(np.int64),
                self.file_labels_phase_ant[index].astype(np.float64))

    def __len__(self):
        return len(self.file_paths)


class CholecSegmapDataset(Dataset):
    """Frames + segmentation maps (both RGB, the same transform) + labels."""
    ant_cols = (8, 15)

    def __init__(self, file_paths, seg_paths, file_labels, transform=None, loader=pil_loader):
        self.file_paths = file_paths
        self.seg_paths = seg_paths
        self.file_labels_phase = file_labels[:, 0]
        self.file_labels_phase_ant = file_labels[:, self.ant_cols[0]:self.ant_cols[1]]
        self.transform = transform
        self.loader = loader

    def __getitem__(self, index):
        imgs = self.loader(self.file_paths[index], mode="RGB")
        segmaps = self.loader(self.seg_paths[index], mode="RGB")
        if self.transform is not None:
            imgs = self.transform(imgs)
            segmaps = self.transform(segmaps)
        return (imgs, segmaps, self.file_labels_phase[index].astype(np.int64),
                self.file_labels_phase_ant[index].astype(np.float64))

    def __len__(self):
        return len(self.file_paths)


class M2caiSegmapDataset(CholecSegmapDataset):
    """m2cai16: anticipation targets are columns 1..8 (8 phases)."""
    ant_cols = (1, 9)


def cv2_resize_linear(img, size):
    """cv2.resize(img, size = (W, H), interpolation=cv2.INTER_LINEAR) for a float32 [H, W, C] array:
    per-axis source index + (1 - f, f) float32 weights, horizontal then vertical float32 blend."""
    if cv2 is not None:
        return cv2.resize(img, size, interpolation=cv2.INTER_LINEAR)
    from svk.preproc import cv2_linear_table
    ow, oh = size
    h, w = img.shape[:2]
    xo, xa = cv2_linear_table(w, ow)
    yo, ya = cv2_linear_table(h, oh)
    x1 = np.minimum(xo + 1, w - 1)
    y1 = np.minimum(yo + 1, h - 1)
    img = img.astype(np.float32)
    rows = img[:, xo] * xa[None, :, 0:1] + img[:, x1] * xa[None, :, 1:2]          # [h, ow, C]
    return (rows[yo] * ya[:, None, 0:1] + rows[y1] * ya[:, None, 1:2]).astype(np.float32)


def _is_flow_geometric(t):
    """Which transforms of a Compose CholecFlowDataset replays on the flow tensor (data_process.py:466-480):
    the synced crop / flip / rotation, and torchvision's CenterCrop, RandomCrop, RandomHorizontalFlip
    and Resize (the flow is already at the 250x250 resize size)."""
    if isinstance(t, (RandomCrop, RandomHorizontalFlip, RandomRotation)):
        return True
    return type(t).__name__ in ("CenterCrop", "RandomCrop", "RandomHorizontalFlip", "Resize")


class CholecFlowDataset(Dataset):
    """CholecSegmapDataset + the RAFT optical flow of the frame (``cutMargin`` -> ``raft_flow_npy``,
    ``.jpg`` -> ``.npy``; zeros when the file is missing): (imgs, segmaps, flow [2, H, W], phase,
    anticipation).  ``decoded=True`` (with ``transform=None``) returns the decoded uint8 [H, W, 3]
    frame / segmap arrays and the raw [H, W, 2] flow instead, for the batched GPU transforms of
    svk.preproc."""

    def __init__(self, file_paths, seg_paths, file_labels, transform=None, loader=pil_loader, decoded=False):
        self.file_paths = file_paths
        self.seg_paths = seg_paths
        self.file_labels_phase = file_labels[:, 0]
        self.file_labels_phase_ant = file_labels[:, 8:15]
        self.transform = transform
        self.loader = loader
        self.target_size = (250, 250)
        self.decoded = decoded

    def _flow(self, img_name, img_size):
        flow_path = img_name.replace("cutMargin", "raft_flow_npy").replace(".jpg", ".npy")
        if os.path.exists(flow_path):
            return np.load(flow_path)                                  # [H, W, 2] float32 (allow_pickle off)
        w, h = img_size
        return np.zeros((h, w, 2), dtype=np.float32)

    def __getitem__(self, index):
        img_name = self.file_paths[index]
        labels = (self.file_labels_phase[index].astype(np.int64), self.file_labels_phase_ant[index].astype(np.float64))
        imgs = self.loader(img_name, mode="RGB")
        segmaps = self.loader(self.seg_paths[index], mode="RGB")
        flow = self._flow(img_name, imgs.size)
        if self.decoded:
            return (np.asarray(imgs), np.asarray(segmaps), np.ascontiguousarray(flow, dtype=np.float32)) + labels
        h0, w0 = flow.shape[:2]
        fr = cv2_resize_linear(flow, self.target_size)
        fr[:, :, 0] *= self.target_size[0] / w0
        fr[:, :, 1] *= self.target_size[1] / h0
        flow_tensor = torch.from_numpy(fr).permute(2, 0, 1).float()
        if self.transform is not None:
            imgs = self.transform(imgs)
            segmaps = self.transform(segmaps)
            steps = getattr(self.transform, "transforms", None)
            if steps is not None:
                for t in steps:
                    if _is_flow_geometric(t):
                        flow_tensor = t(flow_tensor)
            elif _is_flow_geometric(self.transform) and type(self.transform).__name__ != "Resize":
                flow_tensor = self.transform(flow_tensor)
        return (imgs, segmaps, flow_tensor) + labels

    def __len__(self):
        return len(self.file_paths)


class SyntheticDecodedCholecFlow(Dataset):
    """Seeded synthetic items in CholecFlowDataset(decoded=True)'s contract: decoded uint8 RGB frame and
    binary segmap [H, W, 3], raw RAFT-style flow [H, W, 2] f32 (N(0, 2 px)), phase, anticipation.  The
    default frame size is 250x250 (the reference's own data_process.py:493-511 stubs)."""

    def __init__(self, n, seed=0, size=(250, 250)):
        self.n, self.seed, self.size = n, seed, tuple(size)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        r = np.random.default_rng((self.seed, i))
        h, w = self.size
        img = r.integers(0, 256, (h, w, 3), dtype=np.uint8)
        yy, xx = np.mgrid[0:h, 0:w]
        cy, cx, ay, ax = r.uniform(0, h), r.uniform(0, w), r.uniform(10, 70), r.uniform(10, 70)
        m = ((((yy - cy) / ay) ** 2 + ((xx - cx) / ax) ** 2) <= 1).astype(np.uint8) * 255
        seg = np.repeat(m[:, :, None], 3, axis=2)
        flow = (2.0 * r.standard_normal((h, w, 2))).astype(np.float32)
        return img, seg, flow, np.int64(r.integers(0, 7)), r.uniform(0, 1, 7).astype(np.float64)


class SyntheticCholecFlowDataset(Dataset):
    """Seeded synthetic frames with CholecFlowDataset's per-item contract."""

    def __init__(self, n, seed=0, size=224):
        self.n, self.seed, self.size = n, seed, size
        self.mean = torch.tensor(MEAN).view(3, 1, 1)
        self.std = torch.tensor(STD).view(3, 1, 1)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        r = np.random.default_rng((self.seed, i))
        s = self.size
        img = torch.from_numpy(r.integers(0, 256, (3, s, s), dtype=np.uint8)).float() / 255.
        yy, xx = np.mgrid[0:s, 0:s]
        cy, cx, ay, ax = r.uniform(0, s), r.uniform(0, s), r.uniform(10, 70), r.uniform(10, 70)
        m = torch.from_numpy((((yy - cy) / ay) ** 2 + ((xx - cx) / ax) ** 2 <= 1).astype(np.float32))
        seg = m.expand(3, s, s)
        flow = torch.from_numpy((2.0 * r.standard_normal((2, s, s))).astype(np.float32))
        phase = np.int64(r.integers(0, 7))
        ant = r.uniform(0, 1, 7).astype(np.float64)
        return (img - self.mean) / self.std, (seg - self.mean) / self.std, flow, phase, ant
