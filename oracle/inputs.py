"""Synthetic Cholec80-shaped inputs (oracle / test infrastructure).

SURVEY.md §8(d): frames are uint8 RGB ~ U{0..255}, /255, normalised with the
Cholec80 mean/std of train_evp.py:152; segmaps are binary masks (random ellipses)
replicated to 3 channels and put through the same normalisation
(data_process.py:416-462 applies the image transform to masks too); flow is
N(0, 2 px) in ``[B, 1, 2, 224, 224]`` (data_process.py:432-487 layout).
"""
import numpy as np
import torch

MEAN = np.array([0.41757566, 0.26098573, 0.25888634], dtype=np.float32)
STD = np.array([0.21938758, 0.1983, 0.19342837], dtype=np.float32)


def frames(B, seed=0, size=224):
    r = np.random.default_rng(1000 + seed)
    u8 = r.integers(0, 256, size=(B, 3, size, size), dtype=np.uint8)
    x = u8.astype(np.float32) / 255.0
    x = (x - MEAN[None, :, None, None]) / STD[None, :, None, None]
    return torch.from_numpy(x).view(B, 1, 3, size, size)


def segmaps(B, seed=0, size=224):
    r = np.random.default_rng(2000 + seed)
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32)
    m = np.zeros((B, size, size), dtype=np.float32)
    for b in range(B):
        for _ in range(int(r.integers(1, 4))):
            cy, cx = r.uniform(0, size, 2)
            ay, ax = r.uniform(10, 70, 2)
            m[b] = np.maximum(m[b], (((yy - cy) / ay) ** 2 + ((xx - cx) / ax) ** 2 <= 1.0).astype(np.float32))
    x = np.repeat(m[:, None], 3, axis=1)
    x = (x - MEAN[None, :, None, None]) / STD[None, :, None, None]
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).view(B, 1, 3, size, size)


def flow(B, seed=0, size=224):
    r = np.random.default_rng(3000 + seed)
    f = (2.0 * r.standard_normal((B, 1, 2, size, size))).astype(np.float32)
    return torch.from_numpy(f)


def labels(B, seed=0):
    r = np.random.default_rng(4000 + seed)
    phase = torch.from_numpy(r.integers(0, 7, size=(B,)).astype(np.int64))
    ant = torch.from_numpy(r.uniform(0, 1, size=(B, 7)).astype(np.float32))
    return phase, ant


def lfb(T, dim=2048, seed=0):
    """Per-frame long-term features (the LFB pickle rows consumed by tecno/trans_SV_output)."""
    r = np.random.default_rng(5000 + seed)
    return torch.from_numpy(r.standard_normal((1, T, dim)).astype(np.float32))


def video_lengths(n=40, seed=0, lo=1000, hi=6000):
    r = np.random.default_rng(6000 + seed)
    return [int(t) for t in r.integers(lo, hi + 1, size=n)]


def digest(t):
    """Cheap order-sensitive checksum used to verify that regenerated inputs match the fixtures."""
    a = t.detach().double().flatten().numpy()
    w = np.linspace(1.0, 2.0, a.size)
    return np.array([a.sum(), (a * w).sum(), np.abs(a).sum()], dtype=np.float64)
