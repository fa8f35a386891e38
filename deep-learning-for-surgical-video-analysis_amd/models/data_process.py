"""Data-side helpers the hot-path callers import (drop-in subset of models/data_process.py).

* ``SeqSampler``, ``get_useful_start_idx``, ``get_useful_start_idx_LFB`` — the index
  plumbing imported by train_evp.py / generate_evp_LFB.py (data_process.py:189-200,
  307-324), restated.
* ``SyntheticCholecFlowDataset`` — the tensor contract of ``CholecFlowDataset``
  (data_process.py:396-490: image [3,224,224] normalised, segmap [3,224,224] through the
  same normalisation, flow [2,224,224], phase int64, anticipation float64[7]) filled with
  seeded synthetic data.  JPEG decode / augmentation of real Cholec80 frames is out of
  scope for this round; no data ships with the container.
"""
import numpy as np
import torch
from torch.utils.data import Dataset, Sampler

sequence_length = 30
MEAN = (0.41757566, 0.26098573, 0.25888634)   # train_evp.py:152
STD = (0.21938758, 0.1983, 0.19342837)


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
