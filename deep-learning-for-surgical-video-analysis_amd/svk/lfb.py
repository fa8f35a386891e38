"""Long-term feature bank (LFB) extraction — the loop of generate_evp_LFB.py:439-520, MI355X build.

The reference grows a float64 numpy array with ``np.concatenate`` after every batch (quadratic
host copying, generate_evp_LFB.py:457/477/497) and finally pickles it (:513-520), which
``tecno.py`` / ``trans_SV_output.py`` load back (tecno.py:80-85).  Here the (N, 2048) bank is
preallocated once, each batch's features are copied into their rows, frames are sharded across
ranks (one process per GPU) and gathered at the end, and the bank is written in the reference's
pickle format (float64 ndarray) plus an fp32 ``.npy`` sidecar.
"""
import pickle

import numpy as np
import torch

from .shard import shard_range, gather_rows


def extract_lfb(model, dataset, batch_size=200, device=None, rank=0, world=1, group=None):
    """Run ``model(x, y, flow, return_features=True)`` over ``dataset`` items
    (img [3,H,W], segmap [3,H,W], flow [2,H,W], ...) in index order; returns the (N, 2048) float32
    bank (on every rank when world > 1)."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    n = len(dataset)
    a, b = shard_range(n, rank, world)
    local = torch.empty(b - a, 2048, dtype=torch.float32, device=device)
    with torch.no_grad():
        for s in range(a, b, batch_size):
            e = min(s + batch_size, b)
            items = [dataset[i] for i in range(s, e)]
            x = torch.stack([torch.as_tensor(it[0]) for it in items]).to(device, non_blocking=True)
            y = torch.stack([torch.as_tensor(it[1]) for it in items]).to(device, non_blocking=True)
            fl = torch.stack([torch.as_tensor(it[2]) for it in items]).to(device, non_blocking=True)
            f = model(x.view(-1, 1, 3, x.shape[-2], x.shape[-1]), y.view(-1, 1, 3, y.shape[-2], y.shape[-1]),
                      fl.view(-1, 1, 2, fl.shape[-2], fl.shape[-1]), return_features=True)
            local[s - a:e - a] = f
    bank = gather_rows(local, n, group) if world > 1 else local
    return bank


def save_lfb(bank, pkl_path, npy_path=None):
    """Reference format: pickle of a float64 (N, 2048) ndarray (generate_evp_LFB.py:513-520)."""
    arr = bank.detach().cpu().numpy()
    with open(pkl_path, "wb") as f:
        pickle.dump(arr.astype(np.float64), f)
    if npy_path:
        np.save(npy_path, arr.astype(np.float32))
