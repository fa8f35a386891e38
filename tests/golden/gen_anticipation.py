"""Generate tests/golden/anticipation_golden.npz by running the reference's own
generate_phase_anticipation.generate_anticipation_gt (generate_phase_anticipation.py:10-34) in this container.
Run: PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_anticipation.py   (needs /root/reference; not on the GPU box)."""
import contextlib
import io
import os
import sys

import numpy as np
import torch

REF = "/root/reference"


def phase_sequences():
    """Seeded one-hot phase signals [7, T]: ordered phase segments (Cholec80-like) and a random one."""
    r = np.random.default_rng(0)
    seqs = {}
    for name, T in (("v1", 1), ("v2", 40), ("v3", 1800)):
        lens = r.integers(1, max(2, T // 5), size=7)
        labels = np.repeat(np.arange(7), lens)[:T]
        labels = np.concatenate([labels, np.full(T - len(labels), 6)]) if len(labels) < T else labels
        seqs[name] = labels
    seqs["v4"] = r.integers(0, 7, size=600)
    seqs["v5"] = np.full(400, 2)                      # phases that never appear -> horizon everywhere
    return {k: np.stack([(v == p).astype(np.int64) for p in range(7)]) for k, v in seqs.items()}


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import generate_phase_anticipation as gpa
    out = {}
    for name, ph in phase_sequences().items():
        for horizon in (5.0, 3):
            with contextlib.redirect_stdout(io.StringIO()):      # the reference prints every phase code
                t = gpa.generate_anticipation_gt(torch.from_numpy(ph), horizon=horizon)
            out[f"{name}_phases"] = ph.astype(np.int8)
            out[f"{name}_h{horizon}"] = t.numpy()
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "anticipation_golden.npz"), **out)


if __name__ == "__main__":
    main()
