"""Generate tests/golden/metrics_golden.npz by running the reference's own
eval_and_vis.evaluate_strict_boundary (eval_and_vis.py:35-161) in this container on seeded phase sequences.
Run: PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_metrics.py   (needs /root/reference; not on the GPU box)."""
import os
import sys

import numpy as np

REF = "/root/reference"


def sequences():
    """Seeded (gt, pred) pairs: Cholec80-like ordered phases with boundary-shifted / noisy predictions,
    absent phases, tiny runs (t = run length), one-frame videos and random labels."""
    r = np.random.default_rng(0)
    out = {}
    for k, T in enumerate((1, 2, 15, 60, 1733, 4000)):
        lens = r.integers(1, max(2, T // 4), size=7)
        gt = np.repeat(np.arange(7), lens)[:T]
        if len(gt) < T:
            gt = np.concatenate([gt, np.full(T - len(gt), 6)])
        shift = np.roll(gt, int(r.integers(-12, 13)))
        noise = np.where(r.random(T) < 0.1, r.integers(0, 7, size=T), shift)
        out[f"v{k}_gt"], out[f"v{k}_pred"] = gt, noise
    gt = np.repeat([0, 1, 3, 4, 3, 5, 6], [30, 5, 40, 2, 30, 25, 11])     # repeated phase, 2-frame run
    out["v6_gt"], out["v6_pred"] = gt, np.clip(gt + r.integers(-2, 3, size=len(gt)), 0, 6)
    out["v7_gt"], out["v7_pred"] = r.integers(0, 7, size=500), r.integers(0, 7, size=500)
    out["v8_gt"], out["v8_pred"] = np.full(300, 2), np.full(300, 3)         # phases absent from gt -> NaN
    return out


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import eval_and_vis as ev
    seqs = sequences()
    res = {}
    for name in sorted({k.rsplit("_", 1)[0] for k in seqs}):
        for tol in (10, 3, 0):
            acc, prec, rec, jacc = ev.evaluate_strict_boundary(seqs[name + "_gt"], seqs[name + "_pred"], 7, tol)
            res[f"{name}_t{tol}"] = np.array([acc] + list(prec) + list(rec) + list(jacc), dtype=np.float64)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "metrics_golden.npz"),
                        **{k: v.astype(np.int8) for k, v in seqs.items()}, **res)


if __name__ == "__main__":
    main()
