"""CPU restatement of eval_and_vis.evaluate_strict_boundary (eval_and_vis.py:35-161) — test infrastructure only.

Per maximal run [s, e) of ground-truth phase p (eval_and_vis.py:50-62), t = min(tolerance, e - s) (:64-65);
on the ORIGINAL diff = pred - gt, head values (first t frames) and tail values (last t) are set to 0 in the
updated diff when they match the phase rule (:86-110: phases 3/4 head -1, tail +1/+2; 5/6 head -1/-2,
tail +1/+2; others head -1, tail +1).  Per phase (:120-155): NaN triple when the phase is absent from the
ground truth, else TP = #(updated diff == 0 over gt|pred union), Jaccard TP/|union|, precision TP/#pred
(0 without predictions), recall TP/#gt, all x100; accuracy = #(updated diff == 0) / T x 100 (:158-159).
Pinned by tests/golden/metrics_golden.npz (the reference function run on seeded sequences)."""
import numpy as np


def evaluate_strict_boundary(y_gt, y_pred, num_phases=7, tolerance=10):
    g = np.asarray(y_gt, dtype=np.int64)
    q = np.asarray(y_pred, dtype=np.int64)
    diff = q - g
    upd = diff.copy()
    T = len(g)
    i = 0
    while i < T:                                   # maximal runs of one ground-truth value
        j = i
        while j + 1 < T and g[j + 1] == g[i]:
            j += 1
        p, s, e = int(g[i]), i, j + 1
        if 0 <= p < num_phases:
            t = min(tolerance, e - s)
            for k in range(s, s + t):
                d = diff[k]
                if (d == -1) or (p in (5, 6) and d == -2):
                    upd[k] = 0
            for k in range(e - t, e):
                d = diff[k]
                if d == 1 or (p in (3, 4, 5, 6) and d == 2):
                    upd[k] = 0
        i = e
    prec, rec, jacc = [], [], []
    for p in range(num_phases):
        gm, pm = g == p, q == p
        if not gm.any():
            prec.append(np.nan); rec.append(np.nan); jacc.append(np.nan)
            continue
        union = np.where(gm | pm)[0]
        tp = np.sum(upd[union] == 0)
        jacc.append((tp / len(union)) * 100)
        pc, gc = np.sum(pm), np.sum(gm)
        prec.append((tp / pc * 100) if pc > 0 else 0)
        rec.append((tp / gc * 100) if gc > 0 else 0)
    acc = (np.sum(upd == 0) / T) * 100
    return acc, prec, rec, jacc
