"""Relaxed-boundary phase metrics of eval_and_vis.py:35-161 (the Cholec80 Evaluate.m rules) on the GPU.

``svk_phase_metrics`` returns exact integer counts per video (one workgroup per video: run boundaries by
block scans, forgiven head/tail differences, per-phase TP / union / predicted / ground-truth counts); the
ratios are formed here in float64 with the reference's own expressions, so results are identical to
``evaluate_strict_boundary`` bit for bit."""
import numpy as np
import torch

from . import _lib
from .ops import _stream


def _counts(gts, preds, num_phases, tolerance, device):
    lens = [len(g) for g in gts]
    if any(len(p) != n for p, n in zip(preds, lens)):
        raise _lib.SvkError("svk.metrics: every prediction must have its ground truth's length")
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    cat = lambda seqs: torch.from_numpy(np.concatenate([np.asarray(s, dtype=np.int64).reshape(-1) for s in seqs])
                                        if seqs else np.zeros(0, np.int64))
    g = cat(gts).to(device)
    p = cat(preds).to(device)
    o = torch.from_numpy(offs).to(device)
    P = int(num_phases)
    out = torch.zeros(len(gts), 2 + 4 * P, dtype=torch.int64, device=device)
    _lib.call("svk_phase_metrics", g.data_ptr(), p.data_ptr(), o.data_ptr(), len(gts), P, int(tolerance),
              out.data_ptr(), _stream())
    return out.cpu().numpy()


def _ratios(row, P):
    T, total = row[0], row[1]
    prec, rec, jacc = [], [], []
    for k in range(P):
        tp, union, pred_count, gt_count = (np.int64(x) for x in row[2 + 4 * k: 6 + 4 * k])
        if gt_count == 0:                                   # eval_and_vis.py:126-131
            prec.append(np.nan)
            rec.append(np.nan)
            jacc.append(np.nan)
            continue
        jacc.append((tp / union) * 100)
        prec.append((tp / pred_count * 100) if pred_count > 0 else 0)
        rec.append((tp / gt_count * 100) if gt_count > 0 else 0)
    with np.errstate(divide="ignore", invalid="ignore"):
        acc = (np.int64(total) / np.int64(T)) * 100 if T > 0 else np.float64(np.nan)
    return acc, prec, rec, jacc


def evaluate_videos(gts, preds, num_phases=7, tolerance=10, device="cuda"):
    """All videos in one launch -> [(acc, prec_list, rec_list, jacc_list)] per video."""
    if not torch.cuda.is_available():
        raise _lib.SvkError("svk.metrics: no GPU (the MI355X build has no CPU path)")
    rows = _counts(list(gts), list(preds), num_phases, tolerance, device)
    return [_ratios(r, int(num_phases)) for r in rows]


def evaluate_strict_boundary(y_gt, y_pred, num_phases=7, tolerance=10):
    """Drop-in for eval_and_vis.evaluate_strict_boundary (same arguments and return values)."""
    return evaluate_videos([y_gt], [y_pred], num_phases, tolerance)[0]
