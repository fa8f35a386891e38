"""svk_phase_metrics (relaxed-boundary metrics, eval_and_vis.py:35-161) on the GPU: bit-exact against the
reference's golden outputs and against the oracle on seeded random videos (one launch for all)."""
import numpy as np
import pytest

from oracle import metrics as OM
from test_metrics_cpu import cases, flat

pytestmark = pytest.mark.gpu


def _eq(got, ref):
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_array_equal(got[~np.isnan(got)], ref[~np.isnan(ref)])


def test_kernel_matches_reference_golden(cuda):
    from svk.metrics import evaluate_videos, evaluate_strict_boundary
    cs = list(cases())
    for tol in (10, 3, 0):
        sel = [c for c in cs if c[1] == tol]
        res = evaluate_videos([c[2] for c in sel], [c[3] for c in sel], 7, tol)
        for c, r in zip(sel, res):
            _eq(flat(r), c[4])
    c = cs[0]
    _eq(flat(evaluate_strict_boundary(c[2], c[3], 7, c[1])), c[4])


def test_kernel_matches_oracle_random_videos(cuda):
    from svk.metrics import evaluate_videos
    r = np.random.default_rng(5)
    gts, preds = [], []
    for T in list(r.integers(1000, 6001, size=38)) + [1, 7000]:
        lens = r.integers(1, max(2, T // 3), size=int(r.integers(3, 12)))
        gt = np.repeat(r.integers(0, 7, size=len(lens)), lens)[:T]
        gt = np.concatenate([gt, np.full(T - len(gt), 6)]) if len(gt) < T else gt
        pred = np.where(r.random(T) < 0.2, np.clip(gt + r.integers(-2, 3, size=T), 0, 6), np.roll(gt, 7))
        gts.append(gt)
        preds.append(pred)
    for tol in (10, 25):
        res = evaluate_videos(gts, preds, 7, tol)
        for g, p, got in zip(gts, preds, res):
            _eq(flat(got), flat(OM.evaluate_strict_boundary(g, p, 7, tol)))
