"""Relaxed-boundary metrics oracle (oracle/metrics.py) against the reference's own outputs
(tests/golden/metrics_golden.npz, made by tests/golden/gen_metrics.py from eval_and_vis.py:35-161)."""
import os

import numpy as np
import pytest

from oracle import metrics as OM

GOLD = os.path.join(os.path.dirname(__file__), "golden", "metrics_golden.npz")


def cases():
    d = np.load(GOLD)
    for k in sorted(d.files):
        if "_t" in k:
            name, tol = k.rsplit("_t", 1)
            yield name, int(tol), d[name + "_gt"].astype(np.int64), d[name + "_pred"].astype(np.int64), d[k]


def flat(res):
    acc, prec, rec, jacc = res
    return np.array([acc] + list(prec) + list(rec) + list(jacc), dtype=np.float64)


@pytest.mark.parametrize("case", list(cases()), ids=lambda c: f"{c[0]}_t{c[1]}")
def test_oracle_matches_reference_golden(case):
    name, tol, gt, pred, ref = case
    got = flat(OM.evaluate_strict_boundary(gt, pred, 7, tol))
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_array_equal(got[~np.isnan(got)], ref[~np.isnan(ref)])       # bit-exact
