"""Anticipation-target oracle (oracle/labels.py) pinned to golden vectors produced by the reference's own
generate_anticipation_gt (tests/golden/gen_anticipation.py): bit-exact."""
import numpy as np
import pytest
import torch

from oracle import labels as OL

G = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "anticipation_golden.npz"))


@pytest.mark.parametrize("name", ["v1", "v2", "v3", "v4", "v5"])
@pytest.mark.parametrize("horizon", [5.0, 3])
def test_oracle_matches_reference_golden(name, horizon):
    ph = torch.from_numpy(G[f"{name}_phases"].astype(np.int64))
    out = OL.anticipation_gt(ph, horizon)
    np.testing.assert_array_equal(out.numpy(), G[f"{name}_h{horizon}"])
