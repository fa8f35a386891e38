"""svk_anticipation_gt (generate_phase_anticipation.py:10-34 on the GPU) against the reference's own outputs
(golden) and the oracle at a full Cholec80 annotation length: bit-exact."""
import numpy as np
import pytest
import torch

from oracle import labels as OL

pytestmark = pytest.mark.gpu

G = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "anticipation_golden.npz"))


@pytest.mark.parametrize("name", ["v1", "v2", "v3", "v4", "v5"])
@pytest.mark.parametrize("horizon", [5.0, 3])
def test_anticipation_gt_vs_reference_golden(cuda, name, horizon):
    from svk.labels import generate_anticipation_gt
    ph = torch.from_numpy(G[f"{name}_phases"].astype(np.int64)).to(cuda)
    out = generate_anticipation_gt(ph, horizon)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), G[f"{name}_h{horizon}"])


def test_anticipation_gt_full_video(cuda):
    """43 326 annotation rows (video 1's length, generate_phase_anticipation.py:87) of ordered phases."""
    from svk.labels import generate_anticipation_gt
    r = np.random.default_rng(1)
    T = 43326
    labels = np.minimum(np.cumsum(r.random(T) < 7 / T * 1.5), 6)
    ph = torch.from_numpy(np.stack([(labels == p).astype(np.int64) for p in range(7)]))
    out = generate_anticipation_gt(ph.to(cuda), 5.0)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), OL.anticipation_gt(ph, 5.0))
