"""CausalMambaModel oracle (oracle/mamba.py) — CPU checks.  Parity unpinned: mamba_ssm is absent, so the
restated selective scan is checked against properties of the published recurrence instead of golden
vectors: (1) with time-invariant delta/B/C the scan equals the convolution with the powers of
exp(delta A) (the S4 convolutional view), (2) causality, (3) per-video state reset."""
import math

import torch
import torch.nn.functional as F

from oracle import mamba as OM


def test_scan_time_invariant_equals_convolution():
    g = torch.Generator().manual_seed(0)
    Bt, L, Di, N = 2, 40, 3, 8
    u = torch.randn(Bt, L, Di, generator=g, dtype=torch.float64)
    z = torch.randn(Bt, L, Di, generator=g, dtype=torch.float64)
    A = -torch.rand(Di, N, generator=g, dtype=torch.float64) - 0.1
    dlt = torch.rand(Di, generator=g, dtype=torch.float64) * 0.5 + 0.05
    Bv = torch.randn(N, generator=g, dtype=torch.float64)
    Cv = torch.randn(N, generator=g, dtype=torch.float64)
    D = torch.randn(Di, generator=g, dtype=torch.float64)
    y = OM.selective_scan(u, dlt.expand(Bt, L, Di), A, Bv.expand(Bt, L, N), Cv.expand(Bt, L, N), D, z)
    kern = torch.stack([(Cv * torch.exp(dlt[:, None] * A) ** k * dlt[:, None] * Bv).sum(-1) for k in range(L)], 0)
    ref = torch.zeros_like(u)
    for t in range(L):
        ref[:, t] = (kern[:t + 1].flip(0) * u[:, :t + 1]).sum(1)
    ref = (ref + u * D) * F.silu(z)
    torch.testing.assert_close(y, ref, rtol=1e-10, atol=1e-10)


def test_model_is_causal():
    sd = OM.init_state_dict(OM.mamba_shapes(32, 16, 2, 14, d_state=16), 3)
    x = torch.randn(1, 32, 50, generator=torch.Generator().manual_seed(1))
    y = OM.causal_mamba(x, sd, 2, d_state=16)
    x2 = x.clone()
    x2[:, :, 30:] += 1.0
    y2 = OM.causal_mamba(x2, sd, 2, d_state=16)
    assert y.shape == (1, 1, 14, 50)
    torch.testing.assert_close(y[..., :30], y2[..., :30], rtol=0, atol=0)
    assert (y[..., 30:] - y2[..., 30:]).abs().max() > 1e-3


def test_videos_are_independent():
    sd = OM.init_state_dict(OM.mamba_shapes(32, 16, 1, 7, d_state=16), 4)
    x = torch.randn(2, 32, 20, generator=torch.Generator().manual_seed(2))
    y = OM.causal_mamba(x, sd, 1, d_state=16)
    torch.testing.assert_close(y[:, 1:2], OM.causal_mamba(x[1:2], sd, 1, d_state=16))


def test_init_follows_mamba_simple():
    sd = OM.init_state_dict(OM.mamba_shapes(256, 64, 1, 14), 0)
    assert torch.equal(sd["blocks.0.A_log"][5], torch.log(torch.arange(1, 65, dtype=torch.float32)))
    dt = F.softplus(sd["blocks.0.dt_proj.bias"].double())
    assert dt.min() >= 1e-4 - 1e-9 and dt.max() <= 0.1 + 1e-6
    assert sd["blocks.0.dt_proj.weight"].shape == (128, math.ceil(64 / 16))
