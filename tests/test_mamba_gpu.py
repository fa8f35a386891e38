"""CausalMambaModel (mstcn.py:282-343) on the GPU: svk_mamba_conv_silu / svk_mamba_scan and the whole
model against the CPU restatement in oracle/mamba.py (float64).  Parity unpinned (mamba_ssm absent, no
golden vectors; see oracle/mamba.py).  Tolerance: the north star's per-frame logits within 1e-3 (f32),
argmax labels identical wherever the top-2 margin exceeds the tolerance."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import inputs as I, mamba as OM

pytestmark = pytest.mark.gpu


def _rand(g, *shape, scale=1.0):
    return torch.randn(*shape, generator=g, dtype=torch.float64) * scale


@pytest.mark.parametrize("seg", [None, 1 << 30, 32, 96])   # auto / one sequential pass / two-pass segments
@pytest.mark.parametrize("T", [1, 63, 64, 65, 300])
@pytest.mark.parametrize("N", [16, 32, 64])
def test_scan_kernel_vs_oracle(cuda, T, N, seg):
    from svk import ops
    g = torch.Generator().manual_seed(T * 100 + N)
    B, Di, R = 2, 48, 4                       # Di not a multiple of the per-workgroup channel count for N=64
    u = _rand(g, B, T, Di)
    xdbl = _rand(g, B, T, R + 2 * N, scale=0.5)
    z = _rand(g, B, T, Di)
    w_dt = _rand(g, Di, R, scale=0.5)
    b_dt = _rand(g, Di, scale=0.5) - 2.0
    a_neg = -torch.exp(_rand(g, Di, N, scale=0.5))
    d_skip = _rand(g, Di)
    delta = F.softplus(xdbl[..., :R] @ w_dt.t() + b_dt)
    ref = OM.selective_scan(u, delta, a_neg, xdbl[..., R:R + N], xdbl[..., R + N:], d_skip, z)
    c = lambda t: t.float().contiguous().to(cuda)
    y = ops.mamba_scan(c(u).view(B * T, Di), c(xdbl).view(B * T, -1), c(z).view(B * T, Di), c(w_dt), c(b_dt),
                       c(a_neg), c(d_skip), B, T, seg_len=seg)
    torch.cuda.synchronize()
    np.testing.assert_allclose(y.view(B, T, Di).cpu().double().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("K", [2, 3, 4])
def test_conv_silu_kernel_vs_oracle(cuda, K):
    from svk import ops
    g = torch.Generator().manual_seed(K)
    B, T, Di = 2, 70, 128
    xz = _rand(g, B * T, 2 * Di)
    w = _rand(g, Di, K, scale=0.5)
    b = _rand(g, Di, scale=0.1)
    xi = xz[:, :Di].view(B, T, Di).transpose(1, 2)
    ref = F.silu(F.conv1d(xi, w[:, None, :], b, padding=K - 1, groups=Di)[..., :T]).transpose(1, 2)
    xzd = xz.float().to(cuda)
    y = ops.mamba_conv_silu(xzd[:, :Di], w.float().to(cuda), b.float().to(cuda), B, T)
    torch.cuda.synchronize()
    np.testing.assert_allclose(y.view(B, T, Di).cpu().double().numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)


def _model(cuda, stages, layers, f_maps, f_dim, d_state, seed):
    from models import mstcn
    m = mstcn.CausalMambaModel(stages, layers, f_maps, f_dim, 14, True, mamba_d_state=d_state)
    sd = OM.init_state_dict({k: v.shape for k, v in m.state_dict().items()}, seed)
    m.load_state_dict(sd, strict=True)
    return m.to(cuda).eval(), sd


def _check_logits(out, ref):
    o, r = out.cpu().double().numpy(), ref.numpy()
    np.testing.assert_allclose(o, r, rtol=0, atol=1e-3)
    top2 = np.sort(r, axis=-2)[..., -2:, :]
    clear = (top2[..., 1, :] - top2[..., 0, :]) > 2e-3
    assert (o.argmax(-2) == r.argmax(-2))[clear].all()


@pytest.mark.parametrize("T", [1, 65, 1000])
def test_causal_mamba_vs_oracle(cuda, T):
    m, sd = _model(cuda, 4, 10, 64, 256, 64, 7)          # tecno.py:153 with the BASELINE MS-TCN config
    lfb = I.lfb(T, 256, 3)                               # [1, T, 256]
    with torch.no_grad():
        out = m(lfb.to(cuda).transpose(2, 1))            # the caller's call: model(lfb.transpose(2, 1))[-1]
    torch.cuda.synchronize()
    assert out.shape == (1, 1, 14, T)
    _check_logits(out, OM.causal_mamba(lfb.transpose(2, 1), sd, 10))


def test_causal_mamba_batch_and_small_state(cuda):
    m, sd = _model(cuda, 2, 3, 32, 2048, 16, 8)          # reference-logged f_maps=32, f_dim=2048
    x = torch.cat([I.lfb(200, 2048, 4), I.lfb(200, 2048, 5)], 0).transpose(2, 1)   # [2, 2048, 200]
    with torch.no_grad():
        out = m(x.to(cuda))
    torch.cuda.synchronize()
    assert out.shape == (1, 2, 14, 200)
    _check_logits(out, OM.causal_mamba(x, sd, 3, d_state=16))


def test_causal_mamba_prefix_property_full_length(cuda):
    """Full-length video (T = 6000, the top of the synthetic video-length range): the model is causal, so
    the logits of a 6000-frame video restricted to its first 2500 frames equal those of the 2500-frame
    prefix (to f32 rounding: the GEMM tiling may differ with the row count)."""
    m, _ = _model(cuda, 4, 10, 64, 256, 64, 9)
    lfb = I.lfb(6000, 256, 6).to(cuda)
    with torch.no_grad():
        full = m(lfb.transpose(2, 1))
        pre = m(lfb[:, :2500].transpose(2, 1))
    torch.cuda.synchronize()
    assert torch.isfinite(full).all()
    np.testing.assert_allclose(full[..., :2500].cpu().numpy(), pre.cpu().numpy(), rtol=0, atol=1e-5)


@pytest.mark.parametrize("seg", [32, 96, 256])
@pytest.mark.parametrize("N", [16, 64])
def test_ragged_scan_and_conv_vs_oracle(cuda, N, seg):
    """Ragged batch (incl. a 1-frame and an empty video, lengths not multiples of the segment): one launch
    per kernel, each video equal to the oracle on that video alone (state and conv taps restart)."""
    from svk import ops
    g = torch.Generator().manual_seed(N + seg)
    lens = [1, 0, 95, 300, 33]
    M, Di, R, K = sum(lens), 48, 4, 4
    xz = _rand(g, M, 2 * Di)
    w = _rand(g, Di, K, scale=0.5)
    b = _rand(g, Di, scale=0.1)
    xdbl = _rand(g, M, R + 2 * N, scale=0.5)
    z = _rand(g, M, Di)
    w_dt = _rand(g, Di, R, scale=0.5)
    b_dt = _rand(g, Di, scale=0.5) - 2.0
    a_neg = -torch.exp(_rand(g, Di, N, scale=0.5))
    d_skip = _rand(g, Di)
    c = lambda t: t.float().contiguous().to(cuda)
    rg = ops.mamba_ragged(lens, cuda, seg_len=seg)
    xzd = xz.float().to(cuda)
    u = ops.mamba_conv_silu(xzd[:, :Di], c(w), c(b), 1, M, ragged=rg)
    y = ops.mamba_scan(u, c(xdbl), c(z), c(w_dt), c(b_dt), c(a_neg), c(d_skip), 1, M, ragged=rg)
    torch.cuda.synchronize()
    o = 0
    for T in lens:
        if T:
            xi = xz[o:o + T, :Di].t()[None]
            uref = F.silu(F.conv1d(xi, w[:, None, :], b, padding=K - 1, groups=Di)[..., :T]).transpose(1, 2)
            np.testing.assert_allclose(u[o:o + T].cpu().double().numpy(), uref[0].numpy(), rtol=1e-5, atol=1e-5)
            uu = u[o:o + T].cpu().double()[None]
            xd = xdbl[o:o + T][None]
            delta = F.softplus(xd[..., :R] @ w_dt.t() + b_dt)
            ref = OM.selective_scan(uu, delta, a_neg, xd[..., R:R + N], xd[..., R + N:], d_skip, z[o:o + T][None])
            np.testing.assert_allclose(y[o:o + T].cpu().double().numpy(), ref[0].numpy(), rtol=1e-4, atol=1e-4)
        o += T


def test_causal_mamba_ragged_videos(cuda):
    """forward_videos over a ragged batch == the caller's per-video forward, and == the oracle."""
    m, sd = _model(cuda, 4, 10, 64, 256, 64, 7)
    lens = [700, 1, 65, 1500]
    feats = torch.cat([I.lfb(T, 256, 30 + i)[0] for i, T in enumerate(lens)], 0)
    with torch.no_grad():
        out = m.forward_videos(feats.to(cuda), lens)
        per = [m(f[None].to(cuda).transpose(2, 1)) for f in torch.split(feats, lens)]
    torch.cuda.synchronize()
    assert out.shape == (sum(lens), 14)
    for T, got, one, f in zip(lens, m.split_videos(out, lens), per, torch.split(feats, lens)):
        assert got.shape == (1, 1, 14, T)
        np.testing.assert_allclose(got.cpu().numpy(), one.cpu().numpy(), rtol=0, atol=2e-5)
        if T <= 700:
            _check_logits(got, OM.causal_mamba(f[None].transpose(2, 1), sd, 10))
