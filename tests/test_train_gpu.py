"""Training-step parity on the GPU (§8 a13): each backward kernel against torch autograd (f32 on the
CPU, same seeded inputs), then the whole frozen-backbone step (svk.train.EVPTrainStep) against the
oracle's autograd restatement (oracle/train_evp.py) with identical DropPath / Dropout2d masks.

Tolerances: f32 kernels 1e-4..1e-3 relative to the tensor's max magnitude (atomics reorder sums);
full f32 step: every trainable gradient within 2e-3 of max|g| of the fp64 oracle, losses within
1e-4 relative; bf16 step: per-tensor gradient cosine similarity >= 0.98 (median >= 0.995) against the
fp64 oracle (bf16 is the throughput dtype; the reference itself trains under fp16 autocast).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import inputs as I, params as P, train_evp as TR

pytestmark = pytest.mark.gpu


def _close(a, b, tol):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    scale = max(b.abs().max().item(), 1e-6)
    err = (a - b).abs().max().item()
    assert err <= tol * scale, f"max err {err:.3e} > {tol} * {scale:.3e}"


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


@pytest.mark.parametrize("M,C", [(300, 64), (77, 320), (49, 512)])
def test_layernorm_bwd(cuda, M, C):
    from svk import ops
    x, dy, r = _rand(M, C, seed=1), _rand(M, C, seed=2), _rand(M, C, seed=3)
    g, b = 1 + 0.1 * _rand(C, seed=4), 0.1 * _rand(C, seed=5)
    xr = x.clone().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    F.layer_norm(xr, (C,), gr, br, 1e-6).backward(dy)
    dg = torch.zeros(C, device=cuda)
    db = torch.zeros(C, device=cuda)
    dx = ops.layernorm_bwd(x.to(cuda), dy.to(cuda), g.to(cuda), 1e-6, dres=r.to(cuda), dgamma=dg, dbeta=db)
    _close(dx, xr.grad + r, 1e-4)
    _close(dg, gr.grad, 1e-4)
    _close(db, br.grad, 1e-4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,C,affine,res", [(17248, 320, True, False), (4312, 512, True, True), (68992, 128, True, False),
                                            (5003, 64, False, True), (1001, 320, False, False)])
def test_layernorm_bwd_many_rows(cuda, dt, M, C, affine, res):
    """The vectorised backward at the train step's row counts (B = 88): waves walking many row groups (the affine
    grid is capped at 256 blocks; round 6 issues four row groups' loads per iteration), ragged tails, with and
    without the residual gradient and the affine gradients."""
    from svk import ops
    x, dy, r = _rand(M, C, seed=11), _rand(M, C, seed=12), _rand(M, C, seed=13)
    g, b = 1 + 0.1 * _rand(C, seed=14), 0.1 * _rand(C, seed=15)
    xd, dyd, rd = (t.to(dt).double() for t in (x, dy, r))
    xr = xd.clone().requires_grad_(True)
    gr, br = g.double().requires_grad_(True), b.double().requires_grad_(True)
    F.layer_norm(xr, (C,), gr, br, 1e-6).backward(dyd)
    dg = torch.zeros(C, device=cuda) if affine else None
    db = torch.zeros(C, device=cuda) if affine else None
    dx = ops.layernorm_bwd(x.to(cuda, dt), dy.to(cuda, dt), g.to(cuda), 1e-6, dres=r.to(cuda, dt) if res else None,
                           dgamma=dg, dbeta=db)
    tol = 1e-4 if dt == torch.float32 else 2e-2
    _close(dx, xr.grad + (rd if res else 0), tol)
    if affine:
        _close(dg, gr.grad, tol)
        _close(db, br.grad, tol)


@pytest.mark.parametrize("act", ["gelu", "relu"])
def test_act_bwd(cuda, act):
    from svk import ops
    u, dy = _rand(1000, seed=1), _rand(1000, seed=2)
    ur = u.clone().requires_grad_(True)
    (F.gelu(ur) if act == "gelu" else F.relu(ur)).backward(dy)
    _close(ops.act_bwd(u.to(cuda), dy.to(cuda), act), ur.grad, 1e-5)


@pytest.mark.parametrize("M,C", [(88 * 49, 2048), (1000, 64)])
def test_batchnorm_train_fwd_bwd(cuda, M, C):
    from svk import ops
    x, dy = _rand(M, C, seed=1), _rand(M, C, seed=2)
    g, b = 1 + 0.1 * _rand(C, seed=3), 0.1 * _rand(C, seed=4)
    xr = x.clone().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = F.relu(F.batch_norm(xr, None, None, gr, br, True, 0.1, 1e-5))
    y.backward(dy)
    xc = x.to(cuda)
    s1, s2 = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
    ops.colstats(xc, s1, s2)
    yc = ops.bn_apply(xc, s1, s2, g.to(cuda), b.to(cuda), 1e-5, act="relu")
    _close(yc, y, 1e-4)
    dg, db = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
    dx = ops.bn_bwd(xc, dy.to(cuda), s1, s2, g.to(cuda), b.to(cuda), 1e-5, dg, db, relu=True)
    _close(dx, xr.grad, 1e-3)
    _close(dg, gr.grad, 1e-3)
    _close(db, br.grad, 1e-3)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    ops.bn_update_running(s1, s2, M, rm, rv, 0.1)
    _close(rm, 0.1 * x.mean(0), 1e-4)
    _close(rv, 0.9 + 0.1 * x.var(0, unbiased=True), 1e-4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,C", [(65536, 256), (4312, 2048), (7, 24), (0, 64)])
def test_colstats_set_equals_colstats(cuda, dt, M, C):
    """svk_colstats_set (the train step's BN statistics written into [2, C], no zero-fill launches) gives the
    bits of svk_colstats accumulated into zeroed buffers; M = 0 writes zeros."""
    from svk import ops
    x = (torch.randn(M, C, generator=torch.Generator().manual_seed(3)) * 2 + 0.3).to(cuda).to(dt)
    s1, s2 = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
    if M:
        ops.colstats(x, s1, s2)
    got = ops.colstats_set(x) if M else ops.colstats_set(x, out=torch.full((2, C), 5.0, device=cuda))
    torch.cuda.synchronize()
    assert torch.equal(got[0], s1) and torch.equal(got[1], s2)


def test_batchnorm_stats_bit_reproducible(cuda):
    """Round-5 root cause of the intermittent f32 train-gradient failure: the BN batch statistics
    were summed with per-block f32 atomics, so the last bit of the batch mean depended on the order the blocks
    arrived; a pre-ReLU value within that rounding of 0 then flipped its ReLU gate from run to run, and through
    the BN backward the flip moved the whole channel's gradient (head.linear_fuse.conv.weight 1.6 % off).  The
    column reductions are now two-phase and fixed-order.  Here 65 536 rows (1 024 blocks per column) whose sums
    are order-sensitive, and one element per column placed exactly on its column mean (pre-ReLU 0 with beta 0):
    20 repetitions must give bitwise-identical sums, ReLU outputs, dX and dgamma / dbeta.  With the atomic
    reduction this fails on the first repetitions (different last bits of s1 / s2)."""
    from svk import ops
    M, C = 65536, 256
    g = torch.Generator().manual_seed(7)
    x = torch.randn(M, C, generator=g) * 3 + 0.5
    x[123] = x.double().mean(0).float()            # on (or within one rounding of) the column mean
    x = x.to(cuda)
    dy = torch.randn(M, C, generator=g).to(cuda)
    gam, bet = torch.ones(C, device=cuda), torch.zeros(C, device=cuda)
    ref = None
    for _ in range(20):
        s1, s2 = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
        ops.colstats(x, s1, s2)
        y = ops.bn_apply(x, s1, s2, gam, bet, 1e-5, act="relu")
        dg, db = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
        dx = ops.bn_bwd(x, dy, s1, s2, gam, bet, 1e-5, dg, db, relu=True)
        got = [t.clone() for t in (s1, s2, y, dx, dg, db)]
        if ref is None:
            ref = got
            continue
        for name, a, b in zip(("sum", "sumsq", "relu(bn)", "dX", "dgamma", "dbeta"), got, ref):
            assert torch.equal(a, b), f"{name} differs between identical calls: max {(a - b).abs().max().item():.3e}"
    # the gradient buffers accumulate (+=): a second call adds the same sums, dX does not change
    dx2 = ops.bn_bwd(x, dy, ref[0], ref[1], gam, bet, 1e-5, dg, db, relu=True)
    assert torch.equal(dx2, ref[3])
    torch.testing.assert_close(db, 2 * ref[5])


@pytest.mark.parametrize("H,W", [(56, 56), (28, 28), (14, 14)])
def test_resize_bilinear_bwd(cuda, H, W):
    from svk import ops
    B, C = 2, 24
    x = _rand(B, C, H, W, seed=1).requires_grad_(True)
    dy = _rand(B, C, 7, 7, seed=2)
    F.interpolate(x, (7, 7), mode="bilinear", align_corners=False).backward(dy)
    dyt = dy.permute(0, 2, 3, 1).reshape(B, 49, C).contiguous().to(cuda)
    dx = torch.zeros(B, H * W, C, device=cuda)
    ops.resize_bilinear_bwd(dyt, H, W, 7, 7, dx)
    _close(dx, x.grad.permute(0, 2, 3, 1).reshape(B, H * W, C), 1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(1000, 64, 256), (4312, 2048, 512), (37, 7, 512), (500, 48, 40),
                                   (69001, 256, 136), (3000, 200, 72)])
def test_gemm_wgrad(cuda, dt, M, N, K):
    from svk import ops
    dy, x = _rand(M, N, seed=1), _rand(M, K, seed=2)
    dw = torch.full((N, K), 0.5, device=cuda)
    db = torch.full((N,), 0.25, device=cuda)
    ops.gemm_wgrad(dy.to(cuda, dt), x.to(cuda, dt), dw, db)
    ref = dy.to(dt).double().t() @ x.to(dt).double() + 0.5
    _close(dw, ref, 1e-5 if dt == torch.float32 else 1e-2)
    _close(db, dy.to(dt).double().sum(0) + 0.25, 1e-5 if dt == torch.float32 else 1e-2)
    # the 16-bit path is f32-accumulated from exactly representable inputs: much tighter than 1e-2
    if dt != torch.float32:
        err = float((dw.double().cpu() - ref.cpu()).abs().max() / ref.abs().max().cpu())
        assert err < 1e-5, f"relative error {err}"


def _conv_case(B, Cin, H, Cout, k, s, seed):
    x = _rand(B, Cin, H, H, seed=seed)
    w = _rand(Cout, Cin, k, k, seed=seed + 1, scale=0.1)
    return x, w


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,Cin,H,Cout,k,s", [(2, 16, 56, 32, 3, 2), (2, 64, 56, 128, 3, 2), (2, 3, 224, 16, 7, 4),
                                              (3, 128, 28, 320, 3, 2)])
def test_conv_wgrad_dgrad(cuda, dt, B, Cin, H, Cout, k, s):
    from svk import ops
    from svk.pack import pad_channels
    x, w = _conv_case(B, Cin, H, Cout, k, s, 3)
    xr, wr = x.to(dt).double().requires_grad_(True), w.to(dt).double().requires_grad_(True)
    y = F.conv2d(xr, wr, stride=s, padding=k // 2)
    dy = _rand(*y.shape, seed=9).to(dt).double()
    y.backward(dy)
    cp = pad_channels(Cin)
    xn = ops.nchw_to_nhwc(x.to(cuda), dt, cpad=cp)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    dwp = torch.zeros(Cout, k * k * cp, device=cuda)
    dbias = torch.zeros(Cout, device=cuda)
    ops.conv2d_wgrad(xn, dyn, k, s, k // 2, dwp, dbias)
    if dt != torch.float32:   # the 16-bit conv weight gradient runs on wgrad_pk's im2col DMA path
        assert ops._last_kernel().startswith("wgrad_pk") and "conv" in ops._last_kernel(), ops._last_kernel()
    dw = dwp.view(Cout, k, k, cp)[..., :Cin].permute(0, 3, 1, 2)
    tol = 1e-4 if dt == torch.float32 else 2e-2
    _close(dw, wr.grad, tol)
    _close(dbias, dy.sum((0, 2, 3)), tol)
    if Cin >= 8:
        wd = w.permute(1, 2, 3, 0).reshape(Cin, k * k * Cout).to(cuda, dt).contiguous()
        res = _rand(B, H, H, Cin, seed=11).to(cuda, dt)
        dx = ops.conv2d_dgrad(dyn, wd, H, H, Cin, k, s, k // 2, residual=res)
        _close(dx, xr.grad.permute(0, 2, 3, 1) + res.double().cpu(), tol)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,Cin,H,Cout,k,s", [(2, 64, 56, 128, 3, 2), (3, 128, 28, 320, 3, 2), (2, 320, 14, 512, 3, 2),
                                              (2, 16, 56, 32, 3, 2), (2, 8, 64, 16, 7, 4), (1, 24, 15, 40, 3, 2),
                                              (2, 16, 13, 8, 3, 1), (1, 8, 17, 16, 5, 2)])
@pytest.mark.parametrize("residual", [True, False])
def test_conv_dgrad_col2im(cuda, dt, B, Cin, H, Cout, k, s, residual):
    """The train step's conv data gradient as per-tap GEMM + col2im gather (exact MAC count) == fp64 autograd
    and == the transposed-conv gather GEMM it replaces, at the 16-bit tolerance (odd sizes: output maps whose
    last input rows / columns receive fewer taps)."""
    from svk import ops
    x, w = _conv_case(B, Cin, H, Cout, k, s, 5)
    xr, wr = x.to(dt).double().requires_grad_(True), w.to(dt).double()
    y = F.conv2d(xr, wr, stride=s, padding=k // 2)
    dy = _rand(*y.shape, seed=13).to(dt).double()
    y.backward(dy)
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    wc = w.permute(2, 3, 1, 0).reshape(k * k * Cin, Cout).to(cuda, dt).contiguous()
    res = _rand(B, H, H, Cin, seed=17).to(cuda, dt) if residual else None
    dx = ops.conv2d_dgrad_col2im(dyn, wc, H, H, Cin, k, s, k // 2, residual=res)
    ref = xr.grad.permute(0, 2, 3, 1) + (res.double().cpu() if residual else 0.0)
    _close(dx, ref, 2e-2)
    wd = w.permute(1, 2, 3, 0).reshape(Cin, k * k * Cout).to(cuda, dt).contiguous()
    old = ops.conv2d_dgrad(dyn, wd, H, H, Cin, k, s, k // 2, residual=res)
    _close(dx, old.double().cpu(), 2e-2)


def test_patchify_adjoint(cuda):
    """sr-conv data gradient: GEMM with the (i, j, ci) x co packed weight + unpatchify."""
    from svk import ops
    B, C, H, r = 2, 64, 56, 8
    x = _rand(B, C, H, H, seed=1).double().requires_grad_(True)
    w = _rand(C, C, r, r, seed=2, scale=0.05).double()
    y = F.conv2d(x, w, stride=r)
    dy = _rand(*y.shape, seed=3).double()
    y.backward(dy)
    wd = w.permute(2, 3, 1, 0).reshape(r * r * C, C).float().to(cuda)
    dyt = dy.permute(0, 2, 3, 1).reshape(-1, C).float().to(cuda)
    dp = ops.gemm(dyt, wd)
    dx = torch.empty(B, H, H, C, device=cuda)
    ops.unpatchify(dp, B, H // r, H // r, r, C, dx)
    _close(dx, x.grad.permute(0, 2, 3, 1), 1e-5)
    # the same adjoint stored straight from the GEMM epilogue, accumulating onto a residual
    res = _rand(B, H, H, C, seed=4).to(cuda)
    dx2 = res.clone()
    ops.gemm_unpatchify(dyt, wd, dx2, r, residual=dx2)
    _close(dx2, x.grad.permute(0, 2, 3, 1) + res.cpu(), 1e-5)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,C,H,r", [(3, 64, 56, 8), (2, 128, 28, 4), (2, 320, 14, 2), (1, 24, 12, 3)])
def test_unpatchify_split_vs_fused(cuda, dt, B, C, H, r):
    """The training step's split sr-conv data gradient (GEMM -> 16-byte scatter-add, svk_unpatchify's
    vectorised path; C = 24 takes it too) == the fused scatter epilogue of svk_gemm_unpatchify: both round the
    GEMM output to the storage type and add the residual in f32, so the results agree to one ulp."""
    from svk import ops
    K = C
    dyt = _rand(B * (H // r) ** 2, K, seed=5).to(cuda, dt)
    wd = (_rand(r * r * C, K, seed=6) * K ** -0.5).to(cuda, dt)
    res = _rand(B, H, H, C, seed=7).to(cuda, dt)
    fused = res.clone()
    ops.gemm_unpatchify(dyt, wd, fused, r, residual=fused)
    split = res.clone()
    ops.unpatchify(ops.gemm(dyt, wd), B, H // r, H // r, r, C, split, accumulate=True)
    plain = torch.zeros_like(res)
    ops.unpatchify(ops.gemm(dyt, wd), B, H // r, H // r, r, C, plain)
    torch.cuda.synchronize()
    ref = (dyt.double() @ wd.double().t()).view(B, H // r, H // r, r, r, C).permute(0, 1, 3, 2, 4, 5)
    ref = ref.reshape(B, H, H, C)
    ulp = 2.0 ** -7 if dt == torch.bfloat16 else 2.0 ** -10
    for got, want in ((split, fused.double()), (plain, ref), (split, ref + res.double())):
        d = (got.double() - want).abs() / want.abs().clamp_min(1.0)
        assert float(d.max()) <= 2 * ulp, float(d.max())


@pytest.mark.parametrize("tkern", ["1", "0"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Nq,Nk,heads,hd", [(3136, 49, 1, 64), (196, 196, 8, 40), (49, 49, 8, 64), (100, 30, 2, 16),
                                            (196, 196, 5, 64), (130, 100, 3, 32), (70, 150, 2, 64)])
def test_attention_bwd(cuda, monkeypatch, tkern, dt, Nq, Nk, heads, hd):
    """bf16: the transposed-score dQ kernel (attn_bwd_dq_t, default) and the round-5 one (SVK_ATTN_BWD_T=0), every
    key-chunk count NKC = 1..4 and both head-dim paddings; f32: the LDS scalar kernel."""
    from svk import ops
    if dt == torch.float32 and tkern == "0":
        pytest.skip("the switch selects between bf16 kernels")
    monkeypatch.setenv("SVK_ATTN_BWD_T", tkern)
    B, C = 2, heads * hd
    q, k, v = _rand(B, Nq, C, seed=1), _rand(B, Nk, C, seed=2), _rand(B, Nk, C, seed=3)
    do = _rand(B, Nq, C, seed=4)
    scale = hd ** -0.5
    qr, kr, vr = (t.to(dt).double().requires_grad_(True) for t in (q, k, v))
    sp = lambda t, n: t.reshape(B, n, heads, hd).transpose(1, 2)
    a = (sp(qr, Nq) @ sp(kr, Nk).transpose(-1, -2) * scale).softmax(-1)
    o = (a @ sp(vr, Nk)).transpose(1, 2).reshape(B, Nq, C)
    o.backward(do.to(dt).double())
    qc, kc, vc = (t.to(cuda, dt) for t in (q, k, v))
    oc = ops.attention(qc, kc, vc, heads, scale)
    dkv = torch.zeros(B, Nk, 2 * C, device=cuda, dtype=dt)
    dq, _, _ = ops.attention_bwd(qc, kc, vc, oc, do.to(cuda, dt), heads, scale, dkv[:, :, :C], dkv[:, :, C:])
    tol = 1e-4 if dt == torch.float32 else 3e-2
    _close(dq, qr.grad, tol)
    _close(dkv[:, :, :C], kr.grad, tol)
    _close(dkv[:, :, C:], vr.grad, tol)


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("B,Nq,Nk,heads,hd", [(3, 3136, 49, 8, 64), (5, 257, 49, 5, 64), (4, 700, 33, 6, 32)])
def test_attention_bwd_fused_multichunk(cuda, monkeypatch, fused, B, Nq, Nk, heads, hd):
    """The fused bf16 backward (<= 64 keys) with several 64-query chunks per workgroup and a partial last
    chunk: dQ, dK, dV against fp64 autograd (dK / dV are reduced in registers over a workgroup's chunks and
    across workgroups by f32 atomics)."""
    from svk import ops
    monkeypatch.setenv("SVK_ATTN_BWD_FUSED", fused)   # read by svk_attention_bwd at every call
    dt, C = torch.bfloat16, heads * hd
    q, k, v = _rand(B, Nq, C, seed=11), _rand(B, Nk, C, seed=12), _rand(B, Nk, C, seed=13)
    do = _rand(B, Nq, C, seed=14)
    scale = hd ** -0.5
    qr, kr, vr = (t.to(dt).double().requires_grad_(True) for t in (q, k, v))
    sp = lambda t, n: t.reshape(B, n, heads, hd).transpose(1, 2)
    a = (sp(qr, Nq) @ sp(kr, Nk).transpose(-1, -2) * scale).softmax(-1)
    o = (a @ sp(vr, Nk)).transpose(1, 2).reshape(B, Nq, C)
    o.backward(do.to(dt).double())
    qc, kc, vc = (t.to(cuda, dt) for t in (q, k, v))
    oc = ops.attention(qc, kc, vc, heads, scale)
    dkv = torch.zeros(B, Nk, 2 * C, device=cuda, dtype=dt)
    dq, _, _ = ops.attention_bwd(qc, kc, vc, oc, do.to(cuda, dt), heads, scale, dkv[:, :, :C], dkv[:, :, C:])
    _close(dq, qr.grad, 3e-2)
    _close(dkv[:, :, :C], kr.grad, 3e-2)
    _close(dkv[:, :, C:], vr.grad, 3e-2)


def test_phase_loss_and_sgd(cuda):
    from svk import ops
    B = 88
    z, a = _rand(B, 7, seed=1, scale=3), _rand(B, 7, seed=2, scale=2)
    lab = torch.randint(0, 7, (B,), generator=torch.Generator().manual_seed(3))
    at = torch.rand(B, 7, generator=torch.Generator().manual_seed(4))
    zr, ar = z.clone().requires_grad_(True), a.clone().requires_grad_(True)
    lp = F.cross_entropy(zr, lab, reduction="sum")
    la = F.smooth_l1_loss(ar, at, reduction="sum")
    (lp + la).backward()
    loss, dl, da = ops.phase_loss(z.to(cuda), a.to(cuda), lab.to(cuda), at.to(cuda))
    _close(loss, torch.stack([lp, la]), 1e-5)
    _close(dl, zr.grad, 1e-5)
    _close(da, ar.grad, 1e-5)
    # SGD: two steps against torch.optim.SGD
    p0, g1, g2 = _rand(1000, seed=5), _rand(1000, seed=6), _rand(1000, seed=7)
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.SGD([pt], lr=5e-4, momentum=0.9, dampening=0.0, weight_decay=1e-5, nesterov=False)
    pc, buf = p0.to(cuda), torch.zeros(1000, device=cuda)
    for i, g in enumerate((g1, g2)):
        pt.grad = g.clone()
        opt.step()
        ops.sgd(pc, g.to(cuda), buf, 5e-4, 0.9, 0.0, 1e-5, False, first=i == 0)
    _close(pc, pt.detach(), 1e-6)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", ["gelu", "relu"])
def test_gemm_activation_backward_epilogue(cuda, dt, act):
    from svk import ops
    M, N, K = 300, 96, 64
    a, w, u = _rand(M, K, seed=1), _rand(N, K, seed=2, scale=0.1), _rand(M, N, seed=3)
    s = torch.rand(3, generator=torch.Generator().manual_seed(4))
    ur = u.to(dt).double().requires_grad_(True)
    (F.gelu(ur) if act == "gelu" else F.relu(ur)).backward(a.to(dt).double() @ w.to(dt).double().t()
                                                           * s.double().repeat_interleave(100)[:, None])
    out = ops.gemm(a.to(cuda, dt), w.to(cuda, dt), row_scale=s.to(cuda), rows_per=100, dact=act,
                   dact_src=u.to(cuda, dt))
    _close(out, ur.grad, 1e-5 if dt == torch.float32 else 2e-2)


@pytest.mark.parametrize("M,N,K", [(88, 512, 2048), (88, 2048, 512), (256, 512, 2048), (37, 259, 130)])
@pytest.mark.parametrize("mode", ["relu_bias", "residual", "dact_scale"])
def test_gemm_f32_smallm(cuda, M, N, K, mode):
    """The few-row f32 GEMM (the train step's f32 heads: 16 x 16 tiles, K split over 4 waves) with each
    epilogue the head uses, against fp64."""
    from svk import ops
    a, w = _rand(M, K, seed=11), _rand(N, K, seed=12, scale=K ** -0.5)
    b, r, u = _rand(N, seed=13), _rand(M, N, seed=14), _rand(M, N, seed=15)
    s = torch.rand(M, generator=torch.Generator().manual_seed(16))
    ref = a.double() @ w.double().t()
    if mode == "relu_bias":
        out = ops.gemm(a.to(cuda), w.to(cuda), b.to(cuda), act="relu")
        ref = torch.relu(ref + b.double())
    elif mode == "residual":
        out = ops.gemm(a.to(cuda), w.to(cuda), residual=r.to(cuda))
        ref = ref + r.double()
    else:
        out = ops.gemm(a.to(cuda), w.to(cuda), row_scale=s.to(cuda), rows_per=1, dact="relu", dact_src=u.to(cuda))
        ref = ref * s.double()[:, None] * (u.double() > 0)
    assert ops._last_kernel().startswith("gemm_f32_smallm"), ops._last_kernel()
    _close(out, ref, 1e-5)


@pytest.mark.parametrize("M,N,K", [(5000, 16, 16), (3001, 64, 16), (3000, 16, 64), (2048, 32, 128),
                                   (2100, 48, 40), (2500, 10, 12), (4096, 64, 128)])
@pytest.mark.parametrize("mode", ["plain", "gelu_bias", "residual", "dact"])
def test_gemm_skinny(cuda, M, N, K, mode):
    from svk import ops
    a, w = _rand(M, K, seed=1).bfloat16(), _rand(N, K, seed=2, scale=0.2).bfloat16()
    b, r, u = _rand(N, seed=3), _rand(M, N, seed=4).bfloat16(), _rand(M, N, seed=5).bfloat16()
    kw = {}
    ref = a.double() @ w.double().t()
    if mode == "gelu_bias":
        kw = dict(bias=b.to(cuda), act="gelu")
        ref = F.gelu(ref + b.double())
    elif mode == "residual":
        kw = dict(residual=r.to(cuda))
        ref = ref + r.double()
    elif mode == "dact":
        kw = dict(dact="gelu", dact_src=u.to(cuda))
        ur = u.double().requires_grad_(True)
        F.gelu(ur).backward(ref)
        ref = ur.grad
    out = ops.gemm_skinny(a.to(cuda), w.to(cuda), **kw)
    _close(out, ref, 2e-2)


@pytest.mark.parametrize("M,N,K", [(5000, 64, 16), (5000, 16, 16), (3000, 128, 32), (3000, 32, 128),
                                   (2777, 48, 40), (4096, 16, 64), (2500, 10, 12)])
def test_wgrad_skinny(cuda, M, N, K):
    from svk import ops
    dy, x = _rand(M, N, seed=1).bfloat16(), _rand(M, K, seed=2).bfloat16()
    dw = torch.full((N, K), 0.5, device=cuda)
    db = torch.full((N,), 0.25, device=cuda)
    assert ops._skinny_wgrad_ok(dy.to(cuda), x.to(cuda), M, N, K)
    ops.gemm_wgrad(dy.to(cuda), x.to(cuda), dw, db)
    _close(dw, dy.double().t() @ x.double() + 0.5, 1e-3)
    _close(db, dy.double().sum(0) + 0.25, 1e-3)


def test_gemm_row_scale_and_dwconv_pre(cuda):
    from svk import ops
    B, N, K, C = 4, 49, 64, 32
    a, w, r = _rand(B * N, K, seed=1), _rand(C, K, seed=2, scale=0.1), _rand(B * N, C, seed=3)
    s = torch.tensor([0.0, 1.25, 1.25, 0.0])
    out = ops.gemm(a.to(cuda), w.to(cuda), residual=r.to(cuda), row_scale=s.to(cuda), rows_per=N)
    ref = (a @ w.t()) * s.repeat_interleave(N)[:, None] + r
    _close(out, ref, 1e-5)
    x = _rand(2, 7, 7, 64, seed=4).to(cuda)
    taps, bias = _rand(9, 64, seed=5).to(cuda), _rand(64, seed=6).to(cuda)
    pre = torch.empty_like(x)
    y = ops.dwconv3x3(x, taps, bias, act="gelu", pre_out=pre)
    _close(pre, ops.dwconv3x3(x, taps, bias), 1e-6)
    _close(y, F.gelu(pre), 1e-5)


def test_pack_params_gather(cuda):
    """Batched gather: transposes and conv repacks with channel padding."""
    import numpy as np
    from svk.train import _PackTable
    w1 = _rand(5, 3, seed=1)
    w2 = _rand(16, 3, 7, 7, seed=2)
    flat = torch.cat([w1.reshape(-1), w2.reshape(-1)]).to(cuda)
    t = _PackTable(torch.float32)
    i1 = t.add(0, (3, 5), (1, 3))
    i2 = t.add(15, (16, 7, 7, 8), (3 * 49, 7, 1, 49), (16, 7, 7, 3))
    t.finalize(cuda)
    t.run(flat)
    _close(t.tensors[i1], w1.t(), 0)
    ref = F.pad(w2.permute(0, 2, 3, 1), (0, 5))
    _close(t.tensors[i2], ref, 0)


# ---- the full step --------------------------------------------------------------------------------

def _train_inputs(B, seed):
    g = torch.Generator().manual_seed(seed + 100)
    return (I.frames(B, seed), I.segmaps(B, seed), I.flow(B, seed), torch.randint(0, 7, (B,), generator=g),
            torch.rand(B, 7, generator=g))


def _build(variant, cuda, dtype, seed=0):
    from models import mix_transformer_evp as mte
    from svk.train import EVPTrainStep
    m = getattr(mte, variant)()
    sd = P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, seed)
    m.load_state_dict(sd)
    m = m.to(cuda)
    return m, sd, EVPTrainStep(m, dtype=dtype)


def _gpu_relu_gates(tr, sv):
    """The ReLU gates the GPU step took, in the oracle's layouts (oracle/train_evp.py forward_train sites): flow
    BN + ReLU outputs (NHWC saved -> NCHW), the head's BN + ReLU recomputed by the same kernel from the saved
    pre-BN map and batch sums ([B*49, 2048] -> [B, 2048, 7, 7]), and the fc / fc_ant hidden ReLUs."""
    from svk import ops
    from svk.train import BN_EPS
    B = sv["B"]
    gates = {}
    for i, L in enumerate(sv["flow"], start=1):
        gates[f"flow_encoder.bn{i}"] = (L["y"] > 0).permute(0, 3, 1, 2).cpu()
    hd = sv["head"]
    bn = "head.linear_fuse.bn"
    yb = ops.bn_apply(hd["Z"], hd["s1"], hd["s2"], tr.P(bn + ".weight"), tr.P(bn + ".bias"), BN_EPS, act="relu")
    gates[bn] = (yb > 0).view(B, 7, 7, -1).permute(0, 3, 1, 2).cpu()
    gates["head.fc.0"], gates["head.fc_ant.0"] = (hd["hs"][0] > 0).cpu(), (hd["hs"][1] > 0).cpu()
    return gates


@pytest.mark.parametrize("variant", ["mit_b0_evp", "mit_b2_evp", "mit_b3_evp"])
def test_train_step_grads_fp32_vs_oracle(cuda, variant):
    """f32 gradients of every trainable tensor vs fp64 autograd through the oracle; mit_b3_evp is the model
    the reference's own scripts train (train_evp.py:362, finetune_evp.py:273).

    ReLU kinks: a BN + ReLU output within f32 rounding of 0 has no well-defined gradient branch (the fp64 oracle
    and an f32 implementation may land on different sides, and a flipped gate moves the whole channel's BN
    gradient — the round-4 intermittent failure).  The oracle is therefore evaluated on the GPU's
    own gates, after checking that the GPU and the oracle agree on every gate whose pre-activation is farther
    than 1e-5 standard deviations from the kink."""
    B = 3
    m, sd, tr = _build(variant, cuda, torch.float32)
    tr.keep_saved = True
    x, y, fl, lab, ant_t = _train_inputs(B, 1)
    masks = TR.make_masks(B, variant, seed=5)
    # make sure the draw actually drops something (stochastic depth and Dropout2d both exercised)
    assert any((a == 0).any() or (b == 0).any() for st in masks["blocks"] for a, b in st)
    loss, logits, ant = tr.forward_backward(x.to(cuda), y.to(cuda), fl.to(cuda), lab.to(cuda), ant_t.to(cuda),
                                            masks=masks)
    torch.cuda.synchronize()
    gates = _gpu_relu_gates(tr, tr.last_saved)
    pre = {}
    lp, la, grads, stats = TR.loss_and_grads(x, y, fl, lab, ant_t, sd, variant, masks, gates=gates, pre=pre)
    flips = []
    for site, gt in gates.items():
        p = pre[site]
        assert p.shape == gt.shape, (site, p.shape, gt.shape)
        dis = gt != (p > 0)
        if dis.any():
            far = dis & (p.abs() > 1e-5 * p.std())
            assert not far.any(), f"{site}: GPU and oracle disagree on {int(far.sum())} ReLU gates away from the kink"
            flips.append(f"{site}: {int(dis.sum())} gate(s) at |pre| <= {p.abs()[dis].max().item():.2e}")
    if flips:
        print("ReLU gates within rounding of the kink (oracle follows the GPU):", "; ".join(flips))
    np.testing.assert_allclose(loss.cpu().numpy(), [lp.item(), la.item()], rtol=1e-4)
    names = sorted(grads)
    assert set(names) == set(tr.params), "trainable set differs from train_evp.py:379-382"
    # mathematically-zero gradients (conv biases in front of a batch-stat BN) are judged against the
    # global gradient scale rather than their own ~1e-17 magnitude
    gmax = max(g.abs().max().item() for g in grads.values())
    bad = []
    for n in names:
        a, b = tr.params[n].grad.detach().double().cpu(), grads[n]
        scale = max(b.abs().max().item(), 1e-3 * gmax)
        diff = (a - b).abs()
        err = diff.max().item()
        if err > 2e-3 * scale:
            where = np.unravel_index(int(diff.argmax()), tuple(diff.shape))
            nbad = int((diff > 2e-3 * scale).sum())
            bad.append(f"{n}: err {err:.3e} scale {scale:.3e} at {tuple(int(i) for i in where)} "
                       f"(got {a[where].item():.4e} want {b[where].item():.4e}; {nbad} of {diff.numel()} over)")
    assert not bad, "\n".join(bad)
    for prefix, (mean, var) in stats.items():
        bn = m.get_submodule(prefix)
        _close(bn.running_mean, 0.9 * sd[prefix + ".running_mean"] + 0.1 * mean, 1e-4)
        _close(bn.running_var, 0.9 * sd[prefix + ".running_var"] + 0.1 * var, 1e-4)


def test_train_step_fp32_bit_reproducible_forward(cuda):
    """With the deterministic batch statistics the f32 train forward is a pure function of parameters and inputs:
    two forward_backward calls give bitwise-identical logits, BN sums and ReLU gates (the gradients still carry
    f32-atomic reordering noise in the weight-gradient reductions, ~1e-7 relative)."""
    m, sd, tr = _build("mit_b0_evp", cuda, torch.float32)
    tr.keep_saved = True
    x, y, fl, lab, at = (t.to(cuda) for t in _train_inputs(2, 3))
    outs = []
    for _ in range(3):
        loss, logits, ant = tr.forward_backward(x, y, fl, lab, at)
        sv = tr.last_saved
        outs.append([logits.clone(), ant.clone(), sv["head"]["s1"].clone(), sv["head"]["s2"].clone(),
                     sv["head"]["Z"].clone()] + [L["y"].clone() for L in sv["flow"]] + [L["s1"].clone() for L in sv["flow"]])
    for o in outs[1:]:
        for i, (a, b) in enumerate(zip(o, outs[0])):
            assert torch.equal(a, b), f"forward tensor {i} differs between identical steps"


def test_train_step_sgd_update_and_eval_repack(cuda):
    """step() = forward_backward + SGD: parameters move exactly as torch.optim.SGD would move them
    with the same gradients, and the eval-mode forward sees the updated weights."""
    variant = "mit_b0_evp"
    B = 2
    m, sd, tr = _build(variant, cuda, torch.float32)
    x, y, fl, lab, at = _train_inputs(B, 2)
    masks = TR.make_masks(B, variant, seed=1, enabled=False)
    before = {n: p.detach().double().cpu().clone() for n, p in tr.params.items()}
    tr.step(x.to(cuda), y.to(cuda), fl.to(cuda), lab.to(cuda), at.to(cuda), masks=masks)
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().double().cpu() for n, p in tr.params.items()}
    expect, _ = TR.sgd_step(before, grads)
    for n, p in tr.params.items():
        _close(p.detach(), expect[n], 1e-6)
    # eval forward after the step uses the new weights (pack caches invalidated)
    m.eval()
    with torch.no_grad():
        out = m(x.to(cuda), y.to(cuda), fl.to(cuda), return_features=True)
    from oracle import mit_evp as M
    sd2 = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref = M.forward(x, y, sd2, variant, fl, return_features=True)
    _close(out, ref, 1e-3)


def test_train_step_bf16_b2_cosine(cuda):
    variant = "mit_b2_evp"
    B = 4
    m, sd, tr = _build(variant, cuda, torch.bfloat16)
    x, y, fl, lab, at = _train_inputs(B, 3)
    masks = TR.make_masks(B, variant, seed=7)
    lp, la, grads, _ = TR.loss_and_grads(x, y, fl, lab, at, sd, variant, masks)
    loss, _, _ = tr.forward_backward(x.to(cuda), y.to(cuda), fl.to(cuda), lab.to(cuda), at.to(cuda), masks=masks)
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss.cpu().numpy(), [lp.item(), la.item()], rtol=3e-2)
    cos = {}
    for n, g in grads.items():
        a = tr.params[n].grad.detach().double().cpu().reshape(-1)
        b = g.reshape(-1)
        if b.norm() < 1e-6 * max(v.norm().item() for v in grads.values()):
            continue                      # mathematically-zero grads (conv bias before a batch-stat BN)
        cos[n] = (a @ b / (a.norm() * b.norm() + 1e-30)).item()
    worst = sorted(cos.items(), key=lambda kv: kv[1])[:5]
    print("bf16 grad cosine, worst:", worst, "median:", float(np.median(list(cos.values()))))
    assert worst[0][1] >= 0.98, worst
    assert np.median(list(cos.values())) >= 0.995


def test_train_step_b88_benched_config_vs_oracle(cuda):
    """The benched configuration itself (train_evp.py:28 batch 88, mit_b2_evp, bf16 — bench.py
    --workload train) against the fp64 autograd oracle on the same inputs and dropout draws: f32 gradients
    of every trainable tensor within 5e-3 relative L2 (the head / BN / prompt-norm gradients reduce over
    88 x 3136 stage-1 tokens in f32: measured worst 2.9e-3, against <= 2e-3 max-abs at B = 3), bf16
    gradient cosine >= 0.98 (median >= 0.995)."""
    variant, B = "mit_b2_evp", 88
    x, y, fl, lab, at = _train_inputs(B, 4)
    masks = TR.make_masks(B, variant, seed=11)
    m32, sd, tr32 = _build(variant, cuda, torch.float32)
    lp, la, grads, _ = TR.loss_and_grads(x, y, fl, lab, at, sd, variant, masks)
    xd, yd, fd, ld, ad = (t.to(cuda) for t in (x, y, fl, lab, at))
    loss32, _, _ = tr32.forward_backward(xd, yd, fd, ld, ad, masks=masks)
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss32.cpu().numpy(), [lp.item(), la.item()], rtol=1e-4)
    gmax = max(g.abs().max().item() for g in grads.values())
    bad, worst = [], []
    for n, g in grads.items():
        a = tr32.params[n].grad.detach().double().cpu()
        scale = max(g.abs().max().item(), 1e-3 * gmax)
        rel_max = (a - g).abs().max().item() / scale
        rel_l2 = ((a - g).norm() / max(g.norm().item(), 1e-3 * gmax)).item()
        worst.append((rel_l2, rel_max, n))
        if rel_l2 > 5e-3:
            bad.append(f"{n}: rel L2 {rel_l2:.2e}, max {rel_max:.2e}")
    print("B=88 f32 worst (rel L2, rel max):", sorted(worst, reverse=True)[:6])
    assert not bad, bad
    del m32, tr32
    torch.cuda.empty_cache()
    _, _, tr16 = _build(variant, cuda, torch.bfloat16)
    loss16, _, _ = tr16.forward_backward(xd, yd, fd, ld, ad, masks=masks)
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss16.cpu().numpy(), [lp.item(), la.item()], rtol=3e-2)
    cos = []
    for n, g in grads.items():
        a, b = tr16.params[n].grad.detach().double().cpu().reshape(-1), g.reshape(-1)
        if b.norm() < 1e-6 * max(v.norm().item() for v in grads.values()):
            continue
        cos.append((a @ b / (a.norm() * b.norm() + 1e-30)).item())
    print(f"B=88 bf16 grad cosine: min {min(cos):.5f} median {float(np.median(cos)):.5f}")
    assert min(cos) >= 0.98 and np.median(cos) >= 0.995


def test_train_loss_decreases(cuda):
    """Several SGD steps on one fixed batch (device masks, stochastic depth on) reduce the loss."""
    variant = "mit_b0_evp"
    B = 8
    m, sd, tr = _build(variant, cuda, torch.bfloat16)
    tr.hp["lr"] = 2e-3
    x, y, fl, lab, at = (t.to(cuda) for t in _train_inputs(B, 4))
    losses = []
    for _ in range(6):
        loss, _, _ = tr.step(x, y, fl, lab, at)
        losses.append(loss.sum().item())
    assert all(np.isfinite(losses))
    assert losses[-1] < losses[0], losses


def test_train_graph_replay_matches_eager(cuda):
    """capture() + replays reproduce the eager iterations (same masks via the device step counter,
    same SGD trajectory and BatchNorm buffers), to within the run-to-run spread of two eager runs
    (f32 atomics make the bf16 step non-bit-reproducible)."""
    variant = "mit_b0_evp"
    B = 4
    x, y, fl, lab, at = (t.to(cuda) for t in _train_inputs(B, 6))
    runs = []
    for mode in ("eager", "eager", "graph"):
        m, _, t = _build(variant, cuda, torch.bfloat16)
        p0 = {n: p.detach().clone() for n, p in t.params.items()}
        if mode == "eager":
            for _ in range(3):
                t.step(x, y, fl, lab, at)
        else:
            t.step(x, y, fl, lab, at)
            t.capture(x, y, fl, lab, at)
            for _ in range(2):
                t.step(x, y, fl, lab, at)
        torch.cuda.synchronize()
        assert t.steps == 3
        assert int(m.head.linear_fuse.bn.num_batches_tracked) == 3
        runs.append(({n: (p - p0[n]).double() for n, p in t.params.items()}, m.head.linear_fuse.bn.running_mean.clone()))
    (ua, ra), (ub, rb), (ug, rg) = runs
    # relative L2 distance of the whole update vector: graph vs eager must sit within the eager-vs-eager
    # spread (per-tensor max-abs ratios are dominated by mathematically-zero gradients, e.g. conv
    # biases in front of a batch-statistics BatchNorm)
    na = sum(ua[n].pow(2).sum() for n in ua).sqrt().item()
    ee = sum((ua[n] - ub[n]).pow(2).sum() for n in ua).sqrt().item() / na
    # the graph run against the NEARER eager run: the bf16 step is not bit-reproducible (f32 atomics in the
    # weight gradients), and at B = 4 one ReLU gate at its kink can land on either side, which moves the whole
    # 3-step update by ~1.5e-2 relative — observed both as eager-vs-eager 1.55e-2 / graph-vs-eager 2.6e-3 (a
    # round-4 run) and as 2.9e-3 / 1.5e-2 (round 6, first box).  A capture bug (stale masks, parameters or BN
    # buffers in the replay) moves it by O(0.1-1), so the bound keeps a 0.03 floor above that bimodal spread.
    eg = min(sum((u[n] - ug[n]).pow(2).sum() for n in u).sqrt().item() for u in (ua, ub)) / na
    print(f"relative update distance: graph-vs-nearest-eager {eg:.3e}, eager-vs-eager {ee:.3e}")
    assert eg <= max(3 * ee + 1e-3, 0.03), (eg, ee)
    _close(rg, ra, 1e-2)


def _ddp_rank(rank, world, port, out, grad_comm="f32"):
    import os
    import sys
    import torch.distributed as dist
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "deep-learning-for-surgical-video-analysis_amd"), repo]
    from models import mix_transformer_evp as mte
    from svk.train import EVPTrainStep
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = mte.mit_b0_evp()
    m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0))
    m = m.to(dev)
    if rank == 1:                      # diverge rank 1's BN buffers: the step must re-sync them from rank 0
        m.head.linear_fuse.bn.running_mean.add_(1.0)
    tr = EVPTrainStep(m, dtype=torch.float32, drop=False, process_group=dist.group.WORLD, world_size=world,
                      grad_comm=grad_comm)
    x, y, fl, lab, at = (t.to(dev) for t in _train_inputs(2, 20 + rank))
    rm_before = m.head.linear_fuse.bn.running_mean.clone()
    tr.forward_backward(x, y, fl, lab, at)
    local = tr.grad.clone()
    tr.allreduce_grads()
    avg = tr.grad.clone()
    tr.optimizer_step()
    torch.cuda.synchronize()
    out[rank] = (local.cpu(), avg.cpu(), tr.flat.detach().cpu(), rm_before.cpu())
    dist.destroy_process_group()


@pytest.mark.parametrize("grad_comm", ["f32", "bf16"])
def test_train_ddp_two_ranks_gloo(cuda, grad_comm):
    """DDP semantics of the train step with 2 ranks (gloo over the one GPU of the test box; the
    bench's multi-GPU runs use RCCL): averaged gradients, identical parameters after the step.  bf16: the
    compressed all-reduce — averages within bf16 rounding, still identical on both ranks."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = mp.Manager().dict()
    mp.spawn(_ddp_rank, args=(2, port, out, grad_comm), nprocs=2, join=True)
    (l0, a0, p0, _), (l1, a1, p1, _) = out[0], out[1]
    if grad_comm == "f32":
        torch.testing.assert_close(a0, (l0 + l1) / 2, rtol=1e-5, atol=1e-7)
    else:
        ref = (l0 + l1) / 2
        rel = ((a0 - ref).norm() / ref.norm()).item()
        print(f"bf16 all-reduce: relative L2 of the averaged gradient {rel:.3e}")
        assert 0 < rel <= 4e-3
    torch.testing.assert_close(a1, a0)
    torch.testing.assert_close(p1, p0)
    assert not torch.equal(l0, l1)                 # the ranks really saw different frames


def _ddp_capture_rank(rank, world, port, out):
    """Eager bucketed DDP iteration, then capture() + graph replay with the process group: no
    collective is captured (BN broadcast and the two bucket all-reduces run eagerly between the three
    graphs), so the replayed step must keep the ranks' parameters, gradients and BN buffers in sync."""
    import os
    import sys
    import torch.distributed as dist
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "deep-learning-for-surgical-video-analysis_amd"), repo]
    from models import mix_transformer_evp as mte
    from svk.train import EVPTrainStep
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    m = mte.mit_b0_evp()
    m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0))
    m = m.to(dev)
    if rank == 1:
        m.flow_encoder.bn2.running_var.mul_(3.0)
    tr = EVPTrainStep(m, dtype=torch.bfloat16, drop=True, seed=rank, process_group=dist.group.WORLD, world_size=world)
    assert 0 < tr.head_end < tr.n_trainable
    x, y, fl, lab, at = (t.to(dev) for t in _train_inputs(2, 40 + rank))
    tr.step(x, y, fl, lab, at)                     # eager: train_iteration (head bucket overlapped)
    tr.capture(x, y, fl, lab, at)
    assert tr.graph_rest is not None and tr.graph_opt is not None
    flat1 = tr.flat.detach().clone()
    loss, _, _ = tr.step(x, y, fl, lab, at)        # replay
    loss, _, _ = tr.step(x, y, fl, lab, at)        # replay again
    torch.cuda.synchronize()
    v_own = m.flow_encoder.bn2.running_var.clone()  # this rank's own batch statistics went in last
    tr.sync_buffers()                              # what the next step starts with: rank 0's buffers
    torch.cuda.synchronize()
    out[rank] = (flat1.cpu(), tr.flat.detach().cpu(), tr.grad.cpu(), m.flow_encoder.bn2.running_var.cpu(),
                 loss.cpu(), tr.steps, v_own.cpu())
    dist.destroy_process_group()


def test_train_ddp_two_ranks_capture_replay(cuda):
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = mp.Manager().dict()
    mp.spawn(_ddp_capture_rank, args=(2, port, out), nprocs=2, join=True)
    (f0, p0, g0, v0, l0, n0, o0), (f1, p1, g1, v1, l1, n1, o1) = out[0], out[1]
    assert n0 == n1 == 3
    torch.testing.assert_close(f1, f0)
    torch.testing.assert_close(p1, p0)             # identical parameters after two replayed steps
    torch.testing.assert_close(g1, g0)             # averaged gradients
    assert not torch.equal(p0, f0)                 # the replays really stepped
    assert not torch.equal(o0, o1)                 # each rank's BN update used its own frames ...
    torch.testing.assert_close(v1, v0)             # ... and the per-step broadcast re-syncs them from rank 0
    torch.testing.assert_close(v0, o0)
    assert torch.isfinite(l0).all() and not torch.equal(l0, l1)


def _bns(m):
    return [m.head.linear_fuse.bn] + [getattr(m.flow_encoder, f"bn{i}") for i in range(1, 5)]


def _sync_train_state(dst, src):
    """dst := src (parameters, momentum, BN buffers, mask counter, step count), in place: captured graphs stay
    valid; the compute packs are re-derived."""
    with torch.no_grad():
        dst.flat.copy_(src.flat)
        dst.mom.copy_(src.mom)
        dst.counter.copy_(src.counter)
        for bd, bs in zip(_bns(dst.model), _bns(src.model)):
            for nm in ("running_mean", "running_var", "num_batches_tracked"):
                getattr(bd, nm).copy_(getattr(bs, nm))
    dst.steps = src.steps
    dst._refresh_packs()


def _rccl_rank(rank, world, port, out, grad_comm="f32"):
    """World-size-1 DDP over RCCL (the "nccl" backend on ROCm): the bucketed async all-reduce and the
    coalesced BN broadcast run as real RCCL collectives on the box's GPU, eagerly and around the three
    captured graphs; the same steps without a process group are the reference.  Both trainers start every step
    from the same state (the RCCL trainer's, copied into the reference), so each step's update is compared on
    its own: two independent trajectories drift apart by the f32-atomic noise of the weight-gradient reductions,
    and a drifted pre-ReLU value at the kink would flip a gate — a property of ReLU, not of the collectives."""
    import os
    import sys
    import torch.distributed as dist
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "deep-learning-for-surgical-video-analysis_amd"), repo]
    from models import mix_transformer_evp as mte
    from svk.train import EVPTrainStep
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    calls = {"all_reduce": 0, "broadcast": 0}
    real_ar, real_bc = dist.all_reduce, dist.broadcast

    def ar(*a, **k):
        calls["all_reduce"] += 1
        return real_ar(*a, **k)

    def bc(*a, **k):
        calls["broadcast"] += 1
        return real_bc(*a, **k)

    dist.all_reduce, dist.broadcast = ar, bc
    trs = {}
    for mode in ("rccl", "single"):
        m = mte.mit_b0_evp()
        m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0))
        m = m.to(dev)
        grp = dist.group.WORLD if mode == "rccl" else None
        trs[mode] = EVPTrainStep(m, dtype=torch.float32, drop=False, process_group=grp, world_size=world,
                                 grad_comm=grad_comm)
    x, y, fl, lab, at = (t.to(dev) for t in _train_inputs(2, 60))
    rels, rms = [], []
    for k in range(3):                                 # eager train_iteration, then two graph replays
        if k == 1:
            for mode in ("rccl", "single"):
                trs[mode].capture(x, y, fl, lab, at)
            assert trs["rccl"].graph_rest is not None and trs["rccl"].graph_opt is not None
        _sync_train_state(trs["single"], trs["rccl"])
        f0 = trs["rccl"].flat.detach().clone()
        for mode in ("rccl", "single"):
            trs[mode].step(x, y, fl, lab, at)
        torch.cuda.synchronize()
        ur = (trs["rccl"].flat.detach() - f0).double()
        us = (trs["single"].flat.detach() - f0).double()
        rels.append(((ur - us).norm() / us.norm()).item() if us.norm() > 0 else float("inf"))
        rms.append((trs["rccl"].model.head.linear_fuse.bn.running_mean.cpu(),
                    trs["single"].model.head.linear_fuse.bn.running_mean.cpu()))
    out["backend"] = dist.get_backend()
    out["calls"] = dict(calls)
    out["res"] = dict(rels=rels, rms=rms, steps=(trs["rccl"].steps, trs["single"].steps))
    dist.destroy_process_group()


@pytest.mark.parametrize("grad_comm", ["f32", "bf16"])
def test_train_ddp_rccl_world1_capture_replay(cuda, grad_comm):
    """init_process_group("nccl") at world size 1 on the one GPU, then
    train_iteration, capture() and two replays through the bucketed async RCCL all-reduce and the BN
    broadcast; the parameters must follow the no-process-group step."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = mp.Manager().dict()
    mp.spawn(_rccl_rank, args=(1, port, out, grad_comm), nprocs=1, join=True)
    assert out["backend"] == "nccl"
    # 3 steps x (2 gradient buckets + 1 coalesced BN broadcast)
    assert out["calls"]["all_reduce"] == 6 and out["calls"]["broadcast"] == 3, out["calls"]
    res = out["res"]
    assert res["steps"] == (3, 3)
    print(f"RCCL world-1 ({grad_comm} gradient exchange) vs single-process update per step: relative L2 "
          + ", ".join(f"{r:.3e}" for r in res["rels"]))
    assert max(res["rels"]) <= (1e-5 if grad_comm == "f32" else 1e-2), res["rels"]
    for rr, rs in res["rms"]:
        torch.testing.assert_close(rr, rs, rtol=1e-5, atol=1e-6)


# ---- the drop-in train mode: MixVisionTransformerEVP.forward as one autograd node ------------------

def _ref_frozen_model(variant, cuda, seed=0):
    """The model as train_evp.py prepares it: state loaded, backbone frozen by the script's own rule
    (train_evp.py:379-382), moved to the GPU."""
    from models import mix_transformer_evp as mte
    m = getattr(mte, variant)()
    m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, seed))
    for name, param in m.named_parameters():
        if "head" not in name and "prompt" not in name and "flow_encoder" not in name and \
                "cross_attn_s3" not in name and "cross_attn_s4" not in name:
            param.requires_grad = False
    return m.to(cuda)


def _ref_sgd(model, lr=5e-4):
    """train_evp.py:405-419 (multi_optim 1, optimizer_choice 0: the script's defaults)."""
    return torch.optim.SGD([
        {'params': model.prompt_generator.parameters(), 'lr': lr},
        {'params': model.head.parameters(), 'lr': lr},
        {'params': model.flow_encoder.parameters(), 'lr': lr},
        {'params': model.cross_attn_s3.parameters(), 'lr': lr},
        {'params': model.cross_attn_s4.parameters(), 'lr': lr},
    ], lr=lr / 10, momentum=0.9, dampening=0, weight_decay=1e-5, nesterov=False)


def test_train_mode_autograd_grads_equal_native_step_fp32(cuda):
    """model.train(); forward; CE(sum) + SmoothL1(sum); loss.backward() — the parameters' .grad from the
    autograd node equal EVPTrainStep's flat gradient on the same inputs and dropout draws (fp32: the same
    kernels, only the f32 atomic summation order may differ)."""
    from svk.train import EVPTrainStep
    B = 3
    x, y, fl, lab, at = (t.to(cuda) for t in _train_inputs(B, 70))
    m = _ref_frozen_model("mit_b0_evp", cuda)
    m.train()
    yp, ya = m(x, y, fl)
    assert yp.shape == (B, 7) and ya.shape == (B, 7) and yp.requires_grad
    loss = torch.nn.CrossEntropyLoss(reduction="sum")(yp, lab) + torch.nn.SmoothL1Loss(reduction="sum")(ya, at)
    loss.backward()
    torch.cuda.synchronize()
    m2 = _ref_frozen_model("mit_b0_evp", cuda)
    tr = EVPTrainStep(m2, dtype=torch.float32, seed=m.__dict__["_svk_evp_autograd"].seed)
    l2, _, _ = tr.forward_backward(x, y, fl, lab, at)
    torch.cuda.synchronize()
    assert abs(loss.item() - float(l2.sum())) <= 1e-5 * max(1.0, abs(loss.item()))
    n = 0
    # mathematically-zero gradients (a bias in front of a batch-statistics BatchNorm) carry only f32
    # rounding: relative error against 1e-3 of the largest gradient norm at least
    floor = 1e-3 * max(tr.G(name).norm().item() for name in tr.params)
    for name, p in m.named_parameters():
        if not p.requires_grad:
            assert p.grad is None, name
            continue
        g_ref = tr.G(name)
        d = (p.grad - g_ref).norm().item() / max(g_ref.norm().item(), floor)
        assert d <= 1e-4, (name, d)
        n += 1
    assert n == len(tr.params)
    # running statistics updated by the forward, as nn.BatchNorm2d does
    assert int(m.head.linear_fuse.bn.num_batches_tracked) == 1
    torch.testing.assert_close(m.head.linear_fuse.bn.running_mean, m2.head.linear_fuse.bn.running_mean,
                               rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("variant", ["mit_b2_evp", "mit_b3_evp"])
def test_train_evp_loop_verbatim_fp16_b8(cuda, variant):
    """the train_evp.py:473-515 inner loop verbatim for two steps at B = 8 —
    model.train(), autocast(float16) forward, CE(sum) + SmoothL1(sum), scaler.scale(loss).backward(),
    scaler.step(optimizer) with torch's SGD over the script's parameter groups, scaler.update() — against
    the native EVPTrainStep applying the same non-skipped steps with the same dropout draws: the loop's
    parameter updates are as close to the f32 native step as the native f16 step is (relative L2 of the
    update vector within 1.5x + 1e-2 of it; measured values printed), and within 5e-2 of the native f16
    step (the autograd side back-propagates the GradScaler-scaled loss in f16)."""
    from svk.train import EVPTrainStep
    B = 8           # mit_b3_evp: the model train_evp.py:362 itself builds
    x, y, fl, lab, at = (t.to(cuda) for t in _train_inputs(B, 71))
    model = _ref_frozen_model(variant, cuda)
    p0 = {n: p.detach().clone() for n, p in model.named_parameters() if p.requires_grad}
    criterion_phase = torch.nn.CrossEntropyLoss(reduction='sum')
    criterion_reg = torch.nn.SmoothL1Loss(reduction='sum')
    optimizer = _ref_sgd(model)
    scaler = torch.amp.GradScaler("cuda")
    model.train()
    applied = []
    for i in range(2):
        optimizer.zero_grad()
        inputs, segmaps, flow = x.view(-1, 1, 3, 224, 224), y.view(-1, 1, 3, 224, 224), fl.view(-1, 1, 2, 224, 224)
        with torch.autocast(device_type='cuda', dtype=torch.float16):
            outputs_phase, outputs_phase_ant = model.forward(inputs, segmaps, flow)
            loss_phase = criterion_phase(outputs_phase, lab)
            loss_phase_ant = criterion_reg(outputs_phase_ant, at)
            loss = loss_phase + loss_phase_ant
        s0 = scaler.get_scale()
        scaler.scale(loss).backward()
        scaler.step(optimizer)
        scaler.update()
        assert torch.isfinite(loss)
        if scaler.get_scale() >= s0:            # a skipped step (inf/NaN in the f16 gradients) lowers the scale
            applied.append(i)
    print(f"train_evp loop: applied steps {applied}, final scale {scaler.get_scale()}")
    assert applied, "both steps skipped"
    seed = model.__dict__["_svk_evp_autograd"].seed   # the autograd node's mask stream (torch's seed)

    def native(dtype):
        m2 = _ref_frozen_model(variant, cuda)
        tr = EVPTrainStep(m2, dtype=dtype, seed=seed)
        for i in applied:
            tr.counter.fill_(i)                 # the draws of forward i
            tr.step(x, y, fl, lab, at)
        torch.cuda.synchronize()
        return {n: tr.params[n].detach() - p0[n] for n in p0}

    def dist(a, b):
        num = sum((a[n].double() - b[n].double()).pow(2).sum().item() for n in p0)
        return (num / sum(b[n].double().pow(2).sum().item() for n in p0)) ** 0.5

    u_auto = {n: p.detach() - p0[n] for n, p in model.named_parameters() if n in p0}
    u32, u16 = native(torch.float32), native(torch.float16)
    e_auto, e_nat, e_pair = dist(u_auto, u32), dist(u16, u32), dist(u_auto, u16)
    print(f"train_evp loop (fp16 autocast + GradScaler) vs native f32 step: update relative L2 {e_auto:.3e}; "
          f"native f16 step vs f32 {e_nat:.3e}; loop vs native f16 {e_pair:.3e}")
    # the drop-in loop is as accurate as the native step at the same precision
    assert e_auto <= 1.5 * e_nat + 1e-2 and e_pair <= 5e-2
