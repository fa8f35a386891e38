"""Per-kernel parity of the svk HIP kernels against plain torch CPU references (fp64 math on the
same, dtype-rounded inputs).  Tolerances: f32 path (exact f32 MFMA products, f32 accumulation)
rtol/atol 2e-5 relative to the output scale; bf16 path 1.2e-2 (inputs identical, outputs rounded to
bf16 — 8 significant bits); f16 path 2.5e-3 (outputs rounded to f16 — 11 significant bits)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DTS = [torch.float32, torch.bfloat16, torch.float16]
H16 = [torch.bfloat16, torch.float16]


def _tol(dt):
    return {torch.float32: (2e-5, 2e-5), torch.float16: (2.5e-3, 2.5e-3)}.get(dt, (1.2e-2, 1.2e-2))


def _close(got, ref, dt, scale=None):
    rtol, atol = _tol(dt)
    ref = ref.double()
    s = float(ref.abs().max()) if scale is None else scale
    torch.testing.assert_close(got.double().cpu(), ref, rtol=rtol, atol=atol * max(1.0, s))


def _rand(*shape, dt, dev, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dt).to(dev)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("M,N,K", [(1, 7, 2048), (100, 64, 64), (777, 200, 320), (4096, 256, 64), (300, 14, 14),
                                   (513, 2048, 1024), (49, 33, 147)])
@pytest.mark.parametrize("act", [None, "gelu", "relu", "tanh"])
def test_gemm(cuda, dt, M, N, K, act):
    from svk import ops
    a = _rand(M, K, dt=dt, dev=cuda, seed=1)
    w = _rand(N, K, dt=dt, dev=cuda, scale=K ** -0.5, seed=2)
    b = _rand(N, dt=torch.float32, dev=cuda, seed=3)
    r = _rand(M, N, dt=dt, dev=cuda, seed=4)
    got = ops.gemm(a, w, b, act=act, residual=r)
    torch.cuda.synchronize()
    ref = a.cpu().double() @ w.cpu().double().t() + b.cpu().double()
    ref = {None: lambda t: t, "gelu": lambda t: F.gelu(t), "relu": torch.relu, "tanh": torch.tanh}[act](ref)
    ref = ref + r.cpu().double()
    _close(got, ref, dt)


@pytest.mark.parametrize("M,N,K,act,res", [(70000, 512, 128, None, True), (30000, 320, 1280, None, True),
                                           (3000, 136, 80, "gelu", False), (5000, 96, 200, "relu", True),
                                           (40000, 64, 256, None, True), (20001, 16, 16, None, False),
                                           (12544, 2048, 512, "tanh", False)])
@pytest.mark.parametrize("dt", H16)
def test_gemm_persistent_16bit(cuda, M, N, K, act, res, dt):
    """16-bit plain-epilogue GEMMs run on the persistent LDS-DMA kernel (more tiles than resident
    workgroups, K tails, M tails); checked against fp64 and against the tiled kernel (SVK_NO_PK)."""
    import os
    from svk import ops
    a = _rand(M, K, dt=dt, dev=cuda, seed=11)
    w = _rand(N, K, dt=dt, dev=cuda, scale=K ** -0.5, seed=12)
    b = _rand(N, dt=torch.float32, dev=cuda, seed=13)
    r = _rand(M, N, dt=dt, dev=cuda, seed=14) if res else None
    got = ops.gemm(a, w, b, act=act, residual=r)
    os.environ["SVK_NO_PK"] = "1"
    try:
        tiled = ops.gemm(a, w, b, act=act, residual=r)
    finally:
        del os.environ["SVK_NO_PK"]
    torch.cuda.synchronize()
    ref = a.double() @ w.double().t() + b.double()
    ref = {None: lambda t: t, "gelu": lambda t: F.gelu(t), "relu": torch.relu, "tanh": torch.tanh}[act](ref)
    if res:
        ref = ref + r.double()
    _close(got, ref.cpu(), dt)
    _close(got, tiled.double().cpu(), dt)


@pytest.mark.parametrize("M,N,K,uact", [(60000, 256, 64, "gelu"), (20000, 320, 1280, "relu"), (7000, 72, 136, "gelu")])
def test_gemm_persistent_ext_bf16(cuda, M, N, K, uact):
    """Training epilogue on the persistent kernel: row scale (stochastic depth) x activation backward
    from a saved pre-activation + residual; against fp64 and the tiled kernel (SVK_NO_PK)."""
    import os
    from svk import ops
    dt = torch.bfloat16
    a = _rand(M, K, dt=dt, dev=cuda, seed=21)
    w = _rand(N, K, dt=dt, dev=cuda, scale=K ** -0.5, seed=22)
    u = _rand(M, N, dt=dt, dev=cuda, seed=23)
    r = _rand(M, N, dt=dt, dev=cuda, seed=24)
    rows_per = 1000
    s = torch.rand((M + rows_per - 1) // rows_per, generator=torch.Generator().manual_seed(25)).to(cuda)
    kw = dict(residual=r, row_scale=s, rows_per=rows_per, dact=uact, dact_src=u)
    got = ops.gemm(a, w, **kw)
    os.environ["SVK_NO_PK"] = "1"
    try:
        tiled = ops.gemm(a, w, **kw)
    finally:
        del os.environ["SVK_NO_PK"]
    torch.cuda.synchronize()
    ur = u.double().requires_grad_(True)
    g = (a.double() @ w.double().t()) * s.double().repeat_interleave(rows_per)[:M, None]
    (F.gelu(ur) if uact == "gelu" else torch.relu(ur)).backward(g)
    ref = ur.grad + r.double()
    _close(got, ref.cpu(), dt)
    _close(got, tiled.double().cpu(), dt)


@pytest.mark.parametrize("cfg", [0, 10, 20, 30])
@pytest.mark.parametrize("dt", H16)
def test_persistent_tile_configs(cuda, cfg, dt):
    """Every persistent-GEMM tile configuration (forced through svk_tune) on dense and implicit-GEMM
    shapes with M / N / K tails, staged and register epilogues."""
    from svk import ops
    try:
        ops.tune("pk_cfg", cfg)
        for M, N, K, res in ((5000, 320, 1280, True), (777, 136, 200, False), (12544, 512, 512, True)):
            a = _rand(M, K, dt=dt, dev=cuda, seed=51)
            w = _rand(N, K, dt=dt, dev=cuda, scale=K ** -0.5, seed=52)
            b = _rand(N, dt=torch.float32, dev=cuda, seed=53)
            r = _rand(M, N, dt=dt, dev=cuda, seed=54) if res else None
            got = ops.gemm(a, w, b, act="gelu", residual=r)
            ref = F.gelu(a.double() @ w.double().t() + b.double())
            if res:
                ref = ref + r.double()
            _close(got, ref.cpu(), dt)
        x = _rand(6, 28, 28, 128, dt=dt, dev=cuda, seed=55)
        wc = _rand(320, 3 * 3 * 128, dt=dt, dev=cuda, scale=(9 * 128) ** -0.5, seed=56)
        bc = _rand(320, dt=torch.float32, dev=cuda, seed=57)
        got = ops.conv2d_nhwc(x, wc, 3, 2, 1, bias=bc, act="relu")
        wr = wc.double().cpu().view(320, 3, 3, 128).permute(0, 3, 1, 2)
        ref = F.conv2d(x.cpu().double().permute(0, 3, 1, 2), wr, bc.cpu().double(), stride=2, padding=1)
        _close(got, torch.relu(ref).permute(0, 2, 3, 1), dt)
    finally:
        ops.tune("pk_cfg", -1)


@pytest.mark.parametrize("cfg", [70, 71])
@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("act", [None, "gelu", "relu"])
def test_gemm_pingpong_configs(cuda, cfg, dt, act):
    """The 256-row ping-pong GEMM (gemm_pp, BN = 256 / 320, forced through svk_tune) against fp64: M / N / K
    tails, residual on / off, more tiles than resident workgroups (the persistent walk crossing tiles), one
    K-tile per tile, and the MiT-b2 shapes it is meant for."""
    from svk import ops
    try:
        ops.tune("pk_cfg", cfg)
        for M, N, K, res in ((5000, 320, 1280, True), (777, 136, 200, False), (12544, 512, 512, True),
                             (12544, 2048, 1024, False), (3000, 640, 72, True), (300, 1280, 64, False),
                             (50176, 320, 320, True)):
            a = _rand(M, K, dt=dt, dev=cuda, seed=61)
            w = _rand(N, K, dt=dt, dev=cuda, scale=K ** -0.5, seed=62)
            b = _rand(N, dt=torch.float32, dev=cuda, seed=63)
            r = _rand(M, N, dt=dt, dev=cuda, seed=64) if res else None
            got = ops.gemm(a, w, b, act=act, residual=r)
            ref = a.double() @ w.double().t() + b.double()
            ref = {None: lambda t: t, "gelu": lambda t: F.gelu(t), "relu": torch.relu}[act](ref)
            if res:
                ref = ref + r.double()
            assert ops._last_kernel().startswith("gemm_pp"), ops._last_kernel()
            _close(got, ref.cpu(), dt)
    finally:
        ops.tune("pk_cfg", -1)


@pytest.mark.parametrize("cfg", [90, 91, 92, 93])
@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("act", [None, "gelu", "relu"])
def test_gemm_wide_tile_configs(cuda, cfg, dt, act):
    """The wide-tile GEMM (gemm_wt: one 256-thread workgroup per CU, 256 x 256 / 256 x 160 / 256 x 128 tiles, forced
    through svk_tune) against fp64: M / N / K tails, residual on / off, more tiles than workgroups (the persistent
    walk crossing tiles), one K-tile per tile, and the MiT-b2 shapes it is meant for."""
    from svk import ops
    try:
        ops.tune("pk_cfg", cfg)
        for M, N, K, res in ((5000, 320, 1280, True), (777, 136, 192, False), (12544, 512, 512, True),
                             (12544, 2048, 1024, False), (3000, 640, 64, True), (300, 1280, 64, False),
                             (50176, 320, 320, True), (70000, 256, 128, False), (1000, 2052, 128, True)):
            a = _rand(M, K, dt=dt, dev=cuda, seed=61)
            w = _rand(N, K, dt=dt, dev=cuda, scale=K ** -0.5, seed=62)
            b = _rand(N, dt=torch.float32, dev=cuda, seed=63)
            r = _rand(M, N, dt=dt, dev=cuda, seed=64) if res else None
            got = ops.gemm(a, w, b, act=act, residual=r)
            ref = a.double() @ w.double().t() + b.double()
            ref = {None: lambda t: t, "gelu": lambda t: F.gelu(t), "relu": torch.relu}[act](ref)
            if res:
                ref = ref + r.double()
            assert ops._last_kernel().startswith("gemm_wt"), ops._last_kernel()
            _close(got, ref.cpu(), dt)
    finally:
        ops.tune("pk_cfg", -1)


@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("B,HB,CS,ln", [(3, 57, 48, True), (2, 57, 32, True), (1, 20, 48, False), (5, 57, 48, True)])
@pytest.mark.parametrize("C", [64, 16])
def test_conv2d_s2d_ln(cuda, dt, B, HB, CS, ln, C):
    """The stage-1 patch embedding over s2d blocks + LayerNorm in one kernel (svk_conv2d_s2d_ln) against the
    unfused svk path (conv2d_nhwc, then layernorm: same conv rounding, LN statistics summed in another order)
    and fp64; C = 16 is the handcrafted prompt generator's first stem (64 / scale_factor 4 channels)."""
    from svk import ops
    xs = _rand(B, HB, HB, CS, dt=dt, dev=cuda, seed=81)
    w = _rand(C, 4 * CS, dt=dt, dev=cuda, scale=(4 * CS) ** -0.5, seed=82)
    b = _rand(C, dt=torch.float32, dev=cuda, seed=83)
    g = (1 + 0.1 * _rand(C, dt=torch.float32, dev=cuda, seed=84)) if ln else None
    bt = 0.1 * _rand(C, dt=torch.float32, dev=cuda, seed=85) if ln else None
    got = ops.conv2d_s2d_ln(xs, w, b, g, bt, 1e-6)
    assert ops._last_kernel().startswith("stem_s2d_ln"), ops._last_kernel()
    y = ops.conv2d_nhwc(xs, w, 2, 1, 0, bias=b)
    ref16 = ops.layernorm(y.view(-1, C), g, bt, 1e-6).view_as(y) if ln else y
    ulp = 2 ** -8 if dt == torch.bfloat16 else 2 ** -11
    d = (got.float() - ref16.float()).abs().max().item()
    assert d <= 4 * ulp * max(1.0, float(ref16.float().abs().max())), d
    xd = xs.double().cpu().permute(0, 3, 1, 2)
    wd = w.double().cpu().view(C, 2, 2, CS).permute(0, 3, 1, 2)
    yd = F.conv2d(xd, wd, b.double().cpu()).permute(0, 2, 3, 1)
    if ln:
        yd = F.layer_norm(yd, (C,), g.double().cpu(), bt.double().cpu(), 1e-6)
    _close(got, yd, dt)


@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("B,res", [(3, True), (1, False), (5, True)])
@pytest.mark.parametrize("W,K,N,mx", [(14, 1280, 320, True), (14, 1280, 320, False), (7, 2048, 512, True),
                                      (7, 2048, 512, False), (14, 640, 320, True), (7, 1024, 512, True),
                                      (28, 512, 128, True)])
def test_mixffn_dw_fc2(cuda, dt, B, res, W, K, N, mx, monkeypatch):
    """dwconv3x3 + GELU fused into fc2 (svk_mixffn_dw_fc2; the stage-3 / stage-4 shapes 14 x 14, 1280 -> 320 and
    7 x 7, 2048 -> 512; mx: the form with the depthwise conv on MFMA from packed operands,
    svk_mixffn_dw_fc2_packed, also at shorter K) against the unfused svk path (dwconv3x3 + gemm: same
    roundings but for the mx form's 16-bit taps, expected within a few 16-bit ulps) and fp64.  Token counts
    that are not a multiple of the 64 / 32-token tile (masked rows)."""
    from svk import ops
    monkeypatch.setattr(ops, "DWFC2_MX", mx)
    h = _rand(B, W, W, K, dt=dt, dev=cuda, seed=71)
    taps = _rand(9, K, dt=torch.float32, dev=cuda, scale=0.3, seed=72)
    db = _rand(K, dt=torch.float32, dev=cuda, scale=0.1, seed=73)
    w2 = _rand(N, K, dt=dt, dev=cuda, scale=K ** -0.5, seed=74)
    b2 = _rand(N, dt=torch.float32, dev=cuda, seed=75)
    r = _rand(B, W * W, N, dt=dt, dev=cuda, seed=76) if res else None
    got = ops.mixffn_dw_fc2(h, taps, db, w2, b2, residual=r)
    assert ops._last_kernel().startswith("dw_fc2_mx" if mx else "dw_fc2<"), ops._last_kernel()
    if mx:   # the pre-packed call gives the same bits
        pk = ops.mixffn_dw_fc2_pack(taps, db, w2, W)
        assert torch.equal(ops.mixffn_dw_fc2(h, taps, db, w2, b2, residual=r, packed=pk), got)
    g = ops.dwconv3x3(h, taps, db, act="gelu")
    ref16 = ops.gemm(g.view(B, W * W, K), w2, b2, residual=r)
    d = (got.float() - ref16.float()).abs().max().item()
    assert d <= 4 * float(ref16.float().abs().max()) * (2 ** -8 if dt == torch.bfloat16 else 2 ** -11), d
    hd = h.double().cpu().permute(0, 3, 1, 2)
    cv = F.conv2d(hd, taps.double().cpu().t().reshape(K, 1, 3, 3), db.double().cpu(), padding=1, groups=K)
    gd = F.gelu(cv).permute(0, 2, 3, 1).reshape(B, W * W, K)
    ref = gd @ w2.double().cpu().t() + b2.double().cpu()
    if res:
        ref = ref + r.double().cpu()
    _close(got, ref, dt)


@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("B,W,K,N", [(88, 14, 1280, 320), (5, 7, 2048, 512), (3, 14, 640, 320)])
def test_mixffn_dw_fc2_identity(cuda, dt, B, W, K, N):
    """The identity-activation form (svk_mixffn_dw_fc2_packed_act, act none) as the train step uses it: the
    data gradient through a frozen DWConv + fc1, dX = dwconv3x3(dU, flipped taps) · W1, against the unfused
    svk path (dwconv3x3 + gemm: the same roundings, within a few 16-bit ulps) and fp64 (the transposed
    depthwise conv of the fp64 graph)."""
    from svk import ops
    du = _rand(B, W, W, K, dt=dt, dev=cuda, seed=91)
    taps = _rand(9, K, dt=torch.float32, dev=cuda, scale=0.3, seed=92)
    flip = taps.flip(0).contiguous()
    zero, zc = torch.zeros(K, device=cuda), torch.zeros(N, device=cuda)
    w1 = _rand(K, N, dt=dt, dev=cuda, scale=N ** -0.5, seed=93)          # fc1.weight [hid, C]
    w1t = w1.t().contiguous()
    pk = ops.mixffn_dw_fc2_pack(flip, zero, w1t, W)
    got = ops.mixffn_dw_fc2(du, flip, zero, w1t, zc, packed=pk, act="none")
    assert ops._last_kernel().startswith("dw_fc2_mx") and "identity" in ops._last_kernel(), ops._last_kernel()
    dh = ops.dwconv3x3(du, flip, zero)
    ref16 = ops.gemm(dh.view(B, W * W, K), w1t)
    d = (got.float() - ref16.float()).abs().max().item()
    assert d <= 4 * float(ref16.float().abs().max()) * (2 ** -8 if dt == torch.bfloat16 else 2 ** -11), d
    # fp64: the adjoint of the forward depthwise conv (taps as the forward packs them) applied to dU
    kf = taps.to(dt).double().cpu().t().reshape(K, 1, 3, 3)
    dhd = F.conv_transpose2d(du.double().cpu().permute(0, 3, 1, 2), kf, padding=1, groups=K)
    ref = dhd.permute(0, 2, 3, 1).reshape(B, W * W, K) @ w1.double().cpu()
    _close(got, ref, dt)


@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("B,W,K,N", [(88, 14, 1280, 320), (5, 7, 2048, 512), (3, 14, 640, 320)])
def test_mixffn_dw_fc2_train_forward(cuda, dt, B, W, K, N):
    """The training-forward form (svk_mixffn_dw_fc2_packed_ex, round 6): Y = rscale[frame] * (GELU(dwconv3x3(h) +
    dbias) W2^T + b2) + R with the pre-activation U stored, against the path it replaces in svk/train.py
    (dwconv3x3(pre_out=) + gemm(row_scale, residual): U within a 16-bit ulp — the mx form rounds its taps to the
    16-bit type — and Y within a few ulps) and fp64 (taps rounded as the mx form rounds them)."""
    from svk import ops
    h = _rand(B, W, W, K, dt=dt, dev=cuda, seed=171)
    taps = _rand(9, K, dt=torch.float32, dev=cuda, scale=0.3, seed=172)
    db = _rand(K, dt=torch.float32, dev=cuda, scale=0.1, seed=173)
    w2 = _rand(N, K, dt=dt, dev=cuda, scale=K ** -0.5, seed=174)
    b2 = _rand(N, dt=torch.float32, dev=cuda, seed=175)
    r = _rand(B, W * W, N, dt=dt, dev=cuda, seed=176)
    keep = torch.tensor([(0.0 if i % 3 == 1 else 1.25) for i in range(B)], device=cuda)   # DropPath scales
    pk = ops.mixffn_dw_fc2_pack(taps, db, w2, W)
    u = torch.empty_like(h)
    got = ops.mixffn_dw_fc2(h, taps, db, w2, b2, residual=r, packed=pk, pre_out=u, row_scale=keep, rows_per=W * W)
    assert ops._last_kernel().startswith("dw_fc2_mx"), ops._last_kernel()
    u16 = torch.empty_like(h)
    g = ops.dwconv3x3(h, taps, db, act="gelu", pre_out=u16)
    ref16 = ops.gemm(g.view(B, W * W, K), w2, b2, residual=r, row_scale=keep, rows_per=W * W)
    ulp = 2 ** -8 if dt == torch.bfloat16 else 2 ** -11
    du = (u.float() - u16.float()).abs().max().item()
    assert du <= 2 * ulp * float(u16.float().abs().max()), du
    d = (got.float() - ref16.float()).abs().max().item()
    assert d <= 4 * ulp * float(ref16.float().abs().max()), d
    tq = taps.to(dt).double().cpu()                                     # the mx form's 16-bit taps
    hd = h.double().cpu().permute(0, 3, 1, 2)
    cv = F.conv2d(hd, tq.t().reshape(K, 1, 3, 3), db.double().cpu(), padding=1, groups=K)
    _close(u, cv.permute(0, 2, 3, 1), dt)
    gd = F.gelu(cv).permute(0, 2, 3, 1).reshape(B, W * W, K)
    ref = (gd @ w2.double().cpu().t() + b2.double().cpu()) * keep.double().cpu().view(B, 1, 1) + r.double().cpu()
    _close(got, ref, dt)


@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("M,N,K,res,bias", [(50176, 320, 320, True, True), (12544, 512, 512, True, True),
                                            (1000, 320, 80, True, True), (77, 512, 128, True, False),
                                            (130, 320, 40, False, True)])
def test_gemm_ln(cuda, dt, M, N, K, res, bias, monkeypatch):
    """svk_gemm_ln (proj / shared-MLP GEMM + bias + residual + LayerNorm over the full row, packed weights)
    against the unfused svk path (gemm, then layernorm of its rounded output: X bit-identical up to the MFMA
    summation order, H within a few 16-bit ulps) and fp64; ragged M, K tails (80, 40: zero-filled fragments)."""
    from svk import ops
    monkeypatch.setattr(ops, "GEMM_LN", True)
    a = _rand(M, K, dt=dt, dev=cuda, seed=81)
    w = _rand(N, K, dt=dt, dev=cuda, scale=K ** -0.5, seed=82)
    b = _rand(N, dt=torch.float32, dev=cuda, scale=0.1, seed=83) if bias else None
    r = _rand(M, N, dt=dt, dev=cuda, seed=84) if res else None
    g = 1 + _rand(N, dt=torch.float32, dev=cuda, scale=0.1, seed=85)
    bt = _rand(N, dt=torch.float32, dev=cuda, scale=0.1, seed=86)
    pk = ops.gemm_ln_pack(w)
    assert pk is not None
    x, h = ops.gemm_ln(a, pk, N, b, r, g, bt, 1e-6)
    assert ops._last_kernel().startswith("gemm_ln"), ops._last_kernel()
    x16 = ops.gemm(a, w, b, residual=r)
    h16 = ops.layernorm(x16, g, bt, 1e-6)
    ulp = 2 ** -8 if dt == torch.bfloat16 else 2 ** -11
    assert (x.float() - x16.float()).abs().max().item() <= 2 * ulp * max(1.0, x16.float().abs().max().item())
    assert (h.float() - h16.float()).abs().max().item() <= 4 * ulp * max(1.0, h16.float().abs().max().item())
    xd = a.double().cpu() @ w.double().cpu().t() + (b.double().cpu() if bias else 0) + (r.double().cpu() if res else 0)
    hd = F.layer_norm(xd, (N,), g.double().cpu(), bt.double().cpu(), 1e-6)
    _close(x, xd, dt)
    _close(h, hd, dt)


@pytest.mark.parametrize("lds,rows", [(1, 1), (1, 3), (1, 8), (2, -1), (0, -1)])
def test_dwconv_lds_variant(cuda, lds, rows):
    """The LDS-tiled depthwise conv (svk_tune dw_lds = 1) at several strip heights, with the
    pre-activation store, against fp64."""
    from svk import ops
    dt = torch.bfloat16
    try:
        ops.tune("dw_lds", lds)
        ops.tune("dw_rows", rows)
        for B, H, W, C in ((2, 28, 28, 256), (3, 7, 7, 128), (1, 10, 13, 64), (2, 19, 5, 68)):
            x = _rand(B, H, W, C, dt=dt, dev=cuda, seed=61)
            w = _rand(C, 1, 3, 3, dt=torch.float32, dev="cpu", scale=0.4, seed=62)
            b = _rand(C, dt=torch.float32, dev=cuda, seed=63)
            pre = torch.empty_like(x)
            got = ops.dwconv3x3(x, w.reshape(C, 9).t().contiguous().to(cuda), b, act="gelu", pre_out=pre)
            ref = F.conv2d(x.cpu().double().permute(0, 3, 1, 2), w.double(), b.cpu().double(), padding=1, groups=C)
            _close(pre, ref.permute(0, 2, 3, 1), dt)
            _close(got, F.gelu(ref).permute(0, 2, 3, 1), dt)
    finally:
        ops.tune("dw_lds", -1)
        ops.tune("dw_rows", -1)


def test_dwconv_identity_default_is_bit_exact_across_kernels(cuda):
    """The activation-free bf16 depthwise conv (the train step's data gradient: flipped taps, zero bias) runs the
    rolling-window kernel by default (round 6); it must equal the strip and LDS kernels bit for bit (same f32 tap
    order) and fp64 to bf16 rounding — including C % 8 != 0 and maps whose height is not a multiple of the strip."""
    from svk import ops
    dt = torch.bfloat16
    try:
        for B, H, W, C in ((3, 56, 56, 64), (2, 28, 28, 512), (2, 14, 14, 1280), (3, 7, 7, 2048), (2, 19, 5, 68)):
            x = _rand(B, H, W, C, dt=dt, dev=cuda, seed=71)
            w = _rand(C, 1, 3, 3, dt=torch.float32, dev="cpu", scale=0.4, seed=72)
            taps, zero = w.reshape(C, 9).t().contiguous().to(cuda), torch.zeros(C, device=cuda)
            outs = []
            for lds in (-1, 0, 1):
                ops.tune("dw_lds", lds)
                outs.append(ops.dwconv3x3(x, taps, zero))
            for o in outs[1:]:
                assert torch.equal(o, outs[0]), (B, H, W, C)
            ref = F.conv2d(x.cpu().double().permute(0, 3, 1, 2), w.double(), None, padding=1, groups=C)
            _close(outs[0], ref.permute(0, 2, 3, 1), dt)
    finally:
        ops.tune("dw_lds", -1)


@pytest.mark.parametrize("kind", ["conv", "gemm"])
def test_persistent_ktail_ignores_weight_slack(cuda, kind):
    """K-tail steps of the persistent kernel read a zero block for BOTH operands: the bytes past the
    last weight row (NaN here) must never reach the accumulators (0 x NaN = NaN).  Regression for the
    im2col conv path, whose weight loads once ran past the packed weights on K % 64 != 0."""
    from svk import ops
    dt = torch.bfloat16
    if kind == "conv":
        B, H, W, Cin, Cout, k, s, p = 16, 224, 224, 8, 64, 7, 4, 3
        K = k * k * Cin                                     # 392 = 6 x 64 + 8
        x = _rand(B, H, W, Cin, dt=dt, dev=cuda, seed=31)
    else:
        M, Cout, K = 30000, 64, 200
        x = _rand(M, K, dt=dt, dev=cuda, seed=31)
    buf = torch.full((Cout * K + 4096,), float("nan"), device=cuda, dtype=dt)
    w = buf[:Cout * K].view(Cout, K)
    w.copy_(_rand(Cout, K, dt=dt, dev=cuda, scale=K ** -0.5, seed=32))
    b = _rand(Cout, dt=torch.float32, dev=cuda, seed=33)
    if kind == "conv":
        got = ops.conv2d_nhwc(x, w, k, s, p, bias=b)
        wr = w.double().cpu().view(Cout, k, k, Cin).permute(0, 3, 1, 2)
        ref = F.conv2d(x.cpu().double().permute(0, 3, 1, 2), wr, b.cpu().double(), stride=s, padding=p)
        ref = ref.permute(0, 2, 3, 1)
    else:
        got = ops.gemm(x, w, b)
        ref = x.cpu().double() @ w.cpu().double().t() + b.cpu().double()
    torch.cuda.synchronize()
    assert bool(torch.isfinite(got).all())
    _close(got, ref, dt)


@pytest.mark.parametrize("dt", DTS)
def test_gemm_strided_views(cuda, dt):
    """kv[:, :, :C] style inputs and writes into a column slice (head concat buffer)."""
    from svk import ops
    a_full = _rand(3, 50, 96, dt=dt, dev=cuda, seed=5)
    a = a_full[:, :, 16:80]                       # row stride 96, K = 64
    w = _rand(40, 64, dt=dt, dev=cuda, scale=0.125, seed=6)
    out_full = torch.zeros(3, 50, 100, device=cuda, dtype=dt)
    ops.gemm(a, w, out=out_full[:, :, 30:70])
    torch.cuda.synchronize()
    ref = a.cpu().double() @ w.cpu().double().t()
    _close(out_full[:, :, 30:70], ref, dt)
    assert float(out_full[:, :, :30].abs().max()) == 0 and float(out_full[:, :, 70:].abs().max()) == 0


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("B,H,W,Cin,Cout,k,s,p", [(2, 224, 224, 3, 64, 7, 4, 3), (2, 56, 56, 64, 128, 3, 2, 1),
                                                  (3, 56, 56, 64, 64, 8, 8, 0), (2, 224, 224, 2, 64, 7, 4, 3),
                                                  (1, 14, 14, 320, 512, 3, 2, 1), (2, 28, 28, 32, 80, 3, 2, 1),
                                                  (2, 14, 14, 320, 320, 2, 2, 0), (24, 224, 224, 8, 64, 7, 4, 3),
                                                  (24, 224, 224, 8, 16, 7, 4, 3), (40, 56, 56, 64, 64, 8, 8, 0),
                                                  (30, 28, 28, 128, 320, 3, 2, 1), (9, 14, 14, 320, 512, 3, 2, 1)])
def test_conv2d_nhwc(cuda, dt, B, H, W, Cin, Cout, k, s, p):
    from svk import ops
    from svk.pack import conv_w
    x = _rand(B, H, W, Cin, dt=dt, dev=cuda, seed=7)
    w = _rand(Cout, Cin, k, k, dt=torch.float32, dev="cpu", scale=(Cin * k * k) ** -0.5, seed=8).to(dt)
    b = _rand(Cout, dt=torch.float32, dev=cuda, seed=9)
    got = ops.conv2d_nhwc(x, conv_w(w, dt).to(cuda), k, s, p, bias=b, act="relu")
    torch.cuda.synchronize()
    ref = F.conv2d(x.cpu().double().permute(0, 3, 1, 2), w.double(), b.cpu().double(), stride=s, padding=p)
    _close(got, torch.relu(ref).permute(0, 2, 3, 1), dt)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("M,C,eps", [(1000, 64, 1e-6), (333, 320, 1e-5), (64, 512, 1e-6), (17, 14, 1e-5),
                                     (9, 2048, 1e-5), (5, 16, 1e-5)])
def test_layernorm(cuda, dt, M, C, eps):
    from svk import ops
    x = _rand(M, C, dt=dt, dev=cuda, scale=3.0, seed=10) + 0.5
    g = _rand(C, dt=torch.float32, dev=cuda, seed=11)
    b = _rand(C, dt=torch.float32, dev=cuda, seed=12)
    got = ops.layernorm(x, g, b, eps)
    torch.cuda.synchronize()
    ref = F.layer_norm(x.cpu().double(), (C,), g.cpu().double(), b.cpu().double(), eps)
    _close(got, ref, dt)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("B,Nq,Nk,heads,hd", [(2, 3136, 49, 1, 64), (2, 784, 49, 2, 64), (3, 196, 196, 8, 40),
                                              (2, 49, 49, 8, 64), (5, 30, 30, 4, 32), (7, 1, 1, 4, 32),
                                              (2, 196, 49, 5, 32), (1, 100, 256, 1, 64)])
def test_attention(cuda, monkeypatch, dt, B, Nq, Nk, heads, hd):
    """16-bit: the resident-K/V kernel with its default 256-query block, and 64- / 256-query blocks forced
    (SVK_ATTN_QB; round 6) — bit-identical to each other (same per-tile arithmetic) and within tolerance of fp64."""
    from svk import ops
    C = heads * hd
    q = _rand(B, Nq, C, dt=dt, dev=cuda, seed=13)
    kv = _rand(B, Nk, 2 * C, dt=dt, dev=cuda, seed=14)
    k, v = kv[:, :, :C], kv[:, :, C:]
    scale = hd ** -0.5
    got = ops.attention(q, k, v, heads, scale)
    if dt != torch.float32:
        for qb in ("64", "256"):
            monkeypatch.setenv("SVK_ATTN_QB", qb)
            assert torch.equal(ops.attention(q, k, v, heads, scale), got), qb
        monkeypatch.delenv("SVK_ATTN_QB")
    torch.cuda.synchronize()
    qh = q.cpu().double().reshape(B, Nq, heads, hd).transpose(1, 2)
    kh = k.cpu().double().reshape(B, Nk, heads, hd).transpose(1, 2)
    vh = v.cpu().double().reshape(B, Nk, heads, hd).transpose(1, 2)
    ref = ((qh @ kh.transpose(-1, -2)) * scale).softmax(-1) @ vh
    _close(got, ref.transpose(1, 2).reshape(B, Nq, C), dt)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("B,H,W,C", [(2, 56, 56, 256), (1, 7, 7, 2048), (2, 14, 14, 1280), (1, 5, 6, 12),
                                     (3, 28, 28, 512), (2, 30, 17, 128), (1, 9, 3, 64)])
def test_dwconv3x3_gelu(cuda, dt, B, H, W, C):
    from svk import ops
    x = _rand(B, H, W, C, dt=dt, dev=cuda, seed=15)
    w = _rand(C, 1, 3, 3, dt=torch.float32, dev="cpu", scale=0.4, seed=16)
    b = _rand(C, dt=torch.float32, dev=cuda, seed=17)
    got = ops.dwconv3x3(x, w.reshape(C, 9).t().contiguous().to(cuda), b, act="gelu")
    torch.cuda.synchronize()
    ref = F.conv2d(x.cpu().double().permute(0, 3, 1, 2), w.double(), b.cpu().double(), padding=1, groups=C)
    _close(got, F.gelu(ref).permute(0, 2, 3, 1), dt)


@pytest.mark.parametrize("B,H,ln", [(2, 56, False), (2, 56, True), (1, 10, True), (3, 7, False), (5, 3, False),
                                    (1, 15, True), (9, 28, False)])
def test_mixffn_rw(cuda, B, H, ln):
    """Register-window whole MixFFN (svk_mixffn_rw, f16, W = 56, C = 64) against fp64 torch on the same
    rounded inputs (rounding points as test_mixffn_fused).  H = 10 / 7 / 3 / 15 leave partial strips
    (rows past the map are masked, the window's halo rows are zero there); B = 9 gives more units than one
    pass of the persistent grid when few CUs are free."""
    from svk import ops
    dt, W, C = torch.float16, 56, 64
    assert ops.mixffn_rw_supported(dt, W, C)
    xn = _rand(B, H, W, C, dt=dt, dev=cuda, seed=40)
    x = _rand(B, H, W, C, dt=dt, dev=cuda, seed=41)
    w1 = _rand(4 * C, C, dt=dt, dev=cuda, scale=C ** -0.5, seed=42)
    b1 = _rand(4 * C, dt=torch.float32, dev=cuda, scale=0.1, seed=43)
    taps = _rand(9, 4 * C, dt=torch.float32, dev=cuda, scale=0.3, seed=44)
    db = _rand(4 * C, dt=torch.float32, dev=cuda, scale=0.1, seed=45)
    w2 = _rand(C, 4 * C, dt=dt, dev=cuda, scale=(4 * C) ** -0.5, seed=46)
    b2 = _rand(C, dt=torch.float32, dev=cuda, scale=0.1, seed=47)
    gam = (1 + _rand(C, dt=torch.float32, dev=cuda, scale=0.2, seed=48)) if ln else None
    bet = _rand(C, dt=torch.float32, dev=cuda, scale=0.1, seed=49) if ln else None
    got = ops.mixffn_rw(xn, x, w1, b1, taps, db, w2, b2, ln=(gam, bet, 1e-6) if ln else None)
    torch.cuda.synchronize()
    h = (xn.cpu().double() @ w1.cpu().double().t() + b1.cpu().double()).to(dt).double()
    hc = h.permute(0, 3, 1, 2)
    k = taps.cpu().to(dt).double().t().reshape(4 * C, 1, 3, 3)
    g = F.gelu(F.conv2d(hc, k, db.cpu().double(), padding=1, groups=4 * C)).permute(0, 2, 3, 1).to(dt).double()
    ref = x.cpu().double() + g @ w2.cpu().double().t() + b2.cpu().double()
    if ln:
        ref = F.layer_norm(ref.to(dt).double(), (C,), gam.cpu().double(), bet.cpu().double(), 1e-6)
    _close(got, ref, dt)
    # the register-window kernel and the wave-specialised one compute the same rounded quantities
    alt = ops.mixffn_fused(xn, x, w1, b1, ops.mixffn_pack_taps(taps, db, dt), w2, b2,
                           ln=(gam, bet, 1e-6) if ln else None)
    assert (got.float() - alt.float()).abs().max().item() <= 2e-2


@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("B,H,W,C,ln", [(2, 56, 56, 64, False), (2, 56, 56, 32, False), (1, 10, 56, 64, True),
                                        (3, 7, 56, 32, True), (2, 56, 56, 64, True), (5, 3, 56, 64, False)])
def test_mixffn_fused(cuda, dt, B, H, W, C, ln):
    """Whole MixFFN (fc1 -> dwconv3x3 -> GELU -> fc2 + residual [-> LayerNorm]) in one kernel against
    fp64 torch on the same rounded inputs.  The reference rounds where the kernel stores in the map
    dtype: the fc1 output (hidden, on chip), the depthwise taps (autocast casts the conv weight too) and
    the GELU output; H = 7 / 3 leave a partial last strip, B = 5 more strips than one pass of the
    persistent grid covers when few CUs are free (the pipeline runs across strips)."""
    from svk import ops
    assert ops.mixffn_supported(W, C)
    xn = _rand(B, H, W, C, dt=dt, dev=cuda, seed=40)
    x = _rand(B, H, W, C, dt=dt, dev=cuda, seed=41)
    w1 = _rand(4 * C, C, dt=dt, dev=cuda, scale=C ** -0.5, seed=42)
    b1 = _rand(4 * C, dt=torch.float32, dev=cuda, scale=0.1, seed=43)
    taps = _rand(9, 4 * C, dt=torch.float32, dev=cuda, scale=0.3, seed=44)
    db = _rand(4 * C, dt=torch.float32, dev=cuda, scale=0.1, seed=45)
    w2 = _rand(C, 4 * C, dt=dt, dev=cuda, scale=(4 * C) ** -0.5, seed=46)
    b2 = _rand(C, dt=torch.float32, dev=cuda, scale=0.1, seed=47)
    gam = (1 + _rand(C, dt=torch.float32, dev=cuda, scale=0.2, seed=48)) if ln else None
    bet = _rand(C, dt=torch.float32, dev=cuda, scale=0.1, seed=49) if ln else None
    got = ops.mixffn_fused(xn, x, w1, b1, ops.mixffn_pack_taps(taps, db, dt), w2, b2, ln=(gam, bet, 1e-6) if ln else None)
    torch.cuda.synchronize()
    h = (xn.cpu().double() @ w1.cpu().double().t() + b1.cpu().double()).to(dt).double()
    hc = h.permute(0, 3, 1, 2)
    k = taps.cpu().to(dt).double().t().reshape(4 * C, 1, 3, 3)
    g = F.gelu(F.conv2d(hc, k, db.cpu().double(), padding=1, groups=4 * C)).permute(0, 2, 3, 1).to(dt).double()
    ref = x.cpu().double() + g @ w2.cpu().double().t() + b2.cpu().double()
    if ln:
        ref = F.layer_norm(ref.to(dt).double(), (C,), gam.cpu().double(), bet.cpu().double(), 1e-6)
    _close(got, ref, dt)


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("shape", [(2, 3, 224, 224), (1, 3, 13, 32), (2, 1, 20, 8), (1, 2, 9, 12)])
def test_pack_and_gauss(cuda, dt, shape):
    from svk import ops
    x = _rand(*shape, dt=torch.float32, dev=cuda, seed=18)
    C = shape[1]
    got = ops.nchw_to_nhwc(x, dt)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), x.cpu().permute(0, 2, 3, 1).to(dt))
    gg = ops.gauss5x5_reflect(x, dt)
    torch.cuda.synchronize()
    k = torch.tensor([1., 4., 6., 4., 1.], dtype=torch.float64)
    k = (torch.outer(k, k) / 256.).repeat(C, 1, 1, 1)
    ref = F.conv2d(F.pad(x.cpu().double(), (2, 2, 2, 2), mode="reflect"), k, groups=C)
    _close(gg, ref.permute(0, 2, 3, 1), dt)
    # channel padding to 8 (vector path of the first convs): padded channels are exactly zero
    p8 = ops.nchw_to_nhwc(x, dt, cpad=8)
    g8 = ops.gauss5x5_reflect(x, dt, cpad=8)
    torch.cuda.synchronize()
    # (cpad = 8 takes the 4-column vector kernel when W % 4 == 0: bitwise equal to the scalar one)
    assert torch.equal(p8[..., :C].cpu(), got.cpu()) and float(p8[..., C:].abs().max()) == 0
    assert torch.equal(g8[..., :C].cpu(), gg.cpu()) and float(g8[..., C:].abs().max()) == 0


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("H,OH", [(56, 7), (28, 7), (14, 7), (7, 7), (10, 4)])
def test_resize_bilinear(cuda, dt, H, OH):
    from svk import ops
    C = 24
    x = _rand(2, H * H, C, dt=dt, dev=cuda, seed=19)
    out = torch.zeros(2, OH * OH, 2 * C, device=cuda, dtype=dt)
    ops.resize_bilinear(x, H, H, OH, OH, out=out[:, :, C:])
    torch.cuda.synchronize()
    ref = F.interpolate(x.cpu().double().transpose(1, 2).reshape(2, C, H, H), (OH, OH), None, "bilinear", False)
    _close(out[:, :, C:], ref.flatten(2).transpose(1, 2), dt)
    assert float(out[:, :, :C].abs().max()) == 0


@pytest.mark.parametrize("dt", [d for d in DTS if d != torch.float32])
@pytest.mark.parametrize("OH", [7, 4])
def test_resize_bilinear_multi(cuda, dt, OH):
    """The head's four resizes in one launch (svk_resize_bilinear_multi) equal four resize_bilinear calls
    bit for bit, each level at its channel offset of the concatenated row (row stride beyond the levels,
    one level a strided view)."""
    from svk import ops
    dims = [(7, 40), (14, 32), (28, 16), (56, 8)]
    srcs = []
    for i, (H, C) in enumerate(dims):
        t = _rand(3, H * H, 2 * C if i == 1 else C, dt=dt, dev=cuda, seed=60 + i)
        srcs.append((t[:, :, :C] if i == 1 else t, H, H))
    ctot = sum(C for _, C in dims)
    got = torch.full((3, OH * OH, ctot + 8), 7.0, device=cuda, dtype=dt)
    ops.resize_bilinear_multi(srcs, OH, OH, got)
    ref = torch.full_like(got, 7.0)
    off = 0
    for t, H, W in srcs:
        C = t.shape[-1]
        ops.resize_bilinear(t, H, W, OH, OH, out=ref[:, :, off:off + C])
        off += C
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), ref.cpu())


def test_keep_mask_multi(cuda):
    """svk_keep_mask_multi (the train step's DropPath masks in one launch) equals one svk_keep_mask per mask bit
    for bit, with and without the device step counter, seeds past 2^31 included."""
    from svk import ops
    keeps = [1.0 - r for r in (0.0125, 0.05, 0.3, 0.7, 0.9)]
    seeds = [12345, 0x7FFFFFF0 + 17, 0xFFFFFFF0, 3, 0x80000001]
    kt = torch.tensor(keeps, dtype=torch.float32).to(cuda)
    st = torch.tensor([v - (1 << 32) if v >= 1 << 31 else v for v in seeds], dtype=torch.int32).to(cuda)
    for counter in (None, torch.tensor([41], dtype=torch.int64, device=cuda)):
        got = ops.keep_mask_multi(88, kt, st, counter)
        for m, (k, sd) in enumerate(zip(keeps, seeds)):
            assert torch.equal(got[m], ops.keep_mask(88, k, sd, cuda, counter)), m


@pytest.mark.parametrize("dt", DTS)
def test_mean_rows(cuda, dt):
    from svk import ops
    x = _rand(5 * 49, 2048, dt=dt, dev=cuda, seed=20)
    got = ops.mean_rows(x, 49)
    torch.cuda.synchronize()
    torch.testing.assert_close(got.cpu().double(), x.cpu().double().reshape(5, 49, 2048).mean(1), rtol=1e-5, atol=1e-5)


def test_softmax_rows(cuda):
    from svk import ops
    x = _rand(1000, 14, dt=torch.float32, dev=cuda, scale=4.0, seed=21)
    got = ops.softmax_rows(x)
    torch.cuda.synchronize()
    torch.testing.assert_close(got.cpu().double(), x.cpu().double().softmax(-1), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("F_,T,d,causal", [(32, 300, 1, True), (32, 300, 64, True), (64, 2456, 512, True),
                                           (64, 130, 4, False), (32, 77, 128, False), (20, 50, 2, True)])
def test_mstcn_layer(cuda, F_, T, d, causal):
    from svk import ops
    x = _rand(T, F_, dt=torch.float32, dev=cuda, seed=22)
    wd = _rand(F_, F_, 3, dt=torch.float32, dev="cpu", scale=F_ ** -0.5, seed=23)
    bd = _rand(F_, dt=torch.float32, dev=cuda, seed=24)
    w1 = _rand(F_, F_, dt=torch.float32, dev=cuda, scale=F_ ** -0.5, seed=25)
    b1 = _rand(F_, dt=torch.float32, dev=cuda, seed=26)
    got = ops.mstcn_layer(x, wd.permute(2, 1, 0).contiguous().to(cuda), bd, w1.t().contiguous(), b1, d, causal)
    torch.cuda.synchronize()
    xc = x.cpu().double().t()[None]
    pad = 2 * d if causal else d
    h = torch.relu(F.conv1d(xc, wd.double(), bd.cpu().double(), padding=pad, dilation=d))
    if causal:
        h = h[:, :, :-2 * d]
    ref = xc + F.conv1d(h, w1.cpu().double()[:, :, None], b1.cpu().double())
    torch.testing.assert_close(got.cpu().double(), ref[0].t(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("F_,d,causal", [(64, 8, True), (64, 512, True), (32, 4, False), (20, 2, True)])
def test_mstcn_layer_ragged_equals_per_video(cuda, F_, d, causal):
    """One launch over a ragged batch (incl. empty and 1-frame videos, lengths not multiples of the tile)
    == the single-video kernel on each video, bit for bit (taps never cross a video boundary)."""
    from svk import ops
    lens = [1, 0, 17, 300, 16, 2457, 33]
    x = _rand(sum(lens), F_, dt=torch.float32, dev=cuda, seed=27)
    wd = _rand(F_, F_, 3, dt=torch.float32, dev="cpu", scale=F_ ** -0.5, seed=23).permute(2, 1, 0).contiguous().to(cuda)
    bd = _rand(F_, dt=torch.float32, dev=cuda, seed=24)
    w1 = _rand(F_, F_, dt=torch.float32, dev=cuda, scale=F_ ** -0.5, seed=25).t().contiguous()
    b1 = _rand(F_, dt=torch.float32, dev=cuda, seed=26)
    got = ops.mstcn_layer(x, wd, bd, w1, b1, d, causal, tiles=ops.mstcn_tiles(lens, cuda))
    o = 0
    for T in lens:
        if T:
            one = ops.mstcn_layer(x[o:o + T].contiguous(), wd, bd, w1, b1, d, causal)
            assert torch.equal(got[o:o + T], one), f"video of length {T} differs"
        o += T
    torch.cuda.synchronize()


@pytest.mark.parametrize("F_,T,d,causal", [(64, 1000, 8, True), (32, 77, 128, False), (20, 50, 2, True),
                                           (64, 6001, 512, True)])
def test_mstcn_layer_train_bwd(cuda, F_, T, d, causal):
    """Train-mode layer (dropout mask) forward and its backward kernels against fp64 autograd."""
    from svk import ops
    x = _rand(T, F_, dt=torch.float32, dev=cuda, seed=32)
    wd = _rand(F_, F_, 3, dt=torch.float32, dev="cpu", scale=F_ ** -0.5, seed=33)
    bd = _rand(F_, dt=torch.float32, dev=cuda, seed=34)
    w1 = _rand(F_, F_, dt=torch.float32, dev=cuda, scale=F_ ** -0.5, seed=35)
    b1 = _rand(F_, dt=torch.float32, dev=cuda, seed=36)
    mask = ops.keep_mask(T * F_, 0.5, 7, cuda).view(T, F_)
    dy = _rand(T, F_, dt=torch.float32, dev=cuda, seed=37)
    y, h = ops.mstcn_layer_train(x, wd.permute(2, 1, 0).contiguous().to(cuda), bd, w1.t().contiguous(), b1, d, causal,
                                 mask)
    dwd = torch.zeros(F_, F_, 3, device=cuda)
    dbd, dw1, db1 = torch.zeros(F_, device=cuda), torch.zeros(F_, F_, device=cuda), torch.zeros(F_, device=cuda)
    dx = ops.mstcn_layer_bwd(x, h, mask, dy, wd.permute(2, 0, 1).contiguous().to(cuda), w1, dwd, dbd, dw1, db1, d,
                             causal)
    torch.cuda.synchronize()
    xr = x.cpu().double().t()[None].requires_grad_(True)
    pr = [t.cpu().double().requires_grad_(True) for t in (wd, bd, w1, b1)]
    pad = 2 * d if causal else d
    hr = torch.relu(F.conv1d(xr, pr[0], pr[1], padding=pad, dilation=d))
    if causal:
        hr = hr[:, :, :-2 * d]
    ref = xr + F.conv1d(hr, pr[2][:, :, None], pr[3]) * mask.cpu().double().t()[None]
    torch.testing.assert_close(y.cpu().double(), ref[0].t().detach(), rtol=1e-5, atol=1e-5)
    ref.backward(dy.cpu().double().t()[None])
    torch.testing.assert_close(dx.cpu().double(), xr.grad[0].t(), rtol=1e-4, atol=1e-4)
    for got, r in ((dwd, pr[0]), (dbd, pr[1]), (dw1, pr[2]), (db1, pr[3])):
        scale = r.grad.abs().max().item()
        assert (got.cpu().double() - r.grad).abs().max().item() <= 1e-4 * max(scale, 1.0)


@pytest.mark.parametrize("dt", DTS)
def test_window_unfold_and_add(cuda, dt):
    from svk import ops
    x = _rand(75, 14, dt=dt, dev=cuda, seed=27)
    pos = _rand(30, 14, dt=torch.float32, dev=cuda, seed=28)
    got = ops.window_unfold(x, 30, pos=pos)
    torch.cuda.synchronize()
    xc = x.cpu().double()
    padded = torch.cat([torch.zeros(29, 14, dtype=torch.float64), xc], 0)
    ref = padded.unfold(0, 30, 1).transpose(1, 2) + pos.cpu().double()
    _close(got, ref, dt)
    plain = ops.window_unfold(x, 30)
    added = ops.add_bcast(plain, pos)
    torch.cuda.synchronize()
    _close(added, ref, dt)


def test_cast(cuda):
    from svk import ops
    x = _rand(1001, dt=torch.float32, dev=cuda, seed=29)
    y = ops.cast(x, torch.bfloat16)
    z = ops.cast(y, torch.float32)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), x.cpu().to(torch.bfloat16))
    assert torch.equal(z.cpu(), y.cpu().float())


@pytest.mark.parametrize("dt", DTS)
@pytest.mark.parametrize("B,H,Cin,r", [(256, 56, 64, 8), (256, 28, 128, 4), (256, 14, 320, 2), (3, 56, 64, 8),
                                       (5, 28, 128, 4)])
def test_conv2d_ln_sequence_reduction(cuda, dt, B, H, Cin, r):
    """Attention.sr + Attention.norm as one call (split-K slabs reduced inside the LayerNorm for the
    long-K bf16 patchify convs at B = 256) against fp64 conv + LayerNorm."""
    from svk import ops
    from svk.pack import conv_w
    x = _rand(B, H, H, Cin, dt=dt, dev=cuda, seed=71)
    w = _rand(Cin, Cin, r, r, dt=torch.float32, dev="cpu", scale=(Cin * r * r) ** -0.5, seed=72).to(dt)
    b = _rand(Cin, dt=torch.float32, dev=cuda, seed=73)
    g = _rand(Cin, dt=torch.float32, dev=cuda, seed=74)
    be = _rand(Cin, dt=torch.float32, dev=cuda, seed=75)
    got = ops.conv2d_ln_nhwc(x, conv_w(w, dt).to(cuda), r, r, 0, b, g, be, 1e-5)
    torch.cuda.synchronize()
    nb = min(B, 4)                                   # fp64 reference on a few frames (frames are independent)
    ref = F.conv2d(x[:nb].cpu().double().permute(0, 3, 1, 2), w.double(), b.cpu().double(), stride=r)
    ref = F.layer_norm(ref.permute(0, 2, 3, 1), (Cin,), g.cpu().double(), be.cpu().double(), 1e-5)
    _close(got[:nb], ref, dt)
    assert bool(torch.isfinite(got).all())


@pytest.mark.parametrize("B,H,W,C", [(2, 56, 56, 64), (3, 28, 28, 128), (2, 14, 14, 128), (4, 7, 7, 64),
                                     (1, 9, 13, 32), (2, 30, 17, 64), (9, 28, 28, 128), (2, 13, 28, 128),
                                     (1, 33, 28, 128), (3, 14, 14, 320), (2, 7, 7, 512), (1, 17, 9, 320)])
@pytest.mark.parametrize("dt", H16)
def test_mixffn_fc1_dwconv(cuda, B, H, W, C, dt):
    """fc1 -> dwconv3x3 -> GELU in one kernel (hidden kept on chip) against the unfused svk kernels
    (fc1 GEMM, 16-bit hidden, depthwise conv) and fp64 torch on the same 16-bit-rounded hidden."""
    from svk import ops
    hid = 4 * C
    xn = _rand(B, H, W, C, dt=dt, dev=cuda, seed=81)
    w1 = _rand(hid, C, dt=dt, dev=cuda, scale=C ** -0.5, seed=82)
    b1 = _rand(hid, dt=torch.float32, dev=cuda, scale=0.1, seed=83)
    taps = _rand(9, hid, dt=torch.float32, dev=cuda, scale=0.3, seed=84)
    db = _rand(hid, dt=torch.float32, dev=cuda, scale=0.1, seed=85)
    got = ops.mixffn_fc1_dwconv(xn, w1, b1, taps, db, act="gelu")
    h = ops.gemm(xn.view(B, H * W, C), w1, b1).view(B, H, W, hid)
    unfused = ops.dwconv3x3(h, taps, db, act="gelu")
    torch.cuda.synchronize()
    _close(got, unfused.double().cpu(), dt)
    hr = (xn.cpu().double() @ w1.cpu().double().t() + b1.cpu().double()).to(dt).double()
    k = taps.cpu().double().t().reshape(hid, 1, 3, 3)
    ref = F.gelu(F.conv2d(hr.permute(0, 3, 1, 2), k, db.cpu().double(), padding=1, groups=hid)).permute(0, 2, 3, 1)
    _close(got, ref, dt)


@pytest.mark.parametrize("B,H,W,C", [(2, 56, 56, 64), (3, 28, 28, 128), (2, 14, 14, 320), (2, 7, 7, 512),
                                     (1, 30, 17, 64)])
@pytest.mark.parametrize("dt", H16)
def test_mixffn_fc1_dwconv_pre_out(cuda, B, H, W, C, dt):
    """The training forward's fused MixFFN front half: G and the pre-activation map equal the unfused chain the
    train step ran before (fc1 GEMM -> dwconv3x3(pre_out=) -> GELU) within one storage ulp, and the
    pre-activation equals fp64 torch on the same 16-bit-rounded hidden."""
    from svk import ops
    hid = 4 * C
    xn = _rand(B, H, W, C, dt=dt, dev=cuda, seed=91)
    w1 = _rand(hid, C, dt=dt, dev=cuda, scale=C ** -0.5, seed=92)
    b1 = _rand(hid, dt=torch.float32, dev=cuda, scale=0.1, seed=93)
    taps = _rand(9, hid, dt=torch.float32, dev=cuda, scale=0.3, seed=94)
    db = _rand(hid, dt=torch.float32, dev=cuda, scale=0.1, seed=95)
    pre = torch.full((B, H, W, hid), float("nan"), device=cuda, dtype=dt)
    got = ops.mixffn_fc1_dwconv(xn, w1, b1, taps, db, act="gelu", pre_out=pre)
    h = ops.gemm(xn.view(B, H * W, C), w1, b1).view(B, H, W, hid)
    pre_u = torch.empty_like(pre)
    unfused = ops.dwconv3x3(h, taps, db, act="gelu", pre_out=pre_u)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(pre).all())
    _close(got, unfused.double().cpu(), dt)
    _close(pre, pre_u.double().cpu(), dt)
    hr = (xn.cpu().double() @ w1.cpu().double().t() + b1.cpu().double()).to(dt).double()
    k = taps.cpu().double().t().reshape(hid, 1, 3, 3)
    ref = F.conv2d(hr.permute(0, 3, 1, 2), k, db.cpu().double(), padding=1, groups=hid).permute(0, 2, 3, 1)
    _close(pre, ref, dt)
    _close(got, F.gelu(ref), dt)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B,N,Nk,C", [(2, 3136, 49, 64), (3, 300, 64, 64), (1, 17, 5, 64), (2, 784, 49, 128),
                                      (3, 1000, 64, 128), (1, 9, 3, 128)])
def test_attn_block_vs_unfused(cuda, dt, B, N, Nk, C):
    """The fused attention half of a Block (q GEMM -> attention -> proj + residual -> LayerNorm; stage 1 C = 64
    one head, stage 2 C = 128 two heads) == the unfused kernel chain with the same roundings (within two
    storage ulps), and == fp64 torch."""
    from svk import ops
    heads = C // 64
    hn = _rand(B, N, C, dt=dt, dev=cuda, seed=40)
    x = _rand(B, N, C, dt=dt, dev=cuda, seed=41)
    kv = _rand(B, Nk, 2 * C, dt=dt, dev=cuda, seed=42)
    wq = _rand(C, C, dt=dt, dev=cuda, scale=C ** -0.5, seed=43)
    wp = _rand(C, C, dt=dt, dev=cuda, scale=C ** -0.5, seed=44)
    bq = _rand(C, dt=torch.float32, dev=cuda, scale=0.1, seed=45)
    bp = _rand(C, dt=torch.float32, dev=cuda, scale=0.1, seed=46)
    g2 = _rand(C, dt=torch.float32, dev=cuda, seed=47)
    b2 = _rand(C, dt=torch.float32, dev=cuda, seed=48)
    scale = 64 ** -0.5
    y, h2 = ops.attn_block(hn, x, kv, wq, bq, wp, bp, g2, b2, 1e-6, scale)
    q = ops.gemm(hn, wq, bq)
    o = ops.attention(q, kv[:, :, :C], kv[:, :, C:], heads, scale)
    yu = ops.gemm(o, wp, bp, residual=x)
    h2u = ops.layernorm(yu, g2, b2, 1e-6)
    torch.cuda.synchronize()
    ulp = 2.0 ** -10 if dt == torch.float16 else 2.0 ** -7
    for got, ref in ((y, yu), (h2, h2u)):
        d = (got.float() - ref.float()).abs() / ref.float().abs().clamp_min(1.0)
        assert float(d.max()) <= 2 * ulp, float(d.max())
    # fp64 reference of the same math on the same (rounded) inputs
    f = lambda t: t.cpu().double()
    sh = lambda t: t.reshape(B, t.shape[1], heads, 64).transpose(1, 2)
    qd = f(hn) @ f(wq).t() + f(bq)
    att = ((sh(qd) @ sh(f(kv[:, :, :C])).transpose(-1, -2)) * scale).softmax(-1) @ sh(f(kv[:, :, C:]))
    yd = f(x) + att.transpose(1, 2).reshape(B, N, C) @ f(wp).t() + f(bp)
    _close(y, yd, dt)


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,C", [(2 * 3136, 64), (1000, 64), (17, 64), (2 * 784, 128), (33, 128), (3 * 196, 320),
                                 (21, 320)])
def test_prompt_ln_vs_unfused(cuda, dt, M, C):
    """Prompt adapter + norm1 in one kernel == the unfused chain (lightweight GEMM + GELU, shared GEMM +
    residual, LayerNorm) within two storage ulps."""
    from svk import ops
    C4 = C // 4
    x = _rand(M, C, dt=dt, dev=cuda, seed=50)
    sm = _rand(M, C4, dt=dt, dev=cuda, seed=51)
    wl = _rand(C4, C4, dt=dt, dev=cuda, scale=C4 ** -0.5, seed=52)
    ws = _rand(C, C4, dt=dt, dev=cuda, scale=C4 ** -0.5, seed=53)
    bl = _rand(C4, dt=torch.float32, dev=cuda, scale=0.1, seed=54)
    bs = _rand(C, dt=torch.float32, dev=cuda, scale=0.1, seed=55)
    g1 = _rand(C, dt=torch.float32, dev=cuda, seed=56)
    b1 = _rand(C, dt=torch.float32, dev=cuda, seed=57)
    xo, h = ops.prompt_ln(x, sm, wl, bl, ws, bs, g1, b1, 1e-6)
    f = ops.gemm(sm, wl, bl, act="gelu")
    xu = ops.gemm(f, ws, bs, residual=x)
    hu = ops.layernorm(xu, g1, b1, 1e-6)
    torch.cuda.synchronize()
    ulp = 2.0 ** -10 if dt == torch.float16 else 2.0 ** -7
    for got, ref in ((xo, xu), (h, hu)):
        d = (got.float() - ref.float()).abs() / ref.float().abs().clamp_min(1.0)
        assert float(d.max()) <= 2 * ulp, float(d.max())
    # independent fp64 reference (get_prompt + Block.norm1, mix_transformer_evp.py:776-815, 167-169) on the
    # same storage-rounded inputs; the kernel rounds the lightweight GEMM's GELU output to the storage
    # type (as the unfused GEMM does) and normalises the rounded x'
    d64 = lambda t: t.double().cpu()
    f64 = torch.nn.functional.gelu(d64(sm) @ d64(wl).t() + d64(bl)).to(dt).double()
    x64 = d64(x) + f64 @ d64(ws).t() + d64(bs)
    xr = d64(xo)
    mu = xr.mean(1, keepdim=True)
    h64 = (xr - mu) / torch.sqrt(((xr - mu) ** 2).mean(1, keepdim=True) + 1e-6) * d64(g1) + d64(b1)
    for got, ref in ((xo, x64), (h, h64)):
        d = (d64(got) - ref).abs() / ref.abs().clamp_min(1.0)
        assert float(d.max()) <= 2 * ulp, ("fp64", float(d.max()))


@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("B,C,H,W,Cout", [(2, 3, 224, 224, 64), (2, 2, 224, 224, 64), (3, 3, 224, 224, 16),
                                          (1, 3, 36, 20, 32), (2, 2, 12, 28, 8)])
def test_stem_conv_s2d(cuda, dt, B, C, H, W, Cout):
    """The k = 7 / stride-4 stem conv (OverlapPatchEmbed 1, flow conv1) over space-to-depth blocks == the
    8-channel NHWC implicit-GEMM conv it replaces and fp64 torch (same storage-rounded inputs and weights)."""
    from svk import ops
    from svk.pack import conv_w, conv_w_s2d
    x = torch.randn(B, C, H, W, generator=torch.Generator().manual_seed(61))
    w = torch.randn(Cout, C, 7, 7, generator=torch.Generator().manual_seed(62)) * 0.1
    b = torch.randn(Cout, generator=torch.Generator().manual_seed(63)) * 0.1
    xd, wd, bd = x.to(cuda), w.to(cuda), b.to(cuda)
    got = ops.conv2d_stem_s2d(xd, conv_w_s2d(wd, dt, 4), 7, 4, 3, bias=bd, act="relu")
    old = ops.conv2d_nhwc(ops.nchw_to_nhwc(xd, dt, cpad=8), conv_w(wd, dt, 8), 7, 4, 3, bias=bd, act="relu")
    torch.cuda.synchronize()
    assert got.shape == old.shape == (B, (H - 1) // 4 + 1, (W - 1) // 4 + 1, Cout)
    ref = F.relu(F.conv2d(x.to(dt).double(), w.to(dt).double(), b.double(), stride=4, padding=3)).permute(0, 2, 3, 1)
    _close(got, ref, dt)
    _close(got, old.double().cpu(), dt)


@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("C,H,W,extra", [(3, 224, 224, 0), (2, 224, 224, 0), (3, 36, 20, 1), (2, 12, 28, 3),
                                         (3, 8, 8, 4)])
def test_nchw_to_s2d_block_grid(cuda, dt, C, H, W, extra):
    """svk_nchw_to_s2d (pad 3, the float4 path for W % 4 == 0) == the zero-padded map rearranged into 4x4 blocks,
    bitwise, including block grids larger than the image needs (a k = 6 stem; ADVICE r03: the last block
    column's chunk address is clamped into the row, its values masked)."""
    from svk import ops
    B = 2
    nbh, nbw = (H - 1) // 4 + 2 + extra, (W - 1) // 4 + 2 + extra
    x = torch.randn(B, C, H, W, generator=torch.Generator().manual_seed(81)).to(cuda)
    got = ops.nchw_to_s2d(x, dt, 4, 3, nbh, nbw)
    pad = torch.zeros(B, C, 4 * nbh, 4 * nbw, device=cuda)
    hh, ww = min(H, 4 * nbh - 3), min(W, 4 * nbw - 3)
    pad[:, :, 3:3 + hh, 3:3 + ww] = x[:, :, :hh, :ww]
    ref = pad.view(B, C, nbh, 4, nbw, 4).permute(0, 2, 4, 3, 5, 1).reshape(B, nbh, nbw, 16 * C).to(dt)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("dt", H16)
@pytest.mark.parametrize("B,C,H,W", [(2, 3, 224, 224), (1, 3, 36, 20), (2, 2, 12, 28), (1, 1, 9, 13)])
def test_gauss5x5_s2d(cuda, dt, B, C, H, W):
    """GaussianFilter.conv_gauss written as the stem's space-to-depth blocks == svk_gauss5x5_reflect's NHWC map
    rearranged into blocks (bitwise: the same arithmetic per pixel), zeros outside the image."""
    from svk import ops
    x = torch.rand(B, C, H, W, generator=torch.Generator().manual_seed(71)).to(cuda)
    OH, OW = (H - 1) // 4 + 1, (W - 1) // 4 + 1
    got = ops.gauss5x5_s2d(x, dt, 3, OH + 1, OW + 1)
    ref8 = ops.gauss5x5_reflect(x, dt, cpad=8)[..., :3]                       # [B, H, W, 3]
    pad = torch.zeros(B, 4 * (OH + 1), 4 * (OW + 1), 3, device=cuda, dtype=dt)
    pad[:, 3:3 + H, 3:3 + W] = ref8
    ref = pad.view(B, OH + 1, 4, OW + 1, 4, 3).permute(0, 1, 3, 2, 4, 5).reshape(B, OH + 1, OW + 1, 48)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


def test_packed_and_stats_buffers_are_validated(cuda):
    """a dw_fc2 pack built for another (W, N, K) and a wrongly shaped colstats_set output are rejected
    on the host instead of being read / written out of bounds."""
    from svk import ops, _lib
    dt = torch.float16
    h = _rand(2, 14, 14, 1280, dt=dt, dev=cuda, seed=1)
    taps = _rand(9, 1280, dt=torch.float32, dev=cuda, scale=0.3, seed=2)
    db = _rand(1280, dt=torch.float32, dev=cuda, scale=0.1, seed=3)
    w2 = _rand(320, 1280, dt=dt, dev=cuda, scale=1280 ** -0.5, seed=4)
    b2 = _rand(320, dt=torch.float32, dev=cuda, seed=5)
    pk = ops.mixffn_dw_fc2_pack(taps, db, w2, 14)
    ops.mixffn_dw_fc2(h, taps, db, w2, b2, packed=pk)                     # the matching pack runs
    pk_short = ops.mixffn_dw_fc2_pack(taps[:, :640].contiguous(), db[:640].contiguous(), w2[:, :640].contiguous(), 14)
    with pytest.raises(_lib.SvkError, match="packed buffer"):
        ops.mixffn_dw_fc2(h, taps, db, w2, b2, packed=pk_short)          # built for K = 640
    x = _rand(300, 64, dt=dt, dev=cuda, seed=6)
    ops.colstats_set(x, out=torch.empty(2, 64, device=cuda))
    for bad in (torch.empty(2, 32, device=cuda), torch.empty(64, 2, device=cuda).t()):
        with pytest.raises(_lib.SvkError, match="colstats_set"):
            ops.colstats_set(x, out=bad)
