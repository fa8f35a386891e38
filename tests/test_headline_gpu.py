"""Parity of the BENCHED configuration (bench.py's default workload: MiT-b2-EVP + optical-flow fusion,
B = 256 frames, return_features and logits) against the fp32 oracle on the same inputs.

Bars (north star: logits within 1e-3 at fp32, argmax labels bit-exact):
  * fp32 (the precision of the reference's generate_evp_LFB.py): features and both logit heads within
    1e-3 absolute, phase argmax identical for all 256 frames.
  * fp16 (the headline dtype; the precision of the reference's torch.autocast(float16) inference and
    validation passes, train_evp.py:637/760): f16 storage, f32 accumulation / statistics.  Features
    within FP16_FEAT_ATOL absolute, both logit heads within FP16_LOGIT_ATOL = 1e-3 (the north-star bar)
    and the phase argmax identical for all 256 frames (measured values are printed;
    profiles/r02/precision_b256.txt).
  * bf16 (extra key only): features within 5e-2, logits within 2e-2.
"""
import numpy as np
import pytest
import torch

from oracle import inputs as I, params as P, mit_evp as M, shapes as SH

pytestmark = pytest.mark.gpu

B = 256
VARIANT = "mit_b2_evp"
FP16_FEAT_ATOL = 5e-3        # measured 2.3e-3 (|features| <= 2.84)
FP16_LOGIT_ATOL = 1e-3       # the north-star logit bar; measured 5.3e-4 (phase) / 8.2e-4 (anticipation)


def _head_logits(feat, sd):
    f = torch.nn.functional
    y = f.linear(f.relu(f.linear(feat, sd["head.fc.0.weight"], sd["head.fc.0.bias"])), sd["head.fc.2.weight"],
                 sd["head.fc.2.bias"])
    ya = f.linear(f.relu(f.linear(feat, sd["head.fc_ant.0.weight"], sd["head.fc_ant.0.bias"])),
                  sd["head.fc_ant.2.weight"], sd["head.fc_ant.2.bias"])
    return y, ya


@pytest.fixture(scope="module")
def b256():
    sd = P.make_state_dict(SH.mit_evp_shapes(VARIANT), 0)
    x, y, fl = I.frames(B, 21), I.segmaps(B, 21), I.flow(B, 21)
    with torch.no_grad():
        feat = M.forward(x, y, sd, VARIANT, fl, return_features=True)
        yl, ya = _head_logits(feat, sd)
    return sd, (x, y, fl), feat, yl, ya


def _run(cuda, b256, dtype):
    from models import mix_transformer_evp as mte
    sd, (x, y, fl), *_ = b256
    m = getattr(mte, VARIANT)()
    m.load_state_dict(sd)
    m.svk_dtype = dtype
    m = m.to(cuda).eval()
    with torch.no_grad():
        f = m(x.to(cuda), y.to(cuda), fl.to(cuda), return_features=True)
        gl, ga = m(x.to(cuda), y.to(cuda), fl.to(cuda))
    torch.cuda.synchronize()
    return f.float().cpu(), gl.float().cpu(), ga.float().cpu()


def _report(name, f, gl, ga, feat, yl, ya):
    agree = (gl.argmax(1) == yl.argmax(1)).float().mean().item()
    print(f"{name} B={B}: feat max|d| {(f - feat).abs().max():.3e} (|ref| max {feat.abs().max():.2f}), "
          f"logits max|d| {(gl - yl).abs().max():.3e}, ant max|d| {(ga - ya).abs().max():.3e}, "
          f"argmax agreement {agree:.4f}")
    return agree


def test_benched_config_fp32_b256(cuda, b256):
    _, _, feat, yl, ya = b256
    f, gl, ga = _run(cuda, b256, torch.float32)
    _report("fp32", f, gl, ga, feat, yl, ya)
    np.testing.assert_allclose(f.numpy(), feat.numpy(), rtol=0, atol=1e-3)
    np.testing.assert_allclose(gl.numpy(), yl.numpy(), rtol=0, atol=1e-3)
    np.testing.assert_allclose(ga.numpy(), ya.numpy(), rtol=0, atol=1e-3)
    assert torch.equal(gl.argmax(1), yl.argmax(1))                     # argmax labels bit-exact


def test_benched_config_fp16_b256(cuda, b256):
    _, _, feat, yl, ya = b256
    f, gl, ga = _run(cuda, b256, torch.float16)
    agree = _report("fp16", f, gl, ga, feat, yl, ya)
    assert torch.isfinite(f).all()
    np.testing.assert_allclose(f.numpy(), feat.numpy(), rtol=0, atol=FP16_FEAT_ATOL)
    np.testing.assert_allclose(gl.numpy(), yl.numpy(), rtol=0, atol=FP16_LOGIT_ATOL)
    np.testing.assert_allclose(ga.numpy(), ya.numpy(), rtol=0, atol=FP16_LOGIT_ATOL)
    assert agree == 1.0 and torch.equal(gl.argmax(1), yl.argmax(1))


def test_benched_config_bf16_b256(cuda, b256):
    _, _, feat, yl, ya = b256
    f, gl, ga = _run(cuda, b256, torch.bfloat16)
    _report("bf16", f, gl, ga, feat, yl, ya)
    np.testing.assert_allclose(f.numpy(), feat.numpy(), rtol=0, atol=5e-2)
    np.testing.assert_allclose(gl.numpy(), yl.numpy(), rtol=0, atol=2e-2)


@pytest.fixture(scope="module")
def b3_256():
    """mit_b3_evp — the model the reference's scripts build (train_evp.py:362, generate_evp_LFB.py:412) —
    at the benched B = 256, fp32 oracle features and logits."""
    sd = P.make_state_dict(SH.mit_evp_shapes("mit_b3_evp"), 3)
    x, y, fl = I.frames(B, 23), I.segmaps(B, 23), I.flow(B, 23)
    with torch.no_grad():
        feat = M.forward(x, y, sd, "mit_b3_evp", fl, return_features=True)
        yl, ya = _head_logits(feat, sd)
    return sd, (x, y, fl), feat, yl, ya


def test_mit_b3_fp16_b256_vs_oracle(cuda, b3_256):
    """mit_b3_evp (18 stage-3 blocks against b2's 6: the longest 16-bit accumulation chain the callers run)
    in fp16 at B = 256: both logit heads within the north-star 1e-3 of the fp32 oracle, phase argmax
    identical for all 256 frames, features within FP16_FEAT_ATOL."""
    from models import mix_transformer_evp as mte
    sd, (x, y, fl), feat, yl, ya = b3_256
    m = mte.mit_b3_evp()
    m.load_state_dict(sd)
    m.svk_dtype = torch.float16
    m = m.to(cuda).eval()
    with torch.no_grad():
        f = m(x.to(cuda), y.to(cuda), fl.to(cuda), return_features=True).float().cpu()
        gl, ga = (t.float().cpu() for t in m(x.to(cuda), y.to(cuda), fl.to(cuda)))
    agree = _report("mit_b3 fp16", f, gl, ga, feat, yl, ya)
    assert torch.isfinite(f).all()
    np.testing.assert_allclose(f.numpy(), feat.numpy(), rtol=0, atol=FP16_FEAT_ATOL)
    np.testing.assert_allclose(gl.numpy(), yl.numpy(), rtol=0, atol=FP16_LOGIT_ATOL)
    np.testing.assert_allclose(ga.numpy(), ya.numpy(), rtol=0, atol=FP16_LOGIT_ATOL)
    assert agree == 1.0 and torch.equal(gl.argmax(1), yl.argmax(1))


def test_fp16_features_vs_reference_golden(cuda, golden):
    """fp16 path against the vectors the reference itself produced (B = 2, with flow)."""
    from models import mix_transformer_evp as mte
    m = getattr(mte, VARIANT)()
    m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0))
    m.svk_dtype = torch.float16
    m = m.to(cuda).eval()
    with torch.no_grad():
        f = m(I.frames(2).to(cuda), I.segmaps(2).to(cuda), I.flow(2).to(cuda), return_features=True)
        y, _ = m(I.frames(2).to(cuda), I.segmaps(2).to(cuda), I.flow(2).to(cuda))
    torch.cuda.synchronize()
    np.testing.assert_allclose(f.float().cpu().numpy(), golden[f"{VARIANT}_feat_flow"], rtol=0, atol=FP16_FEAT_ATOL)
    np.testing.assert_allclose(y.float().cpu().numpy(), golden[f"{VARIANT}_logits_flow"], rtol=0, atol=FP16_LOGIT_ATOL)


def test_autocast_fp16_region_selects_f16(cuda):
    """Inside torch.autocast("cuda", float16) — the reference's inference/validation regions — the
    modules compute in f16 (svk.default_dtype)."""
    import svk
    with torch.autocast("cuda", dtype=torch.float16):
        assert svk.default_dtype() == torch.float16
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert svk.default_dtype() == torch.bfloat16
    assert svk.default_dtype() == torch.float32


def test_graphed_forward_matches_eager_and_recaptures(cuda):
    """svk.graphs.GraphedForward (bench.py's extraction step): graph replay == eager forward, new inputs
    through run(), and a parameter update or dtype switch triggers a re-capture."""
    from models import mix_transformer_evp as mte
    from svk.graphs import GraphedForward
    m = mte.mit_b0_evp()
    m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0))
    m.svk_dtype = torch.float16
    m = m.to(cuda).eval()
    x, y, fl = I.frames(4, 5).to(cuda), I.segmaps(4, 5).to(cuda), I.flow(4, 5).to(cuda)
    gf = GraphedForward(m, x.clone(), y.clone(), fl.clone())
    with torch.no_grad():
        ref = m(x, y, fl, return_features=True)
        torch.testing.assert_close(gf().clone(), ref, rtol=0, atol=0)
        x2, y2, f2 = I.frames(4, 6).to(cuda), I.segmaps(4, 6).to(cuda), I.flow(4, 6).to(cuda)
        torch.testing.assert_close(gf.run(x2, y2, f2).clone(), m(x2, y2, f2, return_features=True), rtol=0, atol=0)
        g0 = gf.graph
        m.head.linear_fuse.conv.weight.mul_(0.5)             # bumps the parameter version
        torch.testing.assert_close(gf.run(x, y, fl).clone(), m(x, y, fl, return_features=True), rtol=0, atol=0)
        assert gf.graph is not g0
        m.svk_dtype = torch.float32
        torch.testing.assert_close(gf().clone(), m(x, y, fl, return_features=True), rtol=0, atol=0)


def _config5_chain(cuda, b256, dtype):
    """MiT-b2 + flow features at ``dtype`` -> MultiStageModel_S(2, 8, 32, 2048, 14, causal) ->
    Transformer(32, 2048, 14, 30).original_forward on the 256-frame chunk (trans_SV_output.py:276-291),
    and the fp32 oracle chain on the same inputs."""
    from models import mstcn, adapter_transformer, mix_transformer_evp as mte
    from oracle import mstcn as MS, trans_sv as TS
    sd, (x, y, fl), feat, _, _ = b256
    tc = mstcn.MultiStageModel_S(2, 8, 32, 2048, 14, True)
    sd_tc = P.make_state_dict({k: v.shape for k, v in tc.state_dict().items()}, 1)
    tc.load_state_dict(sd_tc)
    tr = adapter_transformer.Transformer(32, 2048, 14, 30)
    sd_tr = P.make_state_dict({k: v.shape for k, v in tr.state_dict().items()}, 2)
    tr.load_state_dict(sd_tr)
    tc, tr = tc.to(cuda).eval(), tr.to(cuda).eval()
    m = getattr(mte, VARIANT)()
    m.load_state_dict(sd)
    m.svk_dtype = dtype
    m = m.to(cuda).eval()
    with torch.no_grad():
        lfb = m(x.to(cuda), y.to(cuda), fl.to(cuda), return_features=True)[None]      # [1, 256, 2048]
        out = tc(lfb.transpose(2, 1))[-1]                                             # [1, 14, 256]
        p_all = tr.original_forward(out, lfb)                                         # [256, 1, 14]
    torch.cuda.synchronize()
    with torch.no_grad():
        rf = feat[None]
        ro = MS.multi_stage_s(rf.transpose(2, 1), sd_tc, 2, 8, True)[-1]
        rp = TS.original_forward(ro, rf, sd_tr, 32)
    got = p_all.float().cpu()
    d_out = (out.float().cpu() - ro).abs().max().item()
    d = (got - rp).abs().max().item()
    agree = (got[:, 0, :7].argmax(-1) == rp[:, 0, :7].argmax(-1)).float().mean().item()
    print(f"config5 {str(dtype)[6:]} B={B}: MS-TCN logits max|d| {d_out:.3e}, chain logits max|d| {d:.3e} "
          f"(|ref| max {rp.abs().max():.2f}), phase argmax agreement {agree:.4f}")
    assert got.shape == (B, 1, 14)
    return got, rp, d, agree


def test_config5_end_to_end_fp32_b256(cuda, b256):
    """BASELINE config 5's chain on the 256-frame chunk at fp32 (trans_SV_output.py's precision): the
    north-star bar — per-frame logits within 1e-3 of the oracle chain, phase argmax identical."""
    got, rp, d, agree = _config5_chain(cuda, b256, torch.float32)
    np.testing.assert_allclose(got.numpy(), rp.numpy(), rtol=0, atol=1e-3)
    assert agree == 1.0


def test_config5_end_to_end_fp16_b256(cuda, b256):
    """BASELINE config 5 as specified (fp16 extraction, 256-frame chunk): the fp16 features (within
    FP16_FEAT_ATOL of fp32) pass through the MS-TCN's 2048 -> 32 input conv and 16 layers, which spreads
    their rounding to ~3.6e-3 on the MS-TCN logits and ~2.5e-3 on the chain's (measured); the bar is the
    phase argmax identical for all 256 frames and the chain logits within 5e-3 (fp16 features: the
    1e-3 logit bar holds at fp32, test above)."""
    got, rp, d, agree = _config5_chain(cuda, b256, torch.float16)
    assert agree == 1.0
    np.testing.assert_allclose(got.numpy(), rp.numpy(), rtol=0, atol=5e-3)
