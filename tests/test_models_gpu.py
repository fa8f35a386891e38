"""Model-level parity on the GPU: the build's drop-in modules (svk HIP kernels) against the golden
vectors produced by the reference and against the oracle.

North-star bar (BASELINE.json): per-frame phase logits within 1e-3 (fp32) and argmax labels
bit-exact.  f32 path: features/logits within 1e-3 absolute of the reference's goldens (observed
~1e-5).  bf16 path: features within 5e-2 absolute (|features| <= ~3), logits within 2e-2 —
stated here because bf16 is the throughput dtype, not the parity dtype.
"""
import numpy as np
import pytest
import torch

from oracle import inputs as I, params as P, mit_evp as M, mstcn as MS, trans_sv as TS, shapes as SH

pytestmark = pytest.mark.gpu


def _model(variant, dev, dtype):
    from models import mix_transformer_evp as mte
    m = getattr(mte, variant)()
    m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 0))
    m.svk_dtype = dtype
    return m.to(dev).eval()


@pytest.mark.parametrize("variant", ["mit_b0_evp", "mit_b2_evp", "mit_b3_evp"])
def test_features_fp32_vs_reference_golden(cuda, golden, variant):
    m = _model(variant, cuda, torch.float32)
    with torch.no_grad():
        f = m(I.frames(2).to(cuda), I.segmaps(2).to(cuda), I.flow(2).to(cuda), return_features=True)
    torch.cuda.synchronize()
    assert f.shape == (2, 2048) and f.dtype == torch.float32
    np.testing.assert_allclose(f.cpu().numpy(), golden[f"{variant}_feat_flow"], rtol=0, atol=1e-3)


@pytest.mark.parametrize("variant", ["mit_b1_evp", "mit_b4_evp", "mit_b5_evp"])
def test_features_fp32_vs_oracle_other_variants(cuda, variant):
    """The variants the reference defines but no golden pins (mix_transformer_evp.py:893-944): B = 2,
    fp32, features and logits against the oracle (pinned by the b0/b2/b3 goldens) within 1e-3."""
    m = _model(variant, cuda, torch.float32)
    x, y, fl = I.frames(2), I.segmaps(2), I.flow(2)
    with torch.no_grad():
        f = m(x.to(cuda), y.to(cuda), fl.to(cuda), return_features=True)
        yl, _ = m(x.to(cuda), y.to(cuda), fl.to(cuda))
    torch.cuda.synchronize()
    sd = P.make_state_dict(SH.mit_evp_shapes(variant), 0)
    with torch.no_grad():
        rf = M.forward(x, y, sd, variant, fl, return_features=True)
        ry, _ = M.forward(x, y, sd, variant, fl)
    assert f.shape == (2, 2048)
    np.testing.assert_allclose(f.cpu().numpy(), rf.numpy(), rtol=0, atol=1e-3)
    np.testing.assert_allclose(yl.cpu().numpy(), ry.numpy(), rtol=0, atol=1e-3)
    assert (yl.argmax(1).cpu() == ry.argmax(1)).all()


def test_b2_logits_fp32_argmax_exact(cuda, golden):
    m = _model("mit_b2_evp", cuda, torch.float32)
    with torch.no_grad():
        y, y_ant = m(I.frames(2).to(cuda), I.segmaps(2).to(cuda), I.flow(2).to(cuda))
        f_nf = m(I.frames(2).to(cuda), I.segmaps(2).to(cuda), None, return_features=True)
    torch.cuda.synchronize()
    ref = golden["mit_b2_evp_logits_flow"]
    np.testing.assert_allclose(y.cpu().numpy(), ref, rtol=0, atol=1e-3)
    np.testing.assert_allclose(y_ant.cpu().numpy(), golden["mit_b2_evp_logits_ant_flow"], rtol=0, atol=1e-3)
    assert (y.argmax(1).cpu().numpy() == ref.argmax(1)).all()
    np.testing.assert_allclose(f_nf.cpu().numpy(), golden["mit_b2_evp_feat_noflow"], rtol=0, atol=1e-3)


def test_b2_stage_outputs_and_prompts_fp32(cuda, golden):
    m = _model("mit_b2_evp", cuda, torch.float32)
    x, y, fl = I.frames(2).to(cuda), I.segmaps(2).to(cuda), I.flow(2).to(cuda)
    with torch.no_grad():
        outs = m.forward_features(x, y)
        f3, f4 = m.flow_encoder(fl)
        hc = m.prompt_generator.init_prompts(y.view(-1, 3, 224, 224))
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        np.testing.assert_allclose(o.double().sum(dim=(2, 3)).cpu().numpy(), golden[f"mit_b2_evp_stage{i + 1}_sum"],
                                   rtol=1e-4, atol=5e-2)
    np.testing.assert_allclose(outs[3].contiguous().cpu().numpy(), golden["mit_b2_evp_stage4"], atol=1e-3)
    np.testing.assert_allclose(f4.cpu().numpy(), golden["mit_b2_evp_flow_s4"], atol=1e-3)
    np.testing.assert_allclose(hc[3].cpu().numpy(), golden["mit_b2_evp_hc4"], atol=1e-3)


def test_b2_bf16_against_oracle_larger_batch(cuda):
    B = 8
    m = _model("mit_b2_evp", cuda, torch.bfloat16)
    x, y, fl = I.frames(B, 3), I.segmaps(B, 3), I.flow(B, 3)
    with torch.no_grad():
        f = m(x.to(cuda), y.to(cuda), fl.to(cuda), return_features=True)
        yl, ya = m(x.to(cuda), y.to(cuda), fl.to(cuda))
    torch.cuda.synchronize()
    sd = P.make_state_dict(SH.mit_evp_shapes("mit_b2_evp"), 0)
    with torch.no_grad():
        ref = M.forward(x, y, sd, "mit_b2_evp", fl, return_features=True)
        rl, ra = M.forward(x, y, sd, "mit_b2_evp", fl)
    np.testing.assert_allclose(f.cpu().numpy(), ref.numpy(), rtol=0, atol=5e-2)
    np.testing.assert_allclose(yl.cpu().numpy(), rl.numpy(), rtol=0, atol=2e-2)
    np.testing.assert_allclose(ya.cpu().numpy(), ra.numpy(), rtol=0, atol=2e-2)


def test_b2_fp32_batch_independence(cuda):
    """Frames are independent: a frame's features do not depend on its batch neighbours."""
    m = _model("mit_b2_evp", cuda, torch.float32)
    x, y, fl = I.frames(5, 4).to(cuda), I.segmaps(5, 4).to(cuda), I.flow(5, 4).to(cuda)
    with torch.no_grad():
        full = m(x, y, fl, return_features=True)
        part = m(x[2:4], y[2:4], fl[2:4], return_features=True)
    torch.cuda.synchronize()
    np.testing.assert_allclose(part.cpu().numpy(), full[2:4].cpu().numpy(), rtol=0, atol=1e-5)


MSTCN_CFGS = {"mstcn_2_8_32_2048_c": (2, 8, 32, 2048, True),
              "mstcn_4_10_64_256_c": (4, 10, 64, 256, True),
              "mstcn_2_4_32_64_nc": (2, 4, 32, 64, False)}


@pytest.mark.parametrize("name", list(MSTCN_CFGS))
def test_mstcn_vs_reference_golden(cuda, golden, name):
    from models import mstcn
    S, L, Fm, D, causal = MSTCN_CFGS[name]
    m = mstcn.MultiStageModel_S(S, L, Fm, D, 14, causal)
    m.load_state_dict(P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 1))
    m = m.to(cuda).eval()
    lfb = I.lfb(300, D, 7).to(cuda)
    with torch.no_grad():
        out = m(lfb.transpose(2, 1))                     # the caller's exact call (trans_SV_output.py:276-279)
    torch.cuda.synchronize()
    assert out.shape == (S, 1, 14, 300)
    np.testing.assert_allclose(out.cpu().numpy(), golden[name], rtol=1e-5, atol=1e-4)
    assert (out[-1].argmax(1).cpu().numpy() == golden[name][-1].argmax(1)).all()


def test_mstcn_full_length_video_vs_oracle(cuda):
    from models import mstcn
    m = mstcn.MultiStageModel_S(4, 10, 64, 256, 14, True)
    sd = P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 5)
    m.load_state_dict(sd)
    m = m.to(cuda).eval()
    lfb = I.lfb(5000, 256, 11)
    with torch.no_grad():
        out = m(lfb.to(cuda).transpose(2, 1))
    torch.cuda.synchronize()
    ref = MS.multi_stage_s(lfb.transpose(2, 1), sd, 4, 10, True)
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=1e-5, atol=2e-4)


@pytest.mark.parametrize("causal", [True, False])
def test_mstcn_ragged_videos_vs_per_video_and_oracle(cuda, causal):
    """forward_videos (one launch per layer for a ragged batch of videos) == the caller's per-video
    forward bit for bit, and == the oracle per video."""
    from models import mstcn
    m = mstcn.MultiStageModel_S(4, 10, 64, 256, 14, causal)
    sd = P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 5)
    m.load_state_dict(sd)
    m = m.to(cuda).eval()
    lens = [1000, 1, 37, 2048, 613]
    feats = torch.cat([I.lfb(T, 256, 20 + i)[0] for i, T in enumerate(lens)], 0)
    with torch.no_grad():
        out = m.forward_videos(feats.to(cuda), lens)
        per = [m(f[None].to(cuda).transpose(2, 1)) for f in torch.split(feats, lens)]
    torch.cuda.synchronize()
    assert out.shape == (4, sum(lens), 14)
    for T, got, one, f in zip(lens, m.split_videos(out, lens), per, torch.split(feats, lens)):
        assert got.shape == (4, 1, 14, T)
        torch.testing.assert_close(got, one, rtol=1e-6, atol=1e-6)
        if T <= 1000:
            ref = MS.multi_stage_s(f[None].transpose(2, 1), sd, 4, 10, causal)
            np.testing.assert_allclose(got.cpu().numpy(), ref.numpy(), rtol=1e-5, atol=2e-4)


@pytest.mark.parametrize("T", [1, 29, 30, 75, 1000])
def test_transformer_original_forward_vs_oracle(cuda, golden, T):
    from models import adapter_transformer
    m = adapter_transformer.Transformer(32, 2048, 14, 30)
    sd = P.make_state_dict({k: v.shape for k, v in m.state_dict().items()}, 2)
    m.load_state_dict(sd)
    m = m.to(cuda).eval()
    g = torch.Generator().manual_seed(T)
    x = torch.randn(1, 14, T, generator=g)
    lf = I.lfb(T, 2048, 9)
    with torch.no_grad():
        out = m.original_forward(x.to(cuda), lf.to(cuda))
        out2 = m.transformer(TS.window_unfold(x, 30).to(cuda),
                             torch.tanh(torch.nn.functional.linear(lf, sd["fc.weight"]).transpose(0, 1)).to(cuda))
    torch.cuda.synchronize()
    ref = TS.original_forward(x, lf, sd, 32)
    assert out.shape == (T, 1, 14)
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=0, atol=1e-4)
    np.testing.assert_allclose(out2.cpu().numpy(), ref.numpy(), rtol=0, atol=1e-4)


def test_lfb_extraction_and_pickle(cuda, tmp_path):
    """generate_evp_LFB-style extraction over a synthetic dataset: rows in index order, equal to a
    direct forward of the same frames; pickle is the reference's float64 (N, 2048) format."""
    import pickle
    from models.data_process import SyntheticCholecFlowDataset
    from svk.lfb import extract_lfb, save_lfb
    m = _model("mit_b0_evp", cuda, torch.float32)
    ds = SyntheticCholecFlowDataset(7, seed=3)
    bank = extract_lfb(m, ds, batch_size=3)
    torch.cuda.synchronize()
    x = torch.stack([ds[i][0] for i in range(7)]).to(cuda)
    y = torch.stack([ds[i][1] for i in range(7)]).to(cuda)
    fl = torch.stack([ds[i][2] for i in range(7)]).to(cuda)
    with torch.no_grad():
        ref = m(x[:, None], y[:, None], fl[:, None], return_features=True)
    np.testing.assert_allclose(bank.cpu().numpy(), ref.cpu().numpy(), rtol=0, atol=1e-5)
    p = tmp_path / "evp_LFB_test.pkl"
    save_lfb(bank, p, tmp_path / "evp_LFB_test.npy")
    with open(p, "rb") as f:
        arr = pickle.load(f)    # our own file
    assert arr.dtype == np.float64 and arr.shape == (7, 2048)
    np.testing.assert_allclose(arr, bank.cpu().numpy().astype(np.float64))


@pytest.mark.parametrize("workers", [0, 2])
def test_lfb_pipeline_decoded_equals_direct_forward(cuda, workers):
    """The pipelined extraction (svk.lfb: DataLoader workers -> pinned uint8 batches -> H2D on a copy stream
    -> GPU frame / flow transforms -> graph replay -> async D2H into the pinned bank) over decoded frames
    equals transforming all frames at once and running the eager forward (10 frames in batches of 4: a
    partial last batch; 250x250 frames as the reference's data_process.py:493-511 stubs)."""
    from models.data_process import SyntheticDecodedCholecFlow
    from svk.lfb import extract_lfb
    from svk.preproc import frame_transform, flow_transform
    m = _model("mit_b0_evp", cuda, torch.float16)
    ds = SyntheticDecodedCholecFlow(10, seed=4)
    bank = extract_lfb(m, ds, batch_size=4, num_workers=workers)
    assert bank.shape == (10, 2048) and bank.is_pinned()
    fr = torch.stack([torch.from_numpy(ds[i][0]) for i in range(10)]).to(cuda)
    sg = torch.stack([torch.from_numpy(ds[i][1]) for i in range(10)]).to(cuda)
    fl = torch.stack([torch.from_numpy(ds[i][2]) for i in range(10)]).to(cuda)
    with torch.no_grad():
        x, y, f = frame_transform(fr), frame_transform(sg), flow_transform(fl)
        # the same batch shapes as the pipeline (kernel choices depend on the batch), last one padded
        refs = []
        for a in range(0, 10, 4):
            idx = [min(i, 9) for i in range(a, a + 4)]
            o = m(x[idx][:, None], y[idx][:, None], f[idx][:, None], return_features=True).float()
            refs.append(o[:min(4, 10 - a)])
        ref = torch.cat(refs)
    torch.cuda.synchronize()
    np.testing.assert_allclose(bank.numpy(), ref.cpu().numpy(), rtol=0, atol=1e-6)


def test_end_to_end_chunk(cuda):
    """SegFormer(b2) -> MS-TCN(2,8,32,2048) -> Transformer(30) on one synthetic 64-frame clip, fp32,
    against the oracle chain (config 5 shape at reduced length)."""
    from models import mstcn, adapter_transformer
    T = 64
    m = _model("mit_b2_evp", cuda, torch.float32)
    tc = mstcn.MultiStageModel_S(2, 8, 32, 2048, 14, True)
    sd_tc = P.make_state_dict({k: v.shape for k, v in tc.state_dict().items()}, 1)
    tc.load_state_dict(sd_tc)
    tr = adapter_transformer.Transformer(32, 2048, 14, 30)
    sd_tr = P.make_state_dict({k: v.shape for k, v in tr.state_dict().items()}, 2)
    tr.load_state_dict(sd_tr)
    tc, tr = tc.to(cuda).eval(), tr.to(cuda).eval()
    x, y, fl = I.frames(T, 9), I.segmaps(T, 9), I.flow(T, 9)
    with torch.no_grad():
        feats = m(x.to(cuda), y.to(cuda), fl.to(cuda), return_features=True)
        lfb = feats[None]
        out = tc(lfb.transpose(2, 1))[-1]
        p_all = tr.original_forward(out, lfb)
    torch.cuda.synchronize()
    sd = P.make_state_dict(SH.mit_evp_shapes("mit_b2_evp"), 0)
    with torch.no_grad():
        rf = M.forward(x, y, sd, "mit_b2_evp", fl, return_features=True)[None]
        ro = MS.multi_stage_s(rf.transpose(2, 1), sd_tc, 2, 8, True)[-1]
        rp = TS.original_forward(ro, rf, sd_tr, 32)
    np.testing.assert_allclose(p_all.cpu().numpy(), rp.numpy(), rtol=0, atol=1e-3)
    assert (p_all[:, 0, :7].argmax(-1).cpu() == rp[:, 0, :7].argmax(-1)).all()
