"""The oracle (CPU restatement) against golden vectors produced by the reference itself
(tests/golden/gen_golden.py).  This is what pins the oracle; GPU tests then compare the HIP
path with the oracle and with the same goldens."""
import numpy as np
import pytest
import torch

from oracle import inputs as I, params as P, mit_evp as M, mstcn as MS, trans_sv as TS, shapes as SH

MSTCN_CFGS = {"mstcn_2_8_32_2048_c": (2, 8, 32, 2048, True),
              "mstcn_4_10_64_256_c": (4, 10, 64, 256, True),
              "mstcn_2_4_32_64_nc": (2, 4, 32, 64, False)}


def test_inputs_regenerate_identically(golden):
    assert np.allclose(I.digest(I.frames(2, 0)), golden["in_digest_frames"], rtol=0, atol=1e-6)
    assert np.allclose(I.digest(I.segmaps(2, 0)), golden["in_digest_segmaps"], rtol=0, atol=1e-6)
    assert np.allclose(I.digest(I.flow(2, 0)), golden["in_digest_flow"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("variant", ["mit_b0_evp", "mit_b2_evp", "mit_b3_evp"])
def test_state_dict_keys_match_reference(golden, variant):
    assert sorted(SH.mit_evp_shapes(variant)) == list(golden[f"{variant}_keys"])


@pytest.mark.parametrize("variant", ["mit_b0_evp", "mit_b2_evp", "mit_b3_evp"])
def test_mit_features_with_flow(golden, variant):
    sd = P.make_state_dict(SH.mit_evp_shapes(variant), 0)
    with torch.no_grad():
        f = M.forward(I.frames(2), I.segmaps(2), sd, variant, I.flow(2), return_features=True)
    np.testing.assert_allclose(f.numpy(), golden[f"{variant}_feat_flow"], rtol=0, atol=2e-5)


def test_mit_b2_no_flow_logits_and_intermediates(golden):
    v = "mit_b2_evp"
    sd = P.make_state_dict(SH.mit_evp_shapes(v), 0)
    x, y, fl = I.frames(2), I.segmaps(2), I.flow(2)
    with torch.no_grad():
        f = M.forward(x, y, sd, v, None, return_features=True)
        yl, ya = M.forward(x, y, sd, v, fl)
        outs = M.forward_features(x, y, sd, M.CONFIGS[v]["depths"])
        f3, f4 = M.flow_encoder(fl, sd)
        hcs = M.init_prompts(y.reshape(-1, 3, 224, 224), sd)
    np.testing.assert_allclose(f.numpy(), golden[f"{v}_feat_noflow"], rtol=0, atol=2e-5)
    np.testing.assert_allclose(yl.numpy(), golden[f"{v}_logits_flow"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(ya.numpy(), golden[f"{v}_logits_ant_flow"], rtol=0, atol=1e-5)
    assert (yl.argmax(1).numpy() == golden[f"{v}_logits_flow"].argmax(1)).all()
    for i, (t, H, W) in enumerate(outs):
        nchw_sum = t.double().sum(dim=1).numpy()
        np.testing.assert_allclose(nchw_sum, golden[f"{v}_stage{i + 1}_sum"], rtol=1e-5, atol=1e-3)
    t4, H4, W4 = outs[3]
    np.testing.assert_allclose(t4.transpose(1, 2).reshape(2, -1, H4, W4).numpy(), golden[f"{v}_stage4"], atol=2e-5)
    np.testing.assert_allclose(f4.numpy(), golden[f"{v}_flow_s4"], atol=2e-5)
    np.testing.assert_allclose(hcs[3].numpy(), golden[f"{v}_hc4"], atol=2e-5)


@pytest.mark.parametrize("name", list(MSTCN_CFGS))
def test_mstcn(golden, name):
    S, L, Fm, D, causal = MSTCN_CFGS[name]
    sh = SH.mstcn_shapes(S, L, Fm, D, 14)
    assert sorted(sh) == list(golden[name + "_keys"])
    sd = P.make_state_dict(sh, 1)
    out = MS.multi_stage_s(I.lfb(300, D, 7).transpose(2, 1), sd, S, L, causal)
    np.testing.assert_allclose(out.numpy(), golden[name], rtol=1e-6, atol=1e-5)


def test_transformer_window_and_fc(golden):
    xg = torch.from_numpy(golden["trans_window_x"])
    np.testing.assert_array_equal(TS.window_unfold(xg, 30).numpy(), golden["trans_window_enc"])
    sd = P.make_state_dict(SH.transformer_shapes(32, 2048, 14), 2)
    lf = I.lfb(xg.shape[-1], 2048, 9)
    feas = torch.tanh(torch.nn.functional.linear(lf, sd["fc.weight"]).transpose(0, 1))
    np.testing.assert_allclose(feas.numpy(), golden["trans_window_dec"], atol=1e-6)
    assert "('d_k', 32)" in golden["trans_ctor"][0] and "('len_q', 30)" in golden["trans_ctor"][0]


def test_vs_attn_known_answer_shapes():
    """vs_attn.py:117-146: MiT-b3 @224 attention maps are (1,h,N,49) with N = 3136/784/196/49."""
    Ns = [(224 // 4) ** 2 // (4 ** s) for s in range(4)]
    assert Ns == [3136, 784, 196, 49]
    for s, sr in enumerate(M.SR_RATIOS):
        side = 224 // (4 * 2 ** s)
        assert (side // sr) ** 2 == 49
