"""LFB pickle format pinned against the reference's writer and reader recipes (no GPU needed).

Writer (generate_evp_LFB.py:295, 457, 502, 513-520): start from ``np.zeros(shape=(0, 2048))`` (float64),
``np.concatenate`` every batch's float32 ``[B, 2048]`` features onto it, ``np.array`` it and
``pickle.dump`` it with the default protocol.  Reader (tecno.py:64-91): ``pickle.load`` -> ``.shape`` ->
``get_long_feature`` picks rows start..start+T-1 -> ``torch.Tensor(np.array(long_feature))`` [1, T, 2048]
-> ``.transpose(2, 1)``.  ``svk.lfb.save_lfb`` must produce the same bytes, and the reader must see the
same arrays."""
import io
import pickle

import numpy as np
import torch

from svk.lfb import save_lfb


def _reference_writer(batches):
    g = np.zeros(shape=(0, 2048))                                   # generate_evp_LFB.py:295
    for f in batches:
        g = np.concatenate((g, f), axis=0)                          # :457
    g = np.array(g)                                                 # :502
    buf = io.BytesIO()
    pickle.dump(g, buf)                                             # :513-520
    return buf.getvalue()


def _tecno_reader(path, start, T):
    with open(path, "rb") as f:                                     # tecno.py:80-85
        lfb = pickle.load(f)
    long_feature = [[lfb[int(start + k)] for k in range(T)]]        # get_long_feature, tecno.py:64-76
    x = torch.Tensor(np.array(long_feature))                        # tecno.py:222
    return lfb, x.transpose(2, 1)                                   # tecno.py:223


def test_save_lfb_bytes_match_reference_recipe(tmp_path):
    r = np.random.default_rng(0)
    batches = [r.standard_normal((n, 2048)).astype(np.float32) for n in (200, 200, 57)]   # B = 200 batches
    bank = torch.from_numpy(np.concatenate(batches))
    pkl = tmp_path / "evp_LFB_test.pkl"
    save_lfb(bank, str(pkl), str(tmp_path / "evp_LFB_test.npy"))
    assert pkl.read_bytes() == _reference_writer(batches)
    lfb, x = _tecno_reader(str(pkl), 150, 300)
    assert lfb.shape == (457, 2048) and lfb.dtype == np.float64      # tecno.py:89 prints .shape
    assert x.shape == (1, 2048, 300) and x.dtype == torch.float32
    np.testing.assert_array_equal(x[0].t().numpy(), np.concatenate(batches)[150:450])
    side = np.load(tmp_path / "evp_LFB_test.npy")
    assert side.dtype == np.float32 and np.array_equal(side, np.concatenate(batches))


def test_empty_bank_matches_reference_recipe(tmp_path):
    pkl = tmp_path / "empty.pkl"
    save_lfb(torch.zeros(0, 2048), str(pkl))
    assert pkl.read_bytes() == _reference_writer([])
