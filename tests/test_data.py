"""Host data path: the AR generator vs the reference's own files and RNG replay (fixtures made by
importing the reference's AR_dat_gen.py, tests/golden/make_ref_fixtures.py), feature assembly vs
the oracle's independent restatement, and the LV/FHN/SV data formats."""
import os

import numpy as np
import pytest

from oracle import nma_oracle as O
from viforssms_amd import data, features

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = np.load(os.path.join(ROOT, "tests", "golden", "ref_rng_replay.npz"))


def _replay(impute):
    np.random.seed(1)
    np.random.seed(1)
    return data.data_gen(5000, impute, 10.0, np.array([5.0, 0.5, 3.0]), 1.0, write=False)


def test_data_gen_bit_exact_vs_reference_files(tmp_path):
    np.random.seed(1)
    np.random.seed(1)
    data.data_gen(5000, 1, 10.0, np.array([5.0, 0.5, 3.0]), 1.0, dat_dir=str(tmp_path))
    for n in ("AR_obs_partial", "AR_obs_binary", "AR_time_till"):
        mine = np.loadtxt(tmp_path / "dat" / (n + ".txt"))
        shipped = np.loadtxt(os.path.join(ROOT, "dat", n + ".txt"))
        assert np.array_equal(mine, shipped), n
        assert np.array_equal(mine, FIX[n]), n


def test_data_gen_impute5_matches_reference_replay():
    obs, ob, tt = _replay(5)
    assert np.array_equal(obs, FIX["AR_obs_partial_imp5"])
    assert np.array_equal(ob, FIX["AR_obs_binary_imp5"])
    assert np.array_equal(tt, FIX["AR_time_till_imp5"])
    # bin pattern 0,0,0,0,1 and time_till 4,3,2,1,5
    assert list(ob[:5]) == [0, 0, 0, 0, 1] and list(tt[:5]) == [4, 3, 2, 1, 5]


def test_numpy_rng_replay_matches_reference_main():
    """After data_gen, AR.main draws 4 permutations then np.random.choice per step (same calls here)."""
    _replay(1)
    from viforssms_amd.vi_ssm import ThetaSpec
    spec = ThetaSpec.build(3, 5, 1.5, 0.5)
    assert np.array_equal(np.array(spec.perms), FIX["perms"])
    for i in range(3):
        picks = np.random.choice(np.arange(0, 5000, 50), size=50, replace=False)
        assert np.array_equal(picks, FIX["picks"][i])


@pytest.mark.parametrize("k,n,M,fw,starts", [(50, 3, 50, 10, [0, 1400, 4950]), (8, 3, 5000, 10, [0]),
                                              (4, 2, 25, 3, [0, 25, 4975])])
def test_ar_features_match_oracle(k, n, M, fw, starts):
    obs, ob, tt = data.load_ar(ROOT)
    tab = features.ar_table(obs, ob, tt, 10.0, 5000, n, k, M, fw)
    ref = O.ar_time_feats(obs, ob, tt, n, k, M, fw, 5000, starts)
    got = tab.windows(starts)
    assert got.shape == (len(starts), n * k + M + 1, fw + 4)
    assert np.array_equal(got, ref)
    f = tab.feeds(starts)
    assert np.array_equal(f["obs"], ref[:, -M:, 0]) and np.array_equal(f["obs_bin"], ref[:, -M:, -1])


def test_ar_paper_shapes():
    """arrays 5151/5152, time_feats [50, 201, 14], flows 201 -> 151 -> 101 -> 51."""
    obs, ob, tt = data.load_ar(ROOT)
    tab = features.ar_table(obs, ob, tt, 10.0, 5000, 3, 50, 50, 10)
    assert len(tab.chans[0]) == 5151 and len(tab.chans[11]) == 5152
    assert tab.windows(np.zeros(50, dtype=int)).shape == (50, 201, 14)


def test_lv_reference_files_and_table():
    obs, ob, tt = data.load_lv()
    assert obs.shape == (2, 500)
    assert list(np.where(ob[0] > 0)[0]) == [99, 199, 299, 399, 499]
    tab = features.lv_table(obs, ob, tt, np.array([100.0, 100.0]), 50.0, 0.1, 500, 3, 20, 50, 10)
    w = tab.windows([0, 50])
    assert w.shape == (2, 3 * 20 + 2 * 50 + 2, 13)
    f = tab.feeds([0, 50])
    assert f["mask"].shape == (2, 2, 51) and f["mask"][0, :, 0].tolist() == [0, 0]
    assert f["shift"][0, :, 0].tolist() == [100.0, 100.0] and f["mask"][1, :, 0].tolist() == [1, 1]
    # obs_eval reshape: interleaved t-major
    flat = np.reshape(obs, -1, "F")
    assert np.allclose(f["obs"][1, :, 3], [flat[2 * (50 + 3)], flat[2 * (50 + 3) + 1]])


def test_lv_generator_format():
    obs, ob, tt, path = data.lv_data_gen(300, obs_every=100, seed=1)
    assert obs.shape == (2, 300) and np.all(path > 0)
    assert list(np.where(ob[0] > 0)[0]) == [99, 199, 299]
    assert np.all(obs[ob == 0] == -1)
    ref_tt = np.loadtxt(os.path.join(ROOT, "dat", "LV_time_till.txt"))
    assert np.allclose(tt[:, :300], ref_tt[:, :300])


def test_sv_table_shapes():
    obs = data.load_sv()
    assert obs.shape == (1509,)
    T = obs.shape[0] - 1
    tab = features.sv_table(obs, -8.5, T, 1.0, T, 5, 50, 52, 5)
    assert tab.kext == 5 * 50 + 52 + 1 and tab.C == 8
    w = tab.windows([0, 1456])
    assert w.shape == (2, 303, 8) and np.all(np.isfinite(w))
    f = tab.feeds([0, 52])
    assert f["dim_one"].shape == (2, 53) and np.allclose(f["dim_one"][1], obs[52:105])
