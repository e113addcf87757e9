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


def _plain_from_brute(mask, shift):
    """per window: one past the last element with mask != 1 or shift != 0 in any row, 0 when none"""
    out = []
    for m, s in zip(mask, shift):
        m, s = np.atleast_2d(m), np.atleast_2d(s)
        bad = np.where(((m != 1.0) | (s != 0.0)).any(0))[0]
        out.append(int(bad[-1]) + 1 if bad.size else 0)
    return out


def test_plain_from_table():
    """features.plain_from_table (VissmElboData.plain_from) == the per-window definition over the FeatureTable's own
    mask / shift feeds: the reference tables (only window 0 pins x_0) and tables with dirty entries anywhere."""
    obs, ob, tt = data.load_lv()
    tab = features.lv_table(obs, ob, tt, np.array([100.0, 100.0]), 50.0, 0.1, 500, 3, 20, 50, 10)
    starts = np.arange(0, 451)
    f = tab.feeds(starts)
    pf = features.plain_from_table(tab.extra["mask_vals"], tab.extra["shift_vals"], tab.M)
    assert pf.dtype == np.int32 and pf.shape == (451,)
    assert pf.tolist() == _plain_from_brute(f["mask"], f["shift"])
    assert pf[0] == 1 and not pf[1:].any()
    rng = np.random.default_rng(3)
    for D in (1, 2):
        for trial in range(20):
            L, M = int(rng.integers(2, 60)), int(rng.integers(0, 20))
            M = min(M, L - 1)
            mv = np.ones((D, L))
            sv = np.zeros((D, L))
            for _ in range(int(rng.integers(0, 4))):
                mv[int(rng.integers(0, D)), int(rng.integers(0, L))] = rng.choice([0.0, 0.5])
                sv[int(rng.integers(0, D)), int(rng.integers(0, L))] = rng.choice([0.0, 3.0])
            pf = features.plain_from_table(mv if D == 2 else mv[0], sv if D == 2 else sv[0], M)
            wins = [(mv[:, s:s + M + 1], sv[:, s:s + M + 1]) for s in range(L - M)]
            assert pf.tolist() == _plain_from_brute([w[0] for w in wins], [w[1] for w in wins])


def test_obs_list_table():
    """features.obs_list_table (VissmElboData.obs_list) == the per-window definition over the FeatureTable's own
    obs_bin feeds: the elements e in [1, M] whose observation row e - 1 is nonzero in either coordinate, ascending,
    -1 padded -- on the reference's LV files (every 100th step observed) and on random sparse masks."""
    obs, ob, tt = data.load_lv()
    tab = features.lv_table(obs, ob, tt, np.array([100.0, 100.0]), 50.0, 0.1, 500, 3, 20, 50, 10)
    starts = np.arange(0, 451)
    f = tab.feeds(starts)
    ol = features.obs_list_table(tab.extra["obs_bin"], tab.M)
    assert ol.dtype == np.int32 and ol.shape[0] == 451
    for s in (0, 49, 50, 51, 99, 450):
        want = (np.flatnonzero((f["obs_bin"][s] != 0).any(0)) + 1).tolist()
        got = [int(e) for e in ol[s] if e >= 0]
        assert got == want and all(e == -1 for e in ol[s][len(got):]), s
    assert ol.shape[1] == max(len([e for e in r if e >= 0]) for r in ol)
    rng = np.random.default_rng(5)
    for trial in range(20):
        L, M = int(rng.integers(2, 80)), int(rng.integers(1, 30))
        M = min(M, L)
        b = (rng.random((2, L)) < rng.choice([0.0, 0.05, 0.5])).astype(np.float64)
        ol = features.obs_list_table(b, M)
        assert ol.shape[0] == L - M + 1
        for s in range(L - M + 1):
            want = (np.flatnonzero((b[:, s:s + M] != 0).any(0)) + 1).tolist()
            assert [int(e) for e in ol[s] if e >= 0] == want


# --- LV / FHN / SV host feeds against the oracle's independent restatement (bit-exact) ---------
@pytest.mark.parametrize("family", ["lv", "fhn"])
@pytest.mark.parametrize("n,k,M,fw,starts", [(3, 20, 50, 10, [0, 50, 450, 50]), (2, 4, 24, 3, [0, 24, 48, 456]),
                                              (3, 20, 500, 10, [0])])
def test_pair_tables_match_oracle_on_reference_files(family, n, k, M, fw, starts):
    """dat/LV_* through features.lv_table / fhn_table == oracle.pair_time_feats
    (lotka_volterra_partial.py:185-204, 366-386; fitz_nag_NVP.py:182-202, 346-366)."""
    obs, ob, tt = data.load_lv()
    x0 = np.array([100.0, 100.0]) if family == "lv" else np.array([2.0, 3.0])
    mk = features.lv_table if family == "lv" else features.fhn_table
    tab = mk(obs, ob, tt, x0, 50.0, 0.1, 500, n, k, M, fw)
    ref = O.pair_time_feats(family, obs, ob, tt, x0, 0.1, 50.0, 500, n, k, M, fw, starts)
    assert np.array_equal(tab.windows(starts), ref["time_feats"])
    f = tab.feeds(starts)
    assert np.array_equal(f["obs_bin"], ref["bin"])
    if family == "lv":
        assert np.array_equal(f["mask"], ref["mask"]) and np.array_equal(f["shift"], ref["shift"])


@pytest.mark.parametrize("family,T,k,starts", [("lv", 5000, 20, [0]), ("fhn", 2000, 20, [0]),
                                               ("lv", 1000, 20, [0, 500, 500])])
def test_pair_tables_match_oracle_at_config_lengths(family, T, k, starts):
    """The BASELINE configs' lengths (LV T = 5000, FHN T = 2000) on simulated series."""
    gen = data.lv_data_gen if family == "lv" else data.fhn_data_gen
    obs, ob, tt, _ = gen(T, dt=0.1, obs_every=100 if family == "lv" else 10, seed=1)
    x0 = np.array([100.0, 100.0]) if family == "lv" else np.array([2.0, 3.0])
    M = T // max(1, len(set(starts)))
    mk = features.lv_table if family == "lv" else features.fhn_table
    tab = mk(obs, ob, tt, x0, T * 0.1, 0.1, T, 3, k, M, 10)
    ref = O.pair_time_feats(family, obs, ob, tt, x0, 0.1, T * 0.1, T, 3, k, M, 10, starts)
    assert np.array_equal(tab.windows(starts), ref["time_feats"])
    f = tab.feeds(starts)
    assert np.array_equal(f["obs_bin"], ref["bin"])
    if family == "lv":
        assert np.array_equal(f["mask"], ref["mask"]) and np.array_equal(f["shift"], ref["shift"])


@pytest.mark.parametrize("n,k,M,fw,starts", [(5, 50, 52, 5, [0, 52, 1456, 52]), (5, 50, 1508, 5, [0]),
                                              (2, 6, 24, 3, [0, 24, 1200])])
def test_sv_table_matches_oracle(n, k, M, fw, starts):
    """dat/SV.dat[300:] through features.sv_table == oracle.sv_time_feats (SV_dense.py:159-185, 304-328)."""
    obs = data.load_sv()
    T = obs.shape[0] - 1
    tab = features.sv_table(obs, -8.5, T, 1.0, T, n, k, M, fw)
    ref = O.sv_time_feats(obs, -8.5, 1.0, T, T, n, k, M, fw, starts)
    assert np.array_equal(tab.windows(starts), ref["time_feats"])
    f = tab.feeds(starts)
    for key in ("mask", "shift", "dim_one"):
        assert np.array_equal(f[key], ref[key]), key
