import os

import pytest

from viforssms_amd import config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_default_file():
    v = config.parseparams(os.path.join(ROOT, "hyperparameters.txt"))
    hp = config.to_hparams(v)
    assert hp.T == 5000 and hp.impute == 1 and hp.x0 == 10.0 and hp.theta == [5.0, 0.5, 3.0]
    assert hp.p == 50 and hp.kernel_len == 50 and hp.batch_dims == 50 and hp.network_dims == [50, 50, 50]
    assert hp.no_flows == 3 and hp.priors == [(0.0, 10.0)] * 3 and hp.feat_window == 10
    assert hp.learn_rate == 1e-3 and hp.grad_clip == 2.5e8


def test_repair_text_roundtrip(tmp_path):
    f = tmp_path / "h.txt"
    f.write_text(config.DEFAULT_FILE)
    assert config.parseparams(str(f)) == config.parseparams(os.path.join(ROOT, "hyperparameters.txt"))


def test_overrides_win():
    hp = config.to_hparams(config.parseparams(os.path.join(ROOT, "hyperparameters.txt")))
    args = config.handle_opts(["h.txt", "-T", "1000", "-i", "5", "-t", "1.0", "-t", "0.2", "-t", "2",
                               "-k", "8", "-b", "1000", "-p", "64", "-x", "3", "-o", "0.5", "-f", "4"])
    hp = config.apply_overrides(hp, args)
    assert (hp.T, hp.impute, hp.kernel_len, hp.batch_dims, hp.p, hp.x0, hp.obs_std, hp.feat_window) == \
        (1000, 5, 8, 1000, 64, 3.0, 0.5, 4)
    assert hp.theta == [1.0, 0.2, 2.0]


def test_bad_file_exits(tmp_path):
    import subprocess
    import sys
    bad = tmp_path / "bad.txt"
    bad.write_text("nonsense\n")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "main.py"), str(bad)], capture_output=True, text=True,
                       cwd=str(tmp_path))
    assert r.returncode != 0 and "valid hyperparameter file" in r.stderr
