"""Observation data for the four model families.

* AR: ``data_gen`` restates AR_dat_gen.py:6-43 (same numpy legacy-RNG draws, same
  files), so ``python main.py hyperparameters.txt`` regenerates dat/AR_*.txt exactly
  as the reference does (checked bit-exactly against the reference's files in tests).
* LV: the reference ships dat/LV_* (2 x 500, obs every 100 steps, -1 elsewhere).
  ``lv_data_gen`` simulates the same SDE by Euler-Maruyama for the scaled configs
   and writes the same format.
* SV: dat/SV.dat (the model uses [300:], SV_dense.py:406).
* FHN: the reference's dat/fitz_nag_* files are missing (.MISSING_LARGE_BLOBS);
  ``fhn_data_gen`` simulates the FHN SDE.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np

REPO_DAT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dat")


def data_gen(T, impute, x0, theta, obs_std, dat_dir=None, write=True):
    """AR(1) simulation + partial observation files (AR_dat_gen.py:6-43).  ``write=False`` draws the
    same random numbers without writing (non-zero ranks of a multi-process run)."""
    dat_dir = os.getcwd() if dat_dir is None else dat_dir
    if write:
        os.makedirs(os.path.join(dat_dir, "dat"), exist_ok=True)
    theta = [float(t) for t in theta]
    n = int(np.int32(T + 1))
    X = np.zeros(n)
    X[0] = x0
    for i in range(1, n):
        X[i] = np.random.normal(X[i - 1] * theta[1] + theta[0], theta[2])
    obs = np.random.normal(loc=X, scale=obs_std)
    picks = obs[impute:][0::impute]
    obs_partial = np.concatenate([np.concatenate((np.zeros(impute - 1), [v])) for v in picks])
    obs_fill = np.concatenate([np.tile(v, impute) for v in picks])
    obs_binary = [0.0 if v == 0 else 1.0 for v in obs_partial]
    time_till = np.zeros(len(obs_binary))
    count = 1
    for i in range(len(obs_binary)):
        if obs_binary[i] == 1.0:
            count = 1
        else:
            time_till[i] = count
            count += 1
    time_till_out = -(time_till - impute)
    if not write:
        return obs_fill, np.asarray(obs_binary), time_till_out
    for name, arr in (("AR_obs_partial", obs_fill), ("AR_obs_binary", obs_binary), ("AR_time_till", time_till_out)):
        with open(os.path.join(dat_dir, "dat", name + ".txt"), "w+") as f:
            np.savetxt(f, arr)
    return obs_fill, np.asarray(obs_binary), time_till_out


def load_ar(dat_dir=None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """AR.py:366-374 (float32 loads)."""
    dat_dir = os.getcwd() if dat_dir is None else dat_dir
    rd = lambda n: np.loadtxt(os.path.join(dat_dir, "dat", n), np.float32)
    return rd("AR_obs_partial.txt"), rd("AR_obs_binary.txt"), rd("AR_time_till.txt")


def _time_till(obs_bin_row: np.ndarray, dt: float) -> np.ndarray:
    """Time to the next observation strictly after each index, as in dat/LV_time_till.txt."""
    T = obs_bin_row.shape[0]
    idx = np.where(obs_bin_row > 0)[0]
    out = np.zeros(T)
    gap = int(idx[1] - idx[0]) if len(idx) > 1 else T
    nxt = np.concatenate([idx, [idx[-1] + gap if len(idx) else T]])
    j = 0
    for i in range(T):
        while j < len(nxt) and nxt[j] <= i:
            j += 1
        out[i] = np.round((nxt[j] - i) * dt, 10)
    return out


def lv_data_gen(target_dims: int, dt: float = 0.1, x0=(100.0, 100.0), theta=(0.5, 0.0025, 0.3),
                obs_every: int = 100, obs_sd: float = 1.0, seed: int = 0, dat_dir: Optional[str] = None):
    """Euler-Maruyama LV path (the SDE of lotka_volterra_partial.py:244-261), observed with N(x, obs_sd)
    noise on both species every ``obs_every`` steps (at indices obs_every-1, 2*obs_every-1, ...), -1 elsewhere.
    Resimulates a step that would leave the positive orthant."""
    rng = np.random.default_rng(seed)
    th = np.asarray(theta, dtype=np.float64)
    x = np.asarray(x0, dtype=np.float64)
    path = np.zeros((2, target_dims))
    for t in range(target_dims):
        while True:
            x1, x2 = x
            a = np.array([th[0] * x1 - th[1] * x1 * x2, th[1] * x1 * x2 - th[2] * x2])
            A = th[0] * x1 + th[1] * x1 * x2
            Bv = th[1] * x1 * x2
            Cc = Bv + th[2] * x2
            cov = dt * np.array([[A, -Bv], [-Bv, Cc]])
            step = rng.multivariate_normal(dt * a, cov)
            nx = x + step
            if np.all(nx > 0):
                break
        x = nx
        path[:, t] = x
    obs = -np.ones((2, target_dims))
    obs_bin = np.zeros((2, target_dims))
    idx = np.arange(obs_every - 1, target_dims, obs_every)
    obs[:, idx] = path[:, idx] + rng.normal(0.0, obs_sd, size=(2, len(idx)))
    obs_bin[:, idx] = 1.0
    tt = np.stack([_time_till(obs_bin[0], dt), _time_till(obs_bin[1], dt)])
    if dat_dir is not None:
        os.makedirs(os.path.join(dat_dir, "dat"), exist_ok=True)
        np.savetxt(os.path.join(dat_dir, "dat", "LV_obs_partial.txt"), obs)
        np.savetxt(os.path.join(dat_dir, "dat", "LV_obs_binary.txt"), obs_bin)
        np.savetxt(os.path.join(dat_dir, "dat", "LV_time_till.txt"), tt)
    return obs.astype(np.float32), obs_bin.astype(np.float32), tt.astype(np.float32), path


def load_lv(dat_dir=None):
    """lotka_volterra_partial.py:481-491."""
    dat_dir = REPO_DAT if dat_dir is None else os.path.join(dat_dir, "dat")
    rd = lambda n: np.loadtxt(os.path.join(dat_dir, n), np.float32)
    return rd("LV_obs_partial.txt"), rd("LV_obs_binary.txt"), rd("LV_time_till.txt")


def load_sv(dat_dir=None):
    """SV_dense.py:406: the model uses SV.dat[300:]."""
    dat_dir = REPO_DAT if dat_dir is None else os.path.join(dat_dir, "dat")
    return np.loadtxt(os.path.join(dat_dir, "SV.dat"), np.float32)[300:]


def fhn_data_gen(target_dims: int, dt: float = 0.1, x0=(2.0, 3.0),
                 theta=(np.log(2.0), 1.0, 1.5, np.log(0.5), np.log(0.3)), obs_every: int = 10,
                 obs_sd: float = 0.1, seed: int = 0, dat_dir: Optional[str] = None):
    """Euler-Maruyama FHN path (fitz_nag_NVP.py:243-252 drift/diffusion, theta raw) observed on both
    coordinates every ``obs_every`` steps with N(x, obs_sd) noise; format as the LV files.  The
    observation scheme is an assumption: the reference's fitz_nag_* files are missing."""
    rng = np.random.default_rng(seed)
    th = np.asarray(theta, dtype=np.float64)
    x = np.asarray(x0, dtype=np.float64)
    path = np.zeros((2, target_dims))
    sd = np.sqrt(dt) * np.array([np.sqrt(np.exp(th[3])), np.sqrt(np.exp(th[4]))])
    for t in range(target_dims):
        x1, x2 = x
        a = np.array([np.exp(th[0]) * (x1 - x1 ** 3 - x2 + th[1]), th[2] * x1 - x2 + 1.4])
        x = x + dt * a + sd * rng.standard_normal(2)
        path[:, t] = x
    obs = -np.ones((2, target_dims))
    obs_bin = np.zeros((2, target_dims))
    idx = np.arange(obs_every - 1, target_dims, obs_every)
    obs[:, idx] = path[:, idx] + rng.normal(0.0, obs_sd, size=(2, len(idx)))
    obs_bin[:, idx] = 1.0
    tt = np.stack([_time_till(obs_bin[0], dt), _time_till(obs_bin[1], dt)])
    if dat_dir is not None:
        os.makedirs(os.path.join(dat_dir, "dat"), exist_ok=True)
        np.savetxt(os.path.join(dat_dir, "dat", "fitz_nag_obs_partial.txt"), obs)
        np.savetxt(os.path.join(dat_dir, "dat", "fitz_nag_obs_binary.txt"), obs_bin)
        np.savetxt(os.path.join(dat_dir, "dat", "fitz_nag_time_till.txt"), tt)
    return obs.astype(np.float32), obs_bin.astype(np.float32), tt.astype(np.float32), path
