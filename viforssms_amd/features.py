"""Window / feature assembly (host side, numpy): the padded per-channel arrays each
reference VI_SSM.__init__ builds once, and the per-step window gather of its train loop.

A ``FeatureTable`` holds the padded channel arrays; ``windows(starts)`` returns the
``time_feats`` feed [n, kernel_ext, C] for window starts (in reference units:
``batch_select``), and ``feeds(starts)`` the per-window ELBO feeds.  Only the
distinct windows of a step are gathered; samples map to them through ``win``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import os

import numpy as np


@dataclass
class FeatureTable:
    family: str
    M: int
    kext: int
    chans: List[np.ndarray]           # padded channel arrays
    stride: int                        # 1 (AR/SV) or 2 (LV/FHN: starts are doubled)
    extra: Dict[str, np.ndarray] = field(default_factory=dict)

    @property
    def C(self) -> int:
        return len(self.chans)

    def windows(self, starts) -> np.ndarray:
        starts = np.asarray(starts, dtype=np.int64)
        out = np.empty((len(starts), self.kext, self.C), dtype=np.float64)
        for r, s in enumerate(starts):
            a = self.stride * int(s)
            for c, arr in enumerate(self.chans):
                out[r, :, c] = arr[a:a + self.kext]
        return out

    def feeds(self, starts, ts: Optional[np.ndarray] = None) -> Dict[str, np.ndarray]:
        """Per-window ELBO feeds (obs/obs_bin/mask/shift/dim_one) in the kernel layouts."""
        starts = np.asarray(starts, dtype=np.int64)
        ts = self.windows(starts) if ts is None else ts
        M = self.M
        n = len(starts)
        out: Dict[str, np.ndarray] = {}
        if self.family == "ar":                                   # AR.py:155, AR.py:170
            out["obs"] = ts[:, -M:, 0]
            out["obs_bin"] = ts[:, -M:, -1]
        elif self.family in ("lv", "fhn"):                        # lotka_volterra_partial.py:218-219, 385-386
            out["obs"] = ts[:, -2 * M:, 0].reshape(n, M, 2).transpose(0, 2, 1)
            ob = self.extra["obs_bin"]
            out["obs_bin"] = np.stack([ob[:, s:s + M] for s in starts])
            if self.family == "lv":                               # lotka_volterra_partial.py:381-384
                mv, sv = self.extra["mask_vals"], self.extra["shift_vals"]
                out["mask"] = np.stack([mv[:, s:s + M + 1] for s in starts])
                out["shift"] = np.stack([sv[:, s:s + M + 1] for s in starts])
        elif self.family == "sv":                                 # SV_dense.py:322-328
            mv, sv, obs = self.extra["mask_vals"], self.extra["shift_vals"], self.extra["obs"]
            out["mask"] = np.stack([mv[0, s:s + M + 1] for s in starts])
            out["shift"] = np.stack([sv[0, s:s + M + 1] for s in starts])
            out["dim_one"] = np.stack([obs[s:s + M + 1] for s in starts])
        return out


def ar_table(obs, obs_bin, time_till, x0, T, n_flows, k, M, fw) -> FeatureTable:
    """AR.py:132-150 (pad = n k + 1; channels [lags 0..fw-1, bin, time, time_till, obs_bin])."""
    pad = n_flows * k + 1
    T = int(np.int32(T))
    obs_pad = [np.concatenate((np.zeros(pad - i), obs, np.zeros(i))) for i in range(fw)]
    time_pad = np.concatenate((np.zeros(pad), np.arange(T + 1)))
    bin_feats = np.float32(np.concatenate((np.ones(pad), np.zeros(T))))
    obs_bin_p = np.concatenate((np.zeros(pad), obs_bin))
    tt = np.concatenate((np.arange(pad + time_till[0], time_till[0], -1), time_till))
    chans = obs_pad + [bin_feats.astype(np.float64), time_pad, tt, obs_bin_p]
    mask_vals = np.concatenate((np.zeros((1, 1)), np.ones((1, T))), axis=1)
    shift_vals = np.concatenate((np.array([[x0]]), np.zeros((1, T))), axis=1)
    return FeatureTable("ar", M, pad + M, chans, 1, {"mask_vals": mask_vals, "shift_vals": shift_vals})


def lv_table(obs, obs_bin, time_till, x0, T, dt, target_dims, n_flows, k, M, fw) -> FeatureTable:
    """lotka_volterra_partial.py:185-204 (interleaved 2-D; lags at stride 5;
    channels [lags, bin_feats (0s then 1s), time, time_till])."""
    flow_dims = 2
    pad = n_flows * k + flow_dims
    obs_flatten = np.reshape(obs, -1, "F")
    obs_pad = [np.concatenate((np.zeros(pad - i), obs_flatten, np.zeros(i))) for i in range(0, fw * 5, 5)]
    time_pad = np.concatenate((np.zeros(pad), np.repeat(np.arange(dt, T + dt, dt), flow_dims)))
    tt_pad = np.reshape(np.repeat(np.arange(np.round(pad * (dt / flow_dims), 1), 0.0, -dt), flow_dims),
                        (flow_dims, -1), "F")
    tt = np.reshape(np.concatenate((tt_pad, time_till), 1), -1, "F")
    bin_feats = np.float32(np.concatenate((np.zeros(pad), np.ones(target_dims * flow_dims))))
    mask_vals = np.concatenate((np.zeros((2, 1)), np.ones((flow_dims, target_dims))), axis=1)
    shift_vals = np.concatenate((np.expand_dims(np.asarray(x0, dtype=np.float64), 1),
                                 np.zeros((flow_dims, target_dims))), axis=1)
    chans = obs_pad + [bin_feats.astype(np.float64), time_pad, tt]
    kext = n_flows * k + flow_dims * M + 2
    return FeatureTable("lv", M, kext, chans, 2, {"obs_bin": np.asarray(obs_bin, dtype=np.float64),
                                                   "mask_vals": mask_vals, "shift_vals": shift_vals})


def fhn_table(obs, obs_bin, time_till, x0, T, dt, target_dims, n_flows, k, M, fw) -> FeatureTable:
    """fitz_nag_NVP.py:182-202 (as LV, but bin_feats is 1s then 0s and the time_till pad
    arange runs to -dt, one pair longer than the other channels' pad)."""
    flow_dims = 2
    pad = n_flows * k + flow_dims
    obs_flatten = np.reshape(obs, -1, "F")
    obs_pad = [np.concatenate((np.zeros(pad - i), obs_flatten, np.zeros(i))) for i in range(0, fw * 5, 5)]
    time_pad = np.concatenate((np.zeros(pad), np.repeat(np.arange(dt, T + dt, dt), flow_dims)))
    tt_pad = np.reshape(np.repeat(np.arange(np.round(pad * (dt / flow_dims), 1), -dt, -dt), flow_dims),
                        (flow_dims, -1), "F")
    tt = np.reshape(np.concatenate((tt_pad, time_till), 1), -1, "F")
    bin_feats = np.float32(np.concatenate((np.ones(pad), np.zeros(target_dims * flow_dims))))
    chans = obs_pad + [bin_feats.astype(np.float64), time_pad, tt]
    kext = n_flows * k + flow_dims * M + 2
    return FeatureTable("fhn", M, kext, chans, 2, {"obs_bin": np.asarray(obs_bin, dtype=np.float64)})


def sv_table(obs, x0, T, dt, target_dims, n_flows, k, M, fw) -> FeatureTable:
    """SV_dense.py:159-185: rolling variances of the series and of its differences (float32
    numpy, as the reference computes them on the float32 load), lags at stride 5, time."""
    var_store = [np.var(obs[i:i + k]) for i in range(0, obs.shape[0] - k)]
    var_pad = np.concatenate((np.zeros((n_flows + 1) * k), var_store), axis=0)
    obs_diff = obs[1:] - obs[:-1]
    var_diff_store = [np.var(obs_diff[i:i + k]) for i in range(0, obs_diff.shape[0] - k)]
    var_diff_pad = np.concatenate((np.zeros((n_flows + 1) * k), np.log(var_diff_store), np.zeros(1)), axis=0)
    obs_pad = [np.concatenate((np.zeros(n_flows * k - i), obs, np.zeros(i))) for i in range(0, fw * 5, 5)]
    time_pad = np.concatenate((np.zeros(n_flows * k + 1), np.arange(0.1, T + dt, dt)))
    mask_vals = np.concatenate((np.zeros((1, 1)), np.ones((1, target_dims))), axis=1)
    shift_vals = np.concatenate((np.array([[x0]]), np.zeros((1, target_dims))), axis=1)
    chans = [np.asarray(c, dtype=np.float64) for c in obs_pad + [time_pad, var_pad, var_diff_pad]]
    kext = n_flows * k + M + 1
    return FeatureTable("sv", M, kext, chans, 1, {"mask_vals": mask_vals, "shift_vals": shift_vals,
                                                   "obs": np.asarray(obs, dtype=np.float64)})


def plain_from_table(mask_vals, shift_vals, M: int) -> np.ndarray:
    """VissmElboData.plain_from per window start s (int32): one past the last element of the window [s, s + M] whose
    mask is not 1 or shift not 0 in any row, 0 when there is none -- from that element on the one-pass ELBO kernel
    evaluates the transform without the mask / shift loads."""
    mv, sv = np.atleast_2d(mask_vals), np.atleast_2d(shift_vals)
    dirty = ((mv != 1.0) | (sv != 0.0)).any(0)
    last = np.maximum.accumulate(np.where(dirty, np.arange(dirty.size), -1))   # last dirty position <= q
    s = np.arange(max(dirty.size - M, 1))
    ld = last[np.minimum(s + M, dirty.size - 1)]
    return np.where(ld >= s, ld - s + 1, 0).astype(np.int32)


def obs_list_table(obs_bin, M: int) -> np.ndarray:
    """VissmElboData.obs_list per window start s (int32 [n_starts, stride]): the elements e in [1, M] of the window
    [s, s + M] whose observation row e - 1 (obs_bin[:, s + e - 1]) is nonzero in either coordinate, ascending,
    padded with -1 -- the one-pass ELBO kernel evaluates the observation term there only (the reference's
    observations are sparse: every 100th LV step, lotka_volterra_partial.py:481-487)."""
    ob = np.atleast_2d(obs_bin)
    hit = (ob != 0).any(0)
    n = max(hit.size - M + 1, 1)
    rows = [np.flatnonzero(hit[s:s + M]) + 1 for s in range(n)]
    stride = max(1, max(len(r) for r in rows))
    out = np.full((n, stride), -1, dtype=np.int32)
    for s, r in enumerate(rows):
        out[s, :len(r)] = r
    return out


class DeviceTable:
    """The FeatureTable's padded channel arrays (and the per-window feed tables) resident on the GPU,
    built once per model; ``batch(uniq_dev, n)`` gathers time_feats and the ELBO feeds of n window
    starts with vissm_gather_windows -- the step's only upload is its int32 window starts."""

    def __init__(self, tab: FeatureTable, device):
        import torch
        self.tab = tab
        self.device = device
        f32 = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device=device)
        Lmax = max(len(c) for c in tab.chans)
        chans = np.zeros((tab.C, Lmax), dtype=np.float32)
        for c, arr in enumerate(tab.chans):
            chans[c, :len(arr)] = arr
        self.chans = f32(chans)
        self.pitch = Lmax
        ex = tab.extra
        self.extra = {}
        if tab.family in ("lv", "fhn"):
            self.extra["obs_bin"] = f32(ex["obs_bin"])
            self.obs_list = torch.as_tensor(obs_list_table(ex["obs_bin"], tab.M), device=device)
        if tab.family in ("lv", "sv"):
            self.extra["mask"] = f32(ex["mask_vals"])
            self.extra["shift"] = f32(ex["shift_vals"])
            pf = plain_from_table(ex["mask_vals"], ex["shift_vals"], tab.M)
            self.plain_from = torch.as_tensor(pf, device=device)
        if tab.family == "sv":
            self.extra["dim_one"] = f32(np.asarray(ex["obs"]).reshape(1, -1))

    def batch(self, uniq_dev, n: int):
        """(ts [n, kext, C], feeds dict) for the window starts uniq_dev (int32 [n] on the device)."""
        import torch
        from .ops import gather_windows
        t, M, K, C = self.tab, self.tab.M, self.tab.kext, self.tab.C
        dev = self.device
        ts = torch.empty(n, K, C, dtype=torch.float32, device=dev)
        gather_windows(self.chans, uniq_dev, ts, n, K, C, stride=t.stride, c_pitch=self.pitch, os=(K * C, C, 1))
        feeds = {}
        if t.family == "ar":                                      # AR.py:155, AR.py:170
            for key, ch in (("obs", 0), ("obs_bin", C - 1)):
                out = torch.empty(n, M, dtype=torch.float32, device=dev)
                gather_windows(self.chans[ch], uniq_dev, out, n, M, 1, offset=K - M, os=(M, 1, 0))
                feeds[key] = out
        elif t.family in ("lv", "fhn"):                           # lotka_volterra_partial.py:218-219, 385-386
            out = torch.empty(n, 2, M, dtype=torch.float32, device=dev)
            gather_windows(self.chans[0], uniq_dev, out, n, M, 2, stride=2, offset=K - 2 * M, j_step=2, c_pitch=1,
                           os=(2 * M, 1, M))
            feeds["obs"] = out
            ob = self.extra["obs_bin"]
            out = torch.empty(n, 2, M, dtype=torch.float32, device=dev)
            gather_windows(ob, uniq_dev, out, n, M, 2, c_pitch=ob.shape[1], os=(2 * M, 1, M))
            feeds["obs_bin"] = out
        if t.family in ("lv", "sv"):                              # lotka_volterra_partial.py:381-384, SV_dense.py:322-328
            D = 2 if t.family == "lv" else 1
            for key in ("mask", "shift"):
                tab = self.extra[key]
                out = torch.empty((n, D, M + 1) if D == 2 else (n, M + 1), dtype=torch.float32, device=dev)
                gather_windows(tab, uniq_dev, out, n, M + 1, D, c_pitch=tab.shape[1], os=(D * (M + 1), 1, M + 1))
                feeds[key] = out
        if t.family == "sv":
            out = torch.empty(n, M + 1, dtype=torch.float32, device=dev)
            gather_windows(self.extra["dim_one"], uniq_dev, out, n, M + 1, 1, os=(M + 1, 1, 0))
            feeds["dim_one"] = out
        if t.family in ("lv", "sv"):
            feeds["plain_from"] = self.plain_from[uniq_dev.long()]
        # the observation list is opt-in (VISSM_ELBO_OBS_LIST=1): its post-pass (a fence, then a read-modify-write of
        # dz at every listed element) measured slower than reading the obs rows at every element -- LV one-pass
        # 0.390 -> 0.397 ms, FHN 0.075 -> 0.127 ms (observations every 100th / 10th step; profiles/r06/ab_r06b.log)
        if t.family in ("lv", "fhn") and os.environ.get("VISSM_ELBO_OBS_LIST", "0") == "1":
            feeds["obs_list"] = self.obs_list[uniq_dev.long()].contiguous()
        return ts, feeds
