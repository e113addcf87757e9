"""AR(1) family: VI_SSM and main() with the reference signatures (AR.py:113-403)."""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

from . import _lib
from .data import load_ar
from .features import ar_table
from .nma import ModelDef, Batch
from .vi_ssm import VISSMBase, ThetaSpec, DistCtx


class VI_SSM(VISSMBase):
    """AR.py:113-362.  ``theta_dist`` is a ThetaSpec (the q(theta) flow architecture; its variables
    live in this model's flat parameter buffer)."""

    def __init__(self, obs, obs_std, x0, theta_dist: ThetaSpec, priors, T, p, kernel_len, batch_dims,
                 network_dims, no_flows, feat_window, obs_bin, time_till, pre_train=False, early_stopping=1e99,
                 learn_rate=1e-3, grad_clip=2.5e8, *, device=None, seed: int = 1,
                 precision: int = _lib.VISSM_PREC_FP32, dist: Optional[DistCtx] = None, log_every: int = 1,
                 init_seed: int = 1):
        T = int(np.int32(T))
        mdef = ModelDef(family="ar", model_id=_lib.MODEL_AR, D=1, M=int(batch_dims), k=int(kernel_len),
                        n_flows=int(no_flows), network_dims=list(network_dims), C_time=int(feat_window) + 4,
                        P_theta=len(priors), scale_num=float(T), priors=list(priors), obs_std=float(obs_std),
                        clip=float(grad_clip), theta_pos=[False, False, True])
        table = ar_table(np.asarray(obs), np.asarray(obs_bin), np.asarray(time_till), float(x0), T,
                         int(no_flows), int(kernel_len), int(batch_dims), int(feat_window))
        self.obs_std = obs_std
        self.kernel_len = int(kernel_len)
        self.no_flows = int(no_flows)
        self.network_dims = list(network_dims)
        self.kernel_ext = self.kernel_len * self.no_flows + int(batch_dims) + 1
        super().__init__(mdef, table, theta_dist, p, pre_train, early_stopping, learn_rate, grad_clip,
                         device=device, seed=seed, precision=precision, dist=dist, log_every=log_every,
                         init_seed=init_seed)

    def pretrain_step(self, batch: Batch, run: int) -> bool:
        """AR.py:201-202, 290-298: Adamax(1e-3, beta1=0.9).minimize(-obs_loss) for runs 0..500."""
        out = self.forward(batch, self.global_step)
        self.minimize((-out["obs"]).sum(), self._opt_pre[0], beta1=0.9, lr=1e-3)
        return run == 500


def build_theta_spec(priors) -> ThetaSpec:
    """AR.py:377-391: 5 x Invert(MAF[5,5,5], elu) with 4 np.random permutations; base N(1.5, 0.5)."""
    return ThetaSpec.build(len(priors), 5, 1.5, 0.5, "elu")


def main(p, kernel_len, T, batch_dims, network_dims, no_flows, priors, feat_window, x0, obs_std, learn_rate=1e-3,
         grad_clip=2.5e8, *, dat_dir: Optional[str] = None, max_runs: Optional[int] = None, device=None,
         precision: int = _lib.VISSM_PREC_FP32, dist: Optional[DistCtx] = None, seed: int = 1,
         pre_train: bool = True, log_every: int = 1, graph: bool = False):
    """AR.main (AR.py:364-403): load dat/AR_*, build q(theta), VI_SSM, train."""
    dat_dir = os.getcwd() if dat_dir is None else dat_dir
    obs, obs_bin, time_till = load_ar(dat_dir)
    theta_dist = build_theta_spec(priors)
    var_model = VI_SSM(obs, obs_std, x0, theta_dist, priors, T, p, kernel_len, batch_dims, network_dims, no_flows,
                       feat_window, obs_bin, time_till, pre_train=pre_train, learn_rate=learn_rate,
                       grad_clip=grad_clip, device=device, precision=precision, dist=dist, seed=seed,
                       log_every=log_every)
    var_model.build_flow()
    var_model.train(tensorboard_path=dat_dir + "/train/", save_path=dat_dir + "/model_saves/AR_save.ckpt",
                    max_runs=max_runs, graph=graph)
    return var_model
