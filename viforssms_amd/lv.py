"""Lotka-Volterra partial observations: VI_SSM with the reference signature
(lotka_volterra_partial.py:162-462) and the module-level driver as run()."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import _lib
from .features import lv_table
from .nma import ModelDef, Batch
from .vi_ssm import VISSMBase, ThetaSpec, DistCtx

PRIORS = [(float(np.log(4.428 / 10)), 1e-4), (float(np.log(0.029 / 10)), 1e-4), (float(np.log(2.957 / 10)), 1e-4)]


def make_theta_spec(P_theta: int = 3) -> ThetaSpec:
    """lotka_volterra_partial.py:494-508: 4 x Invert(MAF[5,5,5], elu), 3 permutations, base N(0, 1)."""
    return ThetaSpec.build(P_theta, 4, 0.0, 1.0, "elu")


class VI_SSM(VISSMBase):
    def __init__(self, obs, obs_bin, time_till, x0, theta_dist: ThetaSpec, priors, dt, T, p, kernel_len, batch_dims,
                 network_dims, target_dims, no_flows, feat_window, learn_rate=1e-3, pre_train=True, *, device=None,
                 seed: int = 1, precision: int = _lib.VISSM_PREC_FP32, dist: Optional[DistCtx] = None,
                 log_every: int = 1, init_seed: int = 1, grad_clip: float = 1e9):
        mdef = ModelDef(family="lv", model_id=_lib.MODEL_LV, D=2, M=int(batch_dims), k=int(kernel_len),
                        n_flows=int(no_flows), network_dims=list(network_dims), C_time=int(feat_window) + 3,
                        P_theta=len(priors), scale_num=float(target_dims), priors=list(priors), dt=float(dt),
                        clip=float(grad_clip), theta_pos=[True, True, True])
        table = lv_table(np.asarray(obs), np.asarray(obs_bin), np.asarray(time_till), np.asarray(x0, dtype=np.float64),
                         float(T), float(dt), int(target_dims), int(no_flows), int(kernel_len), int(batch_dims),
                         int(feat_window))
        self.target_dims = int(target_dims)
        self.dt = float(dt)
        self.pre_train_count = 0
        super().__init__(mdef, table, theta_dist, p, pre_train, 1e99, learn_rate, grad_clip, device=device,
                         seed=seed, precision=precision, dist=dist, log_every=log_every, init_seed=init_seed)

    def target_len(self) -> int:
        return self.target_dims

    def pretrain_step(self, batch: Batch, run: int) -> bool:
        """t1 = Adamax(1e-3, 0.9).minimize((lf_sample - 75)^2) until 1000 consecutive steps have no infinite
        lf_log_prob (lotka_volterra_partial.py:301-302, 388-400: the reference counts np.isinf only, so a NaN
        does not reset the count)."""
        out = self.forward(batch, self.global_step)
        x = self.engine.lf_sample(out["z"], batch)
        finite = not bool(torch.isinf(out["logq"]).any().item())
        self.minimize(((x - 75.0) ** 2).sum(), self._opt_pre[0], beta1=0.9, lr=1e-3)
        self.pre_train_count = self.pre_train_count + 1 if finite else 0
        return self.pre_train_count == 1000


def run(argv=None):
    """Module-level driver of lotka_volterra_partial.py:466-530 (reference hyperparameters; overridable)."""
    import argparse
    from .data import load_lv, lv_data_gen
    from .launch import init_distributed
    ap = argparse.ArgumentParser(description="Lotka-Volterra NMA-VI (lotka_volterra_partial.py)")
    ap.add_argument("-p", type=int, default=50)
    ap.add_argument("--kernel-len", type=int, default=20)
    ap.add_argument("--dt", type=float, default=0.1)
    ap.add_argument("--T", type=float, default=50.0, help="time horizon (target_dims = T / dt)")
    ap.add_argument("--batch-dims", type=int, default=50)
    ap.add_argument("--no-flows", type=int, default=3)
    ap.add_argument("--feat-window", type=int, default=10)
    ap.add_argument("--synthetic", action="store_true", help="simulate data instead of dat/LV_*")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--no-pretrain", action="store_true")
    ap.add_argument("--save-paths", default=None)
    args = ap.parse_args(argv)
    np.random.seed(1)
    ctx = init_distributed()
    target_dims = int(np.int32(args.T / args.dt))
    if args.synthetic or target_dims != 500:
        obs, obs_bin, time_till, _ = lv_data_gen(target_dims, dt=args.dt)
    else:
        obs, obs_bin, time_till = load_lv()
    theta = make_theta_spec()
    model = VI_SSM(obs, obs_bin, time_till, np.array([100.0, 100.0]), theta, PRIORS, args.dt, args.T, args.p,
                   args.kernel_len, args.batch_dims, [50] * 5, target_dims, args.no_flows, args.feat_window,
                   learn_rate=1e-3, pre_train=not args.no_pretrain, dist=ctx)
    model.build_flow()
    if args.save_paths:
        model.save_paths(args.save_paths)
    model.train(tensorboard_path="locally_variant/train/", save_path="model_saves/LV_model_%i_3.ckpt" % args.batch_dims,
                max_runs=args.steps)
    return model
