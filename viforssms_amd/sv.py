"""Stochastic volatility: VI_SSM with the reference signature (SV_dense.py:139-401) and the
module-level driver as run()."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import _lib
from .features import sv_table
from .nma import ModelDef, Batch
from .vi_ssm import VISSMBase, ThetaSpec, DistCtx

PARAM_INIT = [0.001, -0.6, float(np.log(0.08)), float(np.log(0.5))]


def make_theta_spec(P_theta: int = 4) -> ThetaSpec:
    """SV_dense.py:428-442: 5 x Invert(MAF[5,5,5], relu), 4 permutations, base N(0, 1)."""
    return ThetaSpec.build(P_theta, 5, 0.0, 1.0, "relu")


class VI_SSM(VISSMBase):
    def __init__(self, obs, x0, theta_dist: ThetaSpec, priors, dt, T, p, kernel_len, batch_dims, network_dims,
                 target_dims, no_flows, feat_window, learn_rate=1e-3, pre_train=False, *, device=None, seed: int = 1,
                 precision: int = _lib.VISSM_PREC_FP32, dist: Optional[DistCtx] = None, log_every: int = 1,
                 init_seed: int = 1, grad_clip: float = 1e7):
        mdef = ModelDef(family="sv", model_id=_lib.MODEL_SV, D=1, M=int(batch_dims), k=int(kernel_len),
                        n_flows=int(no_flows), network_dims=list(network_dims), C_time=int(feat_window) + 3,
                        P_theta=len(priors), scale_num=float(target_dims), priors=list(priors), dt=float(dt),
                        clip=float(grad_clip), theta_pos=[False, False, True, True])
        table = sv_table(np.asarray(obs, dtype=np.float32), float(x0), float(T), float(dt), int(target_dims),
                         int(no_flows), int(kernel_len), int(batch_dims), int(feat_window))
        self.target_dims = int(target_dims)
        self.obs = np.asarray(obs)
        super().__init__(mdef, table, theta_dist, p, pre_train, 1e99, learn_rate, grad_clip, device=device,
                         seed=seed, precision=precision, dist=dist, log_every=log_every, init_seed=init_seed)

    def target_len(self) -> int:
        return self.target_dims

    def n_pretrain_opts(self) -> int:
        return 2

    def pretrain_step(self, batch: Batch, run: int) -> bool:
        """pre_train_step = minimize((lf_sample + 7)^2) and param_init = minimize((theta - init)^2), both each
        run, Adamax(1e-3, 0.9) with their own slots; 1000 runs (SV_dense.py:251-254, 330-339)."""
        out = self.forward(batch, self.global_step)
        x = self.engine.lf_sample(out["z"], batch)
        target = torch.tensor(PARAM_INIT, dtype=torch.float32, device=x.device)
        self.minimize_pair(((x + 7.0) ** 2).sum(), ((out["theta"] - target) ** 2).sum())
        return run == 1000


def run(argv=None):
    """Module-level driver of SV_dense.py:404-463."""
    import argparse
    from .data import load_sv
    from .launch import init_distributed
    ap = argparse.ArgumentParser(description="Stochastic volatility NMA-VI (SV_dense.py)")
    ap.add_argument("-p", type=int, default=200)
    ap.add_argument("--kernel-len", type=int, default=50)
    ap.add_argument("--batch-dims", type=int, default=52)
    ap.add_argument("--no-flows", type=int, default=5)
    ap.add_argument("--feat-window", type=int, default=5)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--no-pretrain", action="store_true")
    ap.add_argument("--save-paths", default=None)
    args = ap.parse_args(argv)
    np.random.seed(1)
    ctx = init_distributed()
    obs = load_sv()
    T = obs.shape[0] - 1
    dt = 1.0
    target_dims = int(np.int32(T / dt))
    priors = [(0.0, 10.0)] * 4
    theta = make_theta_spec()
    model = VI_SSM(obs, -8.5, theta, priors, dt, T, args.p, args.kernel_len, args.batch_dims, [50] * 5, target_dims,
                   args.no_flows, args.feat_window, learn_rate=1e-4, pre_train=not args.no_pretrain, dist=ctx)
    model.build_flow()
    if args.save_paths:
        model.save_paths(args.save_paths)
    model.train(tensorboard_path="locally_variant/train/", save_path="model_saves/SV_model_%i_v211.ckpt" % args.batch_dims,
                max_runs=args.steps)
    return model
