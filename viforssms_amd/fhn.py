"""FitzHugh-Nagumo: VI_SSM with the reference signature (fitz_nag_NVP.py:159-448) and the
module-level driver as run().  The reference's data files are missing; run() simulates data
(viforssms_amd.data.fhn_data_gen)."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import _lib
from .features import fhn_table
from .nma import ModelDef, Batch
from .vi_ssm import VISSMBase, ThetaSpec, DistCtx

THETA_INIT = [float(np.log(2.0)), 1.0, 1.5, float(np.log(0.5)), float(np.log(0.3))]
# variables that train_paths=False freezes (trainable=train_bool in fitz_nag_NVP.py:78-96)
_PATH_VARS = ("conv/", "theta0/", "theta1/", "theta2/", "hidden", "head/")


def make_theta_spec(P_theta: int = 5) -> ThetaSpec:
    """fitz_nag_NVP.py:480-494: 4 x Invert(MAF[5,5,5], elu), 3 permutations, base N(0, 1)."""
    return ThetaSpec.build(P_theta, 4, 0.0, 1.0, "elu")


class VI_SSM(VISSMBase):
    def __init__(self, obs, obs_bin, time_till, x0, theta_dist: ThetaSpec, priors, dt, T, p, kernel_len, batch_dims,
                 network_dims, target_dims, no_flows, feat_window, learn_rate=1e-3, pre_train=True, train_paths=True,
                 *, device=None, seed: int = 1, precision: int = _lib.VISSM_PREC_FP32,
                 dist: Optional[DistCtx] = None, log_every: int = 1, init_seed: int = 1, grad_clip: float = 2.5e11):
        mdef = ModelDef(family="fhn", model_id=_lib.MODEL_FHN, D=2, M=int(batch_dims), k=int(kernel_len),
                        n_flows=int(no_flows), network_dims=list(network_dims), C_time=int(feat_window) + 3,
                        P_theta=len(priors), scale_num=float(target_dims), priors=list(priors), dt=float(dt),
                        clip=float(grad_clip), theta_pos=[True, False, False, True, True])
        table = fhn_table(np.asarray(obs), np.asarray(obs_bin), np.asarray(time_till), np.asarray(x0, dtype=np.float64),
                          float(T), float(dt), int(target_dims), int(no_flows), int(kernel_len), int(batch_dims),
                          int(feat_window))
        self.target_dims = int(target_dims)
        self.train_paths = train_paths
        self.pre_train_count = 0
        super().__init__(mdef, table, theta_dist, p, pre_train, 1e99, learn_rate, grad_clip, device=device,
                         seed=seed, precision=precision, dist=dist, log_every=log_every, init_seed=init_seed)
        self._frozen = None
        if not train_paths:
            mask = torch.ones_like(self.store.grad)
            for name, (a, n) in self.store.offsets.items():
                if name.startswith("flow") and any(v in name for v in _PATH_VARS):
                    mask[a:a + n] = 0.0
            self._frozen = mask

    def target_len(self) -> int:
        return self.target_dims

    def n_pretrain_opts(self) -> int:
        return 2

    def grad_mask(self):
        return self._frozen

    def pretrain_step(self, batch: Batch, run: int) -> bool:
        """t1 = minimize(lf_sample^2), t2 = minimize((theta - init)^2) each run until 500 consecutive steps
        have no infinite sde log-prob (fitz_nag_NVP.py:288-292, 372-386)."""
        out = self.forward(batch, self.global_step)
        x = self.engine.lf_sample(out["z"], batch)
        target = torch.tensor(THETA_INIT, dtype=torch.float32, device=x.device)
        finite = not bool(torch.isinf(out["sde"]).any().item())   # np.isinf only, as fitz_nag_NVP.py:378
        self.minimize_pair((x ** 2).sum(), ((out["theta"] - target) ** 2).sum())
        self.pre_train_count = self.pre_train_count + 1 if finite else 0
        return self.pre_train_count == 500


def run(argv=None):
    """Module-level driver of fitz_nag_NVP.py:451-523 (synthetic data: the reference files are missing)."""
    import argparse
    from .data import fhn_data_gen
    from .launch import init_distributed
    ap = argparse.ArgumentParser(description="FitzHugh-Nagumo NMA-VI (fitz_nag_NVP.py)")
    ap.add_argument("-p", type=int, default=50)
    ap.add_argument("--kernel-len", type=int, default=20)
    ap.add_argument("--dt", type=float, default=0.1)
    ap.add_argument("--T", type=float, default=100000.0)
    ap.add_argument("--batch-dims", type=int, default=50)
    ap.add_argument("--no-flows", type=int, default=3)
    ap.add_argument("--feat-window", type=int, default=10)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--no-pretrain", action="store_true")
    ap.add_argument("--train", action="store_true", help="train (the reference only samples paths and theta)")
    ap.add_argument("--save-paths", default=None)
    args = ap.parse_args(argv)
    np.random.seed(1)
    ctx = init_distributed()
    target_dims = int(np.int32(args.T / args.dt))
    obs, obs_bin, time_till, _ = fhn_data_gen(target_dims, dt=args.dt)
    priors = [(0.0, 10.0)] * 5
    theta = make_theta_spec()
    model = VI_SSM(obs, obs_bin, time_till, np.array([2.0, 3.0]), theta, priors, args.dt, args.T, args.p,
                   args.kernel_len, args.batch_dims, [50] * 5, target_dims, args.no_flows, args.feat_window,
                   learn_rate=1e-4, pre_train=not args.no_pretrain, dist=ctx)
    model.build_flow()
    if args.save_paths:
        model.save_paths(args.save_paths)
    if args.train:
        model.train(tensorboard_path="locally_variant/train/",
                    save_path="model_saves/fitz_nag_model_%i.ckpt" % args.batch_dims, max_runs=args.steps)
    return model
