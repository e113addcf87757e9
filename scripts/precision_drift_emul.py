"""Error model of the reduced-precision training modes over a trajectory (the tolerance source of
tests/test_gpu_posterior.py for bf16 / bf16x2f / bf16x2).

The GPU test runs K = 20 full training steps (grad of sum(-ELBO) -> clip -> Adamax, AR.py:226-234,
optimisers/adamax.py:42-58) of the AR-cfg shape and compares the q(theta) posterior and the per-sample ELBO after
every step with the float64 oracle's trajectory.  In a reduced-precision mode the two trajectories separate by the
mode's own roundings -- Adamax's normalised steps pass a gradient's rounding straight into the parameters -- so the
bar for such a mode is a property of the mode, computed here WITHOUT the GPU: the same K steps in float64 with every
flow product's operands rounded to bf16 exactly where the HIP kernels round them (oracle/precision_model.py:
forward / recompute activations and weights, the backward chain's weight and gradient operands, the weight-gradient
products' activation and gradient operands; split-weight modes keep the weight operand exact), against the exact
float64 trajectory from the same start, windows and draws as the GPU test.  Adamax turns a rounding into a
parameter step through the gradient's SIGN where a component is near zero, a discrete event: the plain emulation and
REALISATIONS - 1 scaled-domain realisations (oracle/precision_model.py REAL: the kernels round log2(e)-scaled values,
another draw of the same error distribution) give the envelope (max over realisations) per step.

Output: tests/golden/precision_drift.json, per mode and step: the emulated posterior mean / sd drift (max over
(theta0, theta1, e^theta2)) and the per-sample ELBO relative error.  The GPU test holds the kernels to
SAFETY x this envelope + the fp32 case's floor (a GPU run is one more realisation of the same rounding model).
usage: python scripts/precision_drift_emul.py [K] [REALISATIONS]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bridge  # noqa: E402
from oracle import nma_oracle as O  # noqa: E402
from tests.parity_util import build_model, oracle_inputs  # noqa: E402
from oracle.precision_model import MODES, emulate  # noqa: E402
N_POST = 4096


def _rebuild(params, leaves):
    it = iter(leaves)
    flows = [{k: next(it).detach() for k in sorted(P)} for P in params["flows"]]
    mafs = [[(next(it).detach(), next(it).detach(), m) for (w, b, m) in L] for L in params["mafs"]]
    return {"flows": flows, "mafs": mafs}


def _post_stats(theta):
    t = theta.double().clone()
    t[:, 2] = t[:, 2].exp()
    return t.mean(0).numpy(), t.std(0).numpy()


def run(K=20, p=20, M=5000, k=8, T=5000, realisations=4):
    """The GPU test's setup (tests/test_gpu_posterior.py TRAJ / test_ar_posterior_trajectory_matches_oracle)."""
    model = build_model("ar", p, M, k, 3, 50, 3, 10, "cpu", T=T, precision=0, impute=5, condition=True)
    md = model.mdef
    spec = bridge.spec_from_mdef(md, p)
    P0 = bridge.oracle_params(model.store.state_numpy(), spec, model.engine.theta_dist.masks_np)
    g = torch.Generator().manual_seed(17)
    xe = torch.randn(N_POST, md.P_theta, generator=g, dtype=torch.float64) * md.theta_base[1] + md.theta_base[0]
    np.random.seed(5)
    steps = []
    for _ in range(K):   # the windows and draws of every step, as the GPU test takes them
        starts = model.select_windows()
        eps = torch.randn(p, md.kernel_ext, generator=g, dtype=torch.float64)
        x0 = torch.randn(p, md.P_theta, generator=g, dtype=torch.float64) * md.theta_base[1] + md.theta_base[0]
        steps.append((starts, eps, x0, oracle_inputs(model, starts)))
    perms = model.engine.perms

    def post(ps):
        with torch.no_grad():
            th, _ = O.qtheta_sample_logprob(xe, md.theta_base[0], md.theta_base[1], O.build_bijectors(ps, perms), O.elu)
        return _post_stats(th)

    def trajectory(mode, seed=0):
        with emulate(mode, realisation=seed):
            P = P0
            S = [(torch.zeros_like(t), torch.zeros_like(t)) for t in O.param_leaves(P)]
            rec = []
            for starts, eps, x0, (ts, ex) in steps:
                new, S, info = O.train_step(spec, P, S, perms, x0, eps, ts, ex, 1e-3, clip=2.5e8)
                P = _rebuild(P, new)
                m, s = post(P)
                rec.append({"elbo": info["elbo"].double().numpy(), "mean": m, "sd": s})
                print(f"  {mode or 'exact'} step {len(rec) - 1}", flush=True)
            return rec

    exact = trajectory(None)
    out = {"K": K, "shape": {"p": p, "M": M, "k": k, "T": T}, "realisations": realisations, "modes": {},
           "per_realisation": {}}
    for mode in MODES:
        reals = []
        for seed in range(realisations):
            rec = trajectory(mode, seed)
            reals.append([{"dmean": float(np.abs(a["mean"] - b["mean"]).max()),
                           "dsd": float(np.abs(a["sd"] - b["sd"]).max()),
                           "elbo": float(np.max(np.abs(a["elbo"] - b["elbo"]) / np.abs(b["elbo"])))}
                          for a, b in zip(rec, exact)])
        out["per_realisation"][mode] = reals
        out["modes"][mode] = [{key: max(r[s][key] for r in reals) for key in ("dmean", "dsd", "elbo")}
                              for s in range(K)]
        print(mode, [(round(r["dmean"], 7), round(r["elbo"], 6)) for r in out["modes"][mode]], flush=True)
    return out


if __name__ == "__main__":
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "8")))
    res = run(K, realisations=R)
    path = os.path.join(ROOT, "tests", "golden", "precision_drift.json")
    json.dump(res, open(path, "w"), indent=1)
    print("wrote", path)
