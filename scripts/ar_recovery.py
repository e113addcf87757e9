"""Statistical recovery of the AR(1) posterior on the reference's own data ("AR posterior
theta -> (5, 0.5, log 3) on dat/AR_*"): python main.py hyperparameters.txt's model (p 50 windows of M 50,
kernel_len 50, 3 flows, [50]*3, AR.py:364-403 via viforssms_amd.ar) trained with the reference schedule
(501 pre-training runs, then ELBO steps: Adamax lr 1e-3, beta1 0.95, clip 2.5e8) through the captured
step, printing the posterior mean / sd of (theta0, theta1, e^theta2) from 4096 q(theta) draws every
--every steps as JSON lines.  Used by tests/test_gpu_posterior.py and for the DESIGN.md record."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def posterior(model, n=4096, seed=0):
    import torch
    g = torch.Generator(device=model.engine.device).manual_seed(seed)
    md = model.mdef
    x0 = torch.randn(n, md.P_theta, generator=g, device=model.engine.device) * md.theta_base[1] + md.theta_base[0]
    with torch.no_grad():
        th, _ = model.engine.theta_dist.sample_and_log_prob(x0)
    th = th.double()
    th[:, 2] = th[:, 2].exp()
    return th.mean(0).cpu().numpy(), th.std(0).cpu().numpy()


def build(precision="fp32", seed=1):
    np.random.seed(1)
    from viforssms_amd import ar
    from viforssms_amd._lib import TRAIN_PRECISIONS
    from viforssms_amd.config import parseparams, to_hparams
    from viforssms_amd.data import load_ar
    hp = to_hparams(parseparams(os.path.join(ROOT, "hyperparameters.txt")))
    obs, ob, tt = load_ar(os.path.join(ROOT))
    spec = ar.build_theta_spec(hp.priors)
    model = ar.VI_SSM(obs, hp.obs_std, hp.x0, spec, hp.priors, hp.T, hp.p, hp.kernel_len, hp.batch_dims,
                      hp.network_dims, hp.no_flows, hp.feat_window, ob, tt, pre_train=True, learn_rate=hp.learn_rate,
                      grad_clip=hp.grad_clip, device="cuda:0", precision=TRAIN_PRECISIONS[precision], seed=seed,
                      log_every=10 ** 9)
    model.build_flow()
    return model


def diagnostics(model):
    """Optimiser and flow state behind a departure: the step's scalar summaries (ELBO terms, global norm), the
    Adamax step ratio |v| / m (1 = a variable moving at the full learning rate), each flow's head bias (mu, sigma
    pre-activation) and the largest |variable| per group."""
    import torch
    d = {k.split("/")[-1]: round(v, 4) for k, v in model.last.items()}
    o = model._opt_main
    r = (o.v.abs() / o.m.clamp_min(1e-30)).float()
    d["adamax_ratio_mean"] = round(float(r.mean()), 4)
    d["adamax_ratio_gt0.9"] = round(float((r > 0.9).float().mean()), 4)
    st = model.store
    for i in range(model.mdef.n_flows):
        d[f"flow{i}_head_b"] = [round(float(x), 4) for x in st[f"flow{i}/head/bias"].detach().cpu()]
    groups = {}
    for n in st.names():
        key = n.split("/")[0] + "/" + n.split("/")[1].rstrip("0123456789")
        groups[key] = max(groups.get(key, 0.0), float(st[n].detach().abs().max()))
    d["max_abs"] = {k: round(v, 3) for k, v in groups.items()}
    return d


def run(steps=20000, every=1000, precision="fp32", graph=True, out=None, seed=1, diag=False):
    model = build(precision, seed)
    t0 = time.time()
    model.train(None, None, max_runs=501, verbose=False, graph=False)   # pre-training (AR.py:290-298)
    assert not model.pre_train
    recs = []
    done = 0
    while done < steps:
        n = min(every, steps - done)
        model.train(None, None, max_runs=n, verbose=False, graph=graph)
        done += n
        m, s = posterior(model)
        rec = {"step": done, "mean": m.tolist(), "sd": s.tolist(), "elapsed_s": round(time.time() - t0, 1)}
        if diag:
            rec["diag"] = diagnostics(model)
        recs.append(rec)
        print(json.dumps(rec), flush=True)
        if out:
            with open(out, "a") as f:
                f.write(json.dumps(rec) + "\n")
    return model, recs


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--every", type=int, default=1000)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--seed", type=int, default=1, help="Philox seed of the eps / q(theta) base draws")
    ap.add_argument("--diag", action="store_true", help="optimiser / flow diagnostics per record")
    a = ap.parse_args()
    run(a.steps, a.every, a.precision, not a.no_graph, a.out, a.seed, a.diag)
