"""The benchmark's own model (AR(1), T = M = 5000, B = 65536 trajectories, kernel_len 8, bf16 flow products: BASELINE
configs[1]) trained for --steps ELBO steps from its random init (bench.build_model; synthetic series generated with
theta = (5, 0.5, 3)): every --every steps the batch-mean per-sample ELBO and the q(theta) posterior mean / sd of
(theta0, theta1, e^theta2) over 4096 draws, as JSON lines -- that the full-size step trains (finite, improving ELBO,
the posterior moving) and what it costs end to end.  usage: python scripts/ar_cfg_train.py [--steps N] [--every K]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from scripts.ar_recovery import posterior  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--precision", default="bf16")
    a = ap.parse_args()
    from viforssms_amd import _lib
    from viforssms_amd.launch import init_distributed
    args = bench.parse_args(["--precision", a.precision])
    ctx = init_distributed()
    dev = torch.device("cuda", 0)
    model, _ = bench.build_model(args, ctx, dev, _lib.TRAIN_PRECISIONS[a.precision])
    t0 = time.time()
    m, s = posterior(model)
    print(json.dumps({"step": 0, "posterior_mean": [round(x, 4) for x in m], "posterior_sd": [round(x, 4) for x in s]}),
          flush=True)
    for step in range(1, a.steps + 1):
        out = model.elbo_step(model.batch_for(model.select_windows()), step)
        if step % a.every == 0:
            e = out["elbo"].double()
            torch.cuda.synchronize()
            m, s = posterior(model)
            print(json.dumps({"step": step, "elbo_mean": float(e.mean()), "elbo_finite": bool(torch.isfinite(e).all()),
                              "posterior_mean": [round(x, 4) for x in m], "posterior_sd": [round(x, 4) for x in s],
                              "elapsed_s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
