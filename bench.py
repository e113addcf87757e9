"""Benchmark: one full NMA-VI ELBO training step of the AR(1) config on MI355X.

Workload (BASELINE.json configs[1]): AR(1), T = 5000, impute = 5, kernel_len = 8, n_flows = 3,
network_dims = [50, 50, 50], feat_window = 10; "batch_dims" = 65536 mapped to B = 65536
trajectories per GPU, each covering the whole series (window length M = T).
A step = window pick -> feature gather -> base noise (Philox) -> 3 IAF flows -> ELBO densities ->
backward -> [RCCL all-reduce] -> global-norm clip + Adamax.  metric = latent-state transitions/s
= (all ranks' B) * T / step time (weak scaling: B per GPU is fixed).

roofline: the dominant kernel is the IAF-flow backward (flow_bwd_kernel); its algorithmic FLOPs
per launch divided by its average launch time, measured live with HIP events on
the launch stream during the timed steps.  cpu_baseline: the fp32 CPU restatement of the same
step (oracle/, "port") on a bounded sample of trajectories, timed on this host.

Usage: python bench.py [--gpus N --steps K --warmup W]  (N > 1 under torch.distributed.run)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "latent-state transitions/sec (batch_dims×T per step), AR(1) T=5000, 1/2/4/8 GPU"
PEAKS_TFLOPS = {"fp32": 157.3, "bf16": 2500.0, "bf16x3": 2500.0 / 3}  # MI355X dense (MI355X_MICROARCH.md);
# bf16x3 issues three bf16 MFMAs per product, so its ceiling is a third of the bf16 peak


def flow_bwd_flops_per_position(k, H, nh):
    """Algorithmic FLOPs of the flow backward per (sample, head position): recompute forward
    (2kH + 2 nh H^2 + 4H) + hidden dX and dW (4 nh H^2) + head (8H) + first-layer dW_eps and dU (4kH)."""
    return 6 * k * H + 6 * nh * H * H + 12 * H


def measured_traffic(args):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary
    (profiles/traffic.json, written by scripts/traffic_from_pmc.py from separate FETCH_SIZE /
    WRITE_SIZE rocprofv3 passes of this same command), or None when no summary matches."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        e = d.get(args.precision)
        if e and e.get("B") == args.B and e.get("T") == args.T and e.get("k") == args.k:
            return e["bytes_per_launch"]
    except (ValueError, KeyError):
        pass
    return None


def cpu_baseline(args, obs, ob, tt):
    """fp32 CPU restatement (oracle/) of the same step on a bounded sample of trajectories."""
    import torch
    from oracle import nma_oracle as O
    B = args.cpu_B
    spec = O.ModelSpec(family="ar", p=B, M=args.T, k=args.k, n_flows=3, H=50, n_layers=3, C_time=14, P_theta=3,
                       target=float(args.T), priors=[(0.0, 10.0)] * 3, base_loc=1.5, base_scale=0.5)
    g = torch.Generator().manual_seed(0)
    params = O.init_params(spec, g, dtype=torch.float32)
    ts = torch.tensor(O.ar_time_feats(obs, ob, tt, 3, args.k, args.T, 10, args.T, [0] * B), dtype=torch.float32)
    leaves = O.param_leaves(params)
    slots = [(torch.zeros_like(t), torch.zeros_like(t)) for t in leaves]
    perms = [[0, 1, 2], [0, 2, 1], [0, 2, 1], [2, 0, 1]]
    times = []
    t_start = time.time()
    i = 0
    while True:
        eps = torch.randn(B, spec.kernel_ext, generator=g)
        x0 = torch.randn(B, 3, generator=g) * 0.5 + 1.5
        t0 = time.perf_counter()
        new, slots, _ = O.train_step(spec, params, slots, perms, x0, eps, ts, {}, 1e-3, clip=2.5e8)
        times.append(time.perf_counter() - t0)
        i += 1
        if i >= 2 + args.cpu_min_steps or time.time() - t_start > args.cpu_seconds:
            break
    steady = times[2:] if len(times) > 2 else times
    t = float(np.median(steady))
    return {"value": B * args.T / t, "unit": "transitions/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"fp32 CPU restatement of the TF1 step (oracle/nma_oracle.py) on B={B} trajectories x "
                      f"T={args.T}, median of {len(steady)} steps after 2 warm-up ({t:.2f} s/step)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--B", type=int, default=65536, help="trajectories per GPU")
    ap.add_argument("--T", type=int, default=5000)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--precision", choices=["fp32", "bf16", "bf16x3"], default="bf16",
                    help="flow-kernel MFMA operand precision (BASELINE configs[1]: bf16); ELBO densities, "
                         "reductions and the optimizer are fp32 throughout")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-B", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=25.0)
    ap.add_argument("--cpu-min-steps", type=int, default=5)
    args = ap.parse_args()

    import torch
    from viforssms_amd import _lib
    from viforssms_amd.ar import VI_SSM, build_theta_spec
    from viforssms_amd.data import data_gen
    from viforssms_amd.launch import init_distributed

    ctx = init_distributed()
    world, rank = ctx.world, ctx.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    prec = {"fp32": _lib.VISSM_PREC_FP32, "bf16": _lib.VISSM_PREC_BF16, "bf16x3": _lib.VISSM_PREC_BF16X3}[args.precision]

    # synthetic data of the configured shape: data_gen(5000, 5, 10, [5, .5, 3], 1) after seed(1)
    np.random.seed(1)
    np.random.seed(1)
    obs, ob, tt = data_gen(args.T, 5, 10.0, np.array([5.0, 0.5, 3.0]), 1.0, write=False)
    obs, ob, tt = (np.asarray(a, dtype=np.float32) for a in (obs, ob, tt))
    theta_spec = build_theta_spec([(0.0, 10.0)] * 3)
    p_global = args.B * world
    model = VI_SSM(obs, 1.0, 10.0, theta_spec, [(0.0, 10.0)] * 3, args.T, p_global, args.k, args.T, [50, 50, 50], 3,
                   10, ob, tt, pre_train=False, learn_rate=1e-3, grad_clip=2.5e8, device=dev, precision=prec,
                   dist=ctx, log_every=10 ** 9)
    model.build_flow()
    lib = _lib.load()

    def step(i):
        starts = model.select_windows()
        batch = model.batch_for(starts)
        model.elbo_step(batch, i)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    lib.vissm_profile_reset()
    lib.vissm_profile_enable(1)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    lib.vissm_profile_enable(0)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    import ctypes
    tot = ctypes.c_double()
    cnt = ctypes.c_int64()
    _lib.check(lib.vissm_profile_read(_lib.PROF_FLOW_BWD, ctypes.byref(tot), ctypes.byref(cnt)), "profile_read")
    bwd_ms, bwd_n = tot.value, cnt.value
    _lib.check(lib.vissm_profile_read(_lib.PROF_FLOW_FWD, ctypes.byref(tot), ctypes.byref(cnt)), "profile_read")
    fwd_ms, fwd_n = tot.value, cnt.value
    lib.vissm_profile_reset()

    if rank != 0:
        return
    B, T, k, H, nh = args.B, args.T, args.k, 50, 1
    kext = 3 * k + T + 1
    Lh = [kext - i * k - k for i in range(3)]
    fl_pos = flow_bwd_flops_per_position(k, H, nh)
    flops_per_launch = B * fl_pos * sum(Lh) / 3.0
    avg_launch_s = bwd_ms / max(bwd_n, 1) / 1e3
    achieved = flops_per_launch / avg_launch_s / 1e12 if bwd_n else None
    peak = PEAKS_TFLOPS[args.precision]
    kernel = "flow5::bwd_kernel (bf16 matrix cores)" if args.precision != "fp32" else "flow4::bwd_kernel (fp32 matrix cores)"
    traffic = measured_traffic(args)
    value = world * B * T * args.steps / elapsed
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "transitions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic: AR(1) series from data_gen(5000, impute=5, x0=10, theta=[5,.5,3], obs_std=1) after "
                "np.random.seed(1); random-init (glorot) weights; base noise from Philox",
        "config": {"workload": f"AR(1) ELBO train step, T=M={T}, impute=5, kernel_len={k}, no_flows=3, "
                               f"network_dims=[50,50,50], feat_window=10, B={B} trajectories per GPU "
                               f"(BASELINE batch_dims -> B)", "global_batch": B * world, "seq_len": T,
                   "parallelism": f"dp{world}"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": (achieved / peak) if achieved else None, "traffic": traffic,
                     "kernel": kernel, "flops_per_launch": flops_per_launch,
                     "avg_launch_ms": avg_launch_s * 1e3, "launches": bwd_n,
                     "fwd_kernel_avg_ms": fwd_ms / max(fwd_n, 1)},
    }
    if args.cpu_baseline == "auto" and world == 1:
        res["cpu_baseline"] = cpu_baseline(args, obs, ob, tt)
    else:
        res["cpu_baseline"] = None
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
