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
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
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
        if e and e.get("B") == args.B and e.get("T") == args.T and e.get("k") == args.k and args.M == args.T:
            return e["bytes_per_launch"]
    except (ValueError, KeyError):
        pass
    return None


def cpu_baseline(args, obs, ob, tt):
    """fp32 CPU restatement (oracle/) of the same step on a bounded sample of trajectories."""
    import torch
    from oracle import nma_oracle as O
    B = min(args.cpu_B, args.B)
    spec = O.ModelSpec(family="ar", p=B, M=args.M, k=args.k, n_flows=3, H=50, n_layers=3, C_time=14, P_theta=3,
                       target=float(args.T), priors=[(0.0, 10.0)] * 3, base_loc=1.5, base_scale=0.5)
    g = torch.Generator().manual_seed(0)
    params = O.init_params(spec, g, dtype=torch.float32)
    rs = np.random.RandomState(0)
    starts = rs.choice(np.arange(0, args.T, args.M), size=B, replace=args.M * B >= args.T).tolist()
    ts = torch.tensor(O.ar_time_feats(obs, ob, tt, 3, args.k, args.M, 10, args.T, starts), dtype=torch.float32)
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
    return {"value": B * args.M / t, "unit": "transitions/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"fp32 CPU restatement of the TF1 step (oracle/nma_oracle.py) on B={B} trajectories x "
                      f"M={args.M} (T={args.T}, k={args.k}), median of {len(steady)} steps after 2 warm-up "
                      f"({t:.2f} s/step)"}


MODEL_DEFAULTS = {  # per-GPU batch, T, kernel_len
    "ar": (65536, 5000, 8), "sv": (16384, 1508, 50), "lv": (16384, 5000, 20), "fhn": (8192, 2000, 20)}


def build_model(args, ctx, dev, prec):
    """The benchmarked VI_SSM with synthetic data of the configured shape and random-init weights."""
    from viforssms_amd.vi_ssm import ThetaSpec
    world = ctx.world
    p_global = args.B * world
    common = dict(device=dev, precision=prec, dist=ctx, log_every=10 ** 9)
    if args.model == "ar":
        from viforssms_amd.ar import VI_SSM, build_theta_spec
        from viforssms_amd.data import data_gen
        # data_gen(5000, 5, 10, [5, .5, 3], 1) after seed(1), as main.py does
        np.random.seed(1)
        np.random.seed(1)
        obs, ob, tt = data_gen(args.T, 5, 10.0, np.array([5.0, 0.5, 3.0]), 1.0, write=False)
        obs, ob, tt = (np.asarray(a, dtype=np.float32) for a in (obs, ob, tt))
        theta_spec = build_theta_spec([(0.0, 10.0)] * 3)
        model = VI_SSM(obs, 1.0, 10.0, theta_spec, [(0.0, 10.0)] * 3, args.T, p_global, args.k, args.M, [50, 50, 50],
                       3, 10, ob, tt, pre_train=False, learn_rate=1e-3, grad_clip=2.5e8, **common)
        meta = dict(D=1, nh=1, n_flows=3, ar_data=(obs, ob, tt),
                    data="synthetic: AR(1) series from data_gen(5000, impute=5, x0=10, theta=[5,.5,3], obs_std=1) "
                         "after np.random.seed(1); random-init (glorot) weights; base noise from Philox",
                    workload=f"AR(1) ELBO train step, T={args.T}, M={args.M}, impute=5, kernel_len={args.k}, no_flows=3, "
                             f"network_dims=[50,50,50], feat_window=10, B={args.B} trajectories per GPU "
                             f"(BASELINE batch_dims -> B)")
    elif args.model == "sv":
        from viforssms_amd.sv import VI_SSM
        from viforssms_amd.data import load_sv
        obs = load_sv()[: args.T + 1]
        np.random.seed(1)
        spec = ThetaSpec.build(4, 5, 0.0, 1.0, "relu")
        model = VI_SSM(obs, -8.5, spec, [(0.0, 10.0)] * 4, 1.0, args.T, p_global, args.k, args.T, [50] * 5, args.T,
                       5, 5, learn_rate=1e-4, pre_train=False, **common)
        meta = dict(D=1, nh=3, n_flows=5, data="dat/SV.dat[300:] (the reference's series); random-init weights",
                    workload=f"SV ELBO train step (SV_dense.py), T=M={args.T}, kernel_len={args.k}, no_flows=5, "
                             f"network_dims=[50]*5, feat_window=5, B={args.B} per GPU")
    elif args.model == "lv":
        from viforssms_amd.lv import VI_SSM, PRIORS
        from viforssms_amd.data import lv_data_gen
        obs, ob, tt, _ = lv_data_gen(args.T, dt=0.1, obs_every=100, seed=1)
        np.random.seed(1)
        spec = ThetaSpec.build(3, 4, 0.0, 1.0, "elu")
        model = VI_SSM(obs, ob, tt, np.array([100.0, 100.0]), spec, PRIORS, 0.1, args.T * 0.1, p_global, args.k,
                       args.T, [50] * 5, args.T, 3, 10, pre_train=False, **common)
        meta = dict(D=2, nh=3, n_flows=3,
                    data="synthetic: Euler-Maruyama LV path theta=(0.5,0.0025,0.3), x0=(100,100), dt=0.1, obs N(x,1) "
                         "every 100 steps; random-init weights",
                    workload=f"Lotka-Volterra ELBO train step (lotka_volterra_partial.py), T=M={args.T}, "
                             f"kernel_len={args.k}, no_flows=3, network_dims=[50]*5, feat_window=10, B={args.B} per GPU")
    else:
        from viforssms_amd.fhn import VI_SSM
        from viforssms_amd.data import fhn_data_gen
        obs, ob, tt, _ = fhn_data_gen(args.T, dt=0.1, obs_every=10, seed=1)
        np.random.seed(1)
        spec = ThetaSpec.build(5, 4, 0.0, 1.0, "elu")
        model = VI_SSM(obs, ob, tt, np.array([2.0, 3.0]), spec, [(0.0, 10.0)] * 5, 0.1, args.T * 0.1, p_global,
                       args.k, args.T, [50] * 5, args.T, 3, 10, pre_train=False, **common)
        meta = dict(D=2, nh=3, n_flows=3,
                    data="synthetic: Euler-Maruyama FHN path, x0=(2,3), dt=0.1, obs N(x,0.1) every 10 steps; "
                         "random-init weights",
                    workload=f"FitzHugh-Nagumo ELBO train step (fitz_nag_NVP.py), T=M={args.T}, kernel_len={args.k}, "
                             f"no_flows=3, network_dims=[50]*5, feat_window=10, B={args.B} per GPU")
    model.build_flow()
    return model, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", choices=["ar", "lv", "sv", "fhn"], default="ar",
                    help="ar: the BASELINE metric's workload (configs[1]); lv / sv / fhn: configs[2-4] shapes")
    ap.add_argument("--B", type=int, default=None, help="trajectories per GPU (default per model)")
    ap.add_argument("--T", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--M", type=int, default=None,
                    help="AR window length (reference batch_dims of AR.main; default M = T, the BASELINE workload; "
                         "hyperparameters.txt's case is --B 50 --M 50 --k 50)")
    ap.add_argument("--precision", choices=["fp32", "bf16", "bf16x3"], default="bf16",
                    help="flow-kernel MFMA operand precision (BASELINE configs[1]: bf16); ELBO densities, "
                         "reductions and the optimizer are fp32 throughout")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as a captured HIP graph (viforssms_amd.graph; needs warmup >= 3)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-B", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=25.0)
    ap.add_argument("--cpu-min-steps", type=int, default=5)
    args = ap.parse_args()
    dB, dT, dk = MODEL_DEFAULTS[args.model]
    args.B = args.B or dB
    args.T = args.T or dT
    args.k = args.k or dk
    args.M = args.M or args.T
    if args.model != "ar" and args.M != args.T:
        ap.error("--M applies to the AR model only")

    import torch
    from viforssms_amd import _lib
    from viforssms_amd.launch import init_distributed

    ctx = init_distributed()
    world, rank = ctx.world, ctx.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    prec = {"fp32": _lib.VISSM_PREC_FP32, "bf16": _lib.VISSM_PREC_BF16, "bf16x3": _lib.VISSM_PREC_BF16X3}[args.precision]

    model, meta = build_model(args, ctx, dev, prec)
    lib = _lib.load()

    def step(i):
        starts = model.select_windows()
        if args.graph:
            model.graphed_step(starts, i)
        else:
            model.elbo_step(model.batch_for(starts), i)

    if args.graph:
        args.warmup = max(args.warmup, 3)  # two eager warm-up steps, then the capture

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
    stream_ms = {}
    nbytes = ctypes.c_double()
    for kind in (_lib.PROF_ELBO_FWD, _lib.PROF_ELBO_BWD, _lib.PROF_NORMAL):
        _lib.check(lib.vissm_profile_read(kind, ctypes.byref(tot), ctypes.byref(cnt)), "profile_read")
        _lib.check(lib.vissm_profile_bytes(kind, ctypes.byref(nbytes)), "profile_bytes")
        stream_ms[kind] = (tot.value, cnt.value, nbytes.value)
    lib.vissm_profile_reset()

    if rank != 0:
        return
    B, T, k, H, nh, nf, D = args.B, args.M, args.k, 50, meta["nh"], meta["n_flows"], meta["D"]
    kext = nf * k + D * T + D
    Lh = [(kext - i * k - k) // D for i in range(nf)]
    fl_pos = flow_bwd_flops_per_position(k, H, nh)
    flops_per_launch = B * fl_pos * sum(Lh) / nf
    avg_launch_s = bwd_ms / max(bwd_n, 1) / 1e3
    achieved = flops_per_launch / avg_launch_s / 1e12 if bwd_n else None
    peak = PEAKS_TFLOPS[args.precision]
    kernel = "flow5::bwd_kernel (bf16 matrix cores)" if args.precision != "fp32" else "flow4::bwd_kernel (fp32 matrix cores)"
    traffic = measured_traffic(args)
    value = world * B * T * args.steps / elapsed
    res = {
        "metric": METRIC if args.model == "ar" else METRIC.replace("AR(1) T=5000", f"{args.model.upper()} T={T}"),
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
        "data": meta["data"],
        "config": {"workload": meta["workload"], "global_batch": B * world, "seq_len": args.T,
                   "parallelism": f"dp{world}", "hip_graph": bool(args.graph)},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": (achieved / peak) if achieved else None, "traffic": traffic,
                     "kernel": kernel, "flops_per_launch": flops_per_launch,
                     "avg_launch_ms": avg_launch_s * 1e3, "launches": bwd_n,
                     "fwd_kernel_avg_ms": fwd_ms / max(fwd_n, 1)},
    }
    # the HBM-bound streaming kernels of the step: the algorithmic bytes each launch
    # states (libvissm records them with its HIP events: z read / dz written by the log-density kernels,
    # eps written by the base-noise kernel) over the live launch time, against the 8 TB/s HBM peak
    names = {_lib.PROF_ELBO_FWD: "elbo_fwd_kernel (log-densities: reads z)",
             _lib.PROF_ELBO_BWD: "elbo_bwd_kernel (reads z, writes dz)",
             _lib.PROF_NORMAL: "normal_base_kernel (Philox base noise: writes eps)"}
    streaming = []
    for kind, name in names.items():
        ms, n, nb = stream_ms[kind]
        if n and ms > 0:
            gbs = nb / (ms / 1e3) / 1e9
            streaming.append({"kernel": name, "bound": "hbm", "bytes_per_launch": nb / n, "avg_launch_ms": ms / n,
                              "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                              "launches": n})
    res["streaming_rooflines"] = streaming
    if args.cpu_baseline == "auto" and world == 1 and args.model == "ar":
        res["cpu_baseline"] = cpu_baseline(args, *meta["ar_data"])
    else:
        res["cpu_baseline"] = None
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
