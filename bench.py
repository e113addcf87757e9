"""Benchmark: one full NMA-VI ELBO training step of the AR(1) config on MI355X.

Workload (BASELINE.json configs[1]): AR(1), T = 5000, impute = 5, kernel_len = 8, n_flows = 3,
network_dims = [50, 50, 50], feat_window = 10; "batch_dims" = 65536 mapped to B = 65536
trajectories per GPU, each covering the whole series (window length M = T).
A step = window pick -> feature gather -> base noise (Philox) -> 3 IAF flows -> ELBO densities ->
backward -> [RCCL all-reduce] -> global-norm clip + Adamax.  metric = latent-state transitions/s
= (all ranks' B) * T / step time (weak scaling: B per GPU is fixed).

roofline: the dominant kernel is the IAF-flow backward (flow_bwd_kernel); its algorithmic FLOPs per
launch (2 x F_fwd per sample and head position, SURVEY.md §8d -- the recomputed forward is not
counted) divided by its average launch time, measured live with HIP events on the launch stream
during the timed steps; mixed_roof_frac prices the same FLOPs with the vector terms at the fp32
vector peak.  step_roofline: sum of every kernel's t_min under its own roof / measured step time.
parity_precision: the same step timed at the precisions that hold the per-sample ELBO within 1e-4 of the
oracle -- bf16x2 (split weights in every weight product, forward and backward: gradient within 1e-3 too), bf16x2f
(split-weight forward only), bf16x3f and bf16x3 (every operand split; gradient within 1e-3 too).
cpu_baseline: the fp32 CPU restatement of the same step (oracle/, "port") on a bounded sample of
trajectories, timed on this host, plus the AR plumbing config (p = 50, M = 50, k = 50) at true size.

Usage: python bench.py [--gpus N --steps K --warmup W]  (N > 1: launched by torch.distributed.run with
--gpus N, or started as plain `python bench.py --gpus N`, which spawns the N ranks itself)
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
PEAKS_TFLOPS = {"fp32": 157.3, "bf16": 2500.0, "bf16x3": 2500.0 / 3, "bf16x3f": 2500.0, "bf16x2f": 2500.0,
                "bf16x2": 2500.0 / 2}  # MI355X dense (MI355X_MICROARCH.md);
# bf16x3 issues three bf16 MFMAs per product, so its ceiling is a third of the bf16 peak (bf16x2: two per weight
# product; priced at half the peak)
VALU_PEAK_TFLOPS = 157.3  # fp32 vector (packed FMA) peak


def flow_fwd_flops_per_position(k, H, nh, bn=False):
    """SURVEY.md §8(d) algorithmic FLOPs of one flow's forward per (sample, head position):
    F_fwd = 2kH + 3H + nh (2H^2 + 2H [+ 2H BN]) + 4H + 6.  Returns (F_mfma, F_valu): the nh 2H^2
    hidden contractions are the matrix-core terms, the rest vector work."""
    f_mfma = nh * 2 * H * H
    f_all = 2 * k * H + 3 * H + nh * (2 * H * H + 2 * H + (2 * H if bn else 0)) + 4 * H + 6
    return f_mfma, f_all - f_mfma


def flow_bwd_flops_per_position(k, H, nh, bn=False):
    """Algorithmic backward FLOPs = 2 F_fwd; the forward the kernel recomputes is
    not counted (reported separately as recompute_flops_per_launch)."""
    f_mfma, f_valu = flow_fwd_flops_per_position(k, H, nh, bn)
    return 2 * (f_mfma + f_valu)


def mixed_roof_s(positions, k, H, nh, bn, mfma_peak_tflops, passes):
    """t_min of `passes` x F_fwd per position with the MFMA terms at the matrix-core peak and the
    rest at the fp32 vector peak (157.3 TFLOP/s) -- SURVEY.md §8(d)'s roof for the flow kernels."""
    f_mfma, f_valu = flow_fwd_flops_per_position(k, H, nh, bn)
    return passes * positions * (f_mfma / (mfma_peak_tflops * 1e12) + f_valu / (VALU_PEAK_TFLOPS * 1e12))


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


def _cpu_ar_step_rate(B, M, k, T, obs, ob, tt, seconds, min_steps):
    """Median seconds per step of the fp32 CPU restatement (oracle/) of the AR step at (B, M, k)."""
    import torch
    from oracle import nma_oracle as O
    spec = O.ModelSpec(family="ar", p=B, M=M, k=k, n_flows=3, H=50, n_layers=3, C_time=14, P_theta=3,
                       target=float(T), priors=[(0.0, 10.0)] * 3, base_loc=1.5, base_scale=0.5)
    g = torch.Generator().manual_seed(0)
    params = O.init_params(spec, g, dtype=torch.float32)
    rs = np.random.RandomState(0)
    leaves = O.param_leaves(params)
    slots = [(torch.zeros_like(t), torch.zeros_like(t)) for t in leaves]
    perms = [[0, 1, 2], [0, 2, 1], [0, 2, 1], [2, 0, 1]]
    times = []
    t_start = time.time()
    while True:
        # window draw as AR.py:263-265 (fresh windows every step, like the reference loop)
        starts = rs.choice(np.arange(0, T, M), size=B, replace=M * B >= T).tolist()
        ts = torch.tensor(O.ar_time_feats(obs, ob, tt, 3, k, M, 10, T, starts), dtype=torch.float32)
        eps = torch.randn(B, spec.kernel_ext, generator=g)
        x0 = torch.randn(B, 3, generator=g) * 0.5 + 1.5
        t0 = time.perf_counter()
        _, slots, _ = O.train_step(spec, params, slots, perms, x0, eps, ts, {}, 1e-3, clip=2.5e8)
        times.append(time.perf_counter() - t0)
        if len(times) >= 2 + min_steps or time.time() - t_start > seconds:
            break
    steady = times[2:] if len(times) > 2 else times
    return float(np.median(steady)), len(steady), torch.get_num_threads()


def host_cpu():
    """The host the CPU baseline runs on: logical CPUs of the machine (os.cpu_count), CPUs this process
    may run on (`nproc`: sched_getaffinity), the torch intra-op thread count actually used, and the
    /proc/cpuinfo model name."""
    import torch
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        nproc = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        nproc = os.cpu_count()
    return {"cpu_model": model, "nproc": nproc, "machine_cpus": os.cpu_count(), "threads_used": torch.get_num_threads(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cgroup_cpus():
    """CPUs granted by the cgroup v2 quota (cpu.max "quota period"), or None when unlimited / unreadable: on a
    shared GPU box `nproc` lists the whole machine while the job's share is smaller."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def cpu_baseline(args, obs, ob, tt):
    """fp32 CPU restatement (oracle/) of the same step on a bounded sample of trajectories, timed at the
    process's default thread count (OMP_NUM_THREADS: the box's CPU share) and at `nproc` threads
    (len(sched_getaffinity)); `value` / `cores` are the faster of the two."""
    import torch
    B = min(args.cpu_B, args.B)
    host = host_cpu()
    default_threads = torch.get_num_threads()
    host["cgroup_cpus"] = cgroup_cpus()
    # nproc threads unless the cgroup grants fewer CPUs: on the GPU box nproc = 256 while the quota is 16, and 256
    # threads on 16 CPUs ran one step in 134 s (2.4e3 transitions/s, profiles/r04/bench_full_r04b.json) -- an
    # oversubscription artefact, not the host's rate
    usable = host["nproc"] if not host["cgroup_cpus"] else min(host["nproc"], max(1, int(host["cgroup_cpus"])))
    lines = []
    for threads in sorted({default_threads, usable}):
        torch.set_num_threads(threads)
        secs = args.cpu_seconds if threads == default_threads else args.cpu_seconds / 2
        t, n, _ = _cpu_ar_step_rate(B, args.M, args.k, args.T, obs, ob, tt, secs, args.cpu_min_steps)
        lines.append({"threads": threads, "value": B * args.M / t, "s_per_step": t, "steps": n})
    torch.set_num_threads(default_threads)
    best = max(lines, key=lambda x: x["value"])
    return {"value": best["value"], "unit": "transitions/s", "cores": best["threads"], "kind": "port", "host": host,
            "by_threads": lines,
            "sample": f"fp32 CPU restatement of the TF1 step (oracle/nma_oracle.py) on B={B} trajectories x "
                      f"M={args.M} (T={args.T}, k={args.k}), median of the steps after 2 warm-up, at "
                      f"{' and '.join(str(x['threads']) for x in lines)} torch threads (nproc = {host['nproc']}, "
                      f"cgroup CPU quota = {host['cgroup_cpus']}: threads capped at the quota); value = the faster "
                      f"({best['threads']} threads, "
                      f"{best['s_per_step']:.2f} s/step)"}


def cpu_baseline_ar_plumbing(args):
    """SURVEY.md §8(d) config 1 at its true size: `python main.py hyperparameters.txt` (p = 50 windows
    of M = 50, k = 50, data_gen(5000, impute=1, ...) after np.random.seed(1)), fp32 CPU restatement."""
    from viforssms_amd.data import data_gen
    np.random.seed(1)
    obs, ob, tt = data_gen(5000, 1, 10.0, np.array([5.0, 0.5, 3.0]), 1.0, write=False)
    t, n, cores = _cpu_ar_step_rate(50, 50, 50, 5000, obs, ob, tt, args.cpu_seconds / 2, max(args.cpu_min_steps, 10))
    return {"value": 50 * 50 / t, "unit": "transitions/s", "cores": cores, "kind": "port",
            "ms_per_step": t * 1e3,
            "sample": f"AR plumbing config (hyperparameters.txt: p=50, M=50, k=50, T=5000) at its true size, fp32 CPU "
                      f"restatement, median of {n} steps after 2 warm-up"}


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
        meta = dict(D=1, nh=1, n_flows=3, bn=False, ar_data=(obs, ob, tt),
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
        meta = dict(D=1, nh=3, n_flows=5, bn=True, data="dat/SV.dat[300:] (the reference's series); random-init weights",
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
        meta = dict(D=2, nh=3, n_flows=3, bn=True,
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
        meta = dict(D=2, nh=3, n_flows=3, bn=True,
                    data="synthetic: Euler-Maruyama FHN path, x0=(2,3), dt=0.1, obs N(x,0.1) every 10 steps; "
                         "random-init weights",
                    workload=f"FitzHugh-Nagumo ELBO train step (fitz_nag_NVP.py), T=M={args.T}, kernel_len={args.k}, "
                             f"no_flows=3, network_dims=[50]*5, feat_window=10, B={args.B} per GPU")
    model.build_flow()
    return model, meta


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (default: the launcher's WORLD_SIZE, else 1)")
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
    ap.add_argument("--precision", choices=["fp32", "bf16", "bf16x2", "bf16x3", "bf16x3f", "bf16x2f"], default="bf16",
                    help="flow-kernel MFMA operand precision (BASELINE configs[1]: bf16); ELBO densities, "
                         "reductions and the optimizer are fp32 throughout")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as a captured HIP graph (viforssms_amd.graph; needs warmup >= 3)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--fuse", choices=["on", "off"], default="on",
                    help="AR at bf16 / bf16x3: run the last flow fused with the ELBO terms (vissm_flow_ar_elbo_fused)")
    ap.add_argument("--parity-line", choices=["auto", "off"], default="auto",
                    help="also time the step at bf16x3 (AR, bf16, 1 GPU) and report it as parity_precision")
    ap.add_argument("--families", choices=["auto", "off"], default="auto",
                    help="AR run: also time LV (every GPU count), SV and FHN (one GPU) at their per-GPU shapes "
                         "and report them under family_lines")
    ap.add_argument("--family-steps", type=int, default=3)
    ap.add_argument("--cpu-B", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=25.0)
    ap.add_argument("--cpu-min-steps", type=int, default=5)
    args = ap.parse_args(argv)
    dB, dT, dk = MODEL_DEFAULTS[args.model]
    args.B = args.B or dB
    args.T = args.T or dT
    args.k = args.k or dk
    args.M = args.M or args.T
    if args.model != "ar" and args.M != args.T:
        ap.error("--M applies to the AR model only")
    return args


def measure(args, ctx, dev, parity_line: bool):
    """Build args.model's workload, time it (warm-up, then exactly args.steps steps between barrier +
    synchronize, max over ranks) and return the result dict (on every rank; rank 0 prints it)."""
    import ctypes
    import torch
    from viforssms_amd import _lib

    world, rank = ctx.world, ctx.rank
    if world > 1:
        import torch.distributed as dist
    prec = _lib.TRAIN_PRECISIONS[args.precision]
    model, meta = build_model(args, ctx, dev, prec)
    model.engine.fuse_last = args.fuse == "on"
    lib = _lib.load()

    def step(i):
        starts = model.select_windows()
        if args.graph:
            model.graphed_step(starts, i)
        else:
            model.elbo_step(model.batch_for(starts), i)

    if args.graph:
        args.warmup = max(args.warmup, 3)  # two eager warm-up steps, then the capture

    kinds = (_lib.PROF_FLOW_FWD, _lib.PROF_FLOW_BWD, _lib.PROF_ELBO_FWD, _lib.PROF_ELBO_BWD, _lib.PROF_NORMAL,
             _lib.PROF_FLOW_BWD_NODU, _lib.PROF_FLOW_BWD_DU, _lib.PROF_FLOW_FUSED)

    def timed(first_step):
        """Warm-up, then EXACTLY args.steps timed steps between barrier + synchronize on both sides;
        max over ranks.  Returns (elapsed_s, {profile kind: (ms, launches, algorithmic bytes)})."""
        for i in range(args.warmup):
            step(first_step + i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        lib.vissm_profile_reset()
        lib.vissm_profile_enable(1)
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(first_step + args.warmup + i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        lib.vissm_profile_enable(0)
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        tot, cnt, nbytes = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        prof = {}
        for kind in kinds:
            _lib.check(lib.vissm_profile_read(kind, ctypes.byref(tot), ctypes.byref(cnt)), "profile_read")
            _lib.check(lib.vissm_profile_bytes(kind, ctypes.byref(nbytes)), "profile_bytes")
            prof[kind] = (tot.value, cnt.value, nbytes.value)
        lib.vissm_profile_reset()
        return elapsed, prof

    elapsed, prof = timed(0)
    # parity-precision lines: the same step at the precisions that hold the per-sample ELBO within
    # north_star's 1e-4 of the float64 oracle, timed the same way
    px = None
    if parity_line and args.precision == "bf16" and args.model == "ar" and world == 1 and not args.graph:
        px = []
        for name, mode, note in (
                ("bf16x2", _lib.VISSM_PREC_BF16X2,
                 "every product with a weight operand as split-bf16 weights x bf16 activations (w_hi x + w_lo x), the "
                 "forward, the backward's recompute and its chain (W dZ, w_eps dA0, the head backward) alike; "
                 "weight-gradient products single bf16: per-sample ELBO within 1e-4 AND gradient within 1e-3 of the "
                 "float64 oracle (tests/test_gpu_config_parity.py, tests/test_gpu_fused.py)"),
                ("bf16x2f", _lib.VISSM_PREC_BF16X2F,
                 "forward flow products with split-bf16 weights (w_hi x + w_lo x: the weights' rounding, coherent "
                 "over a path, removed) and bf16 activations, backward products bf16 (the last flow fused with the "
                 "ELBO terms, its recompute on split weights): per-sample ELBO within 1e-4 of the float64 oracle, "
                 "gradient at bf16 accuracy (tests/test_gpu_config_parity.py, tests/test_gpu_fused.py)"),
                ("bf16x3f", _lib.VISSM_PREC_BF16X3F,
                 "forward flow products bf16x3 (the values reaching the ELBO), backward products bf16: per-sample "
                 "ELBO within 1e-4 of the float64 oracle, gradient at bf16 accuracy (tests/test_gpu_config_parity.py)"),
                ("bf16x3", _lib.VISSM_PREC_BF16X3,
                 "every flow product split bf16 hi+lo (three MFMAs): ELBO within 1e-4 and gradient within 1e-3 of "
                 "the float64 oracle")):
            model.engine.precision = mode
            px_elapsed, px_prof = timed(args.warmup + args.steps)
            b_ms, b_n, _ = px_prof[_lib.PROF_FLOW_BWD]
            f_ms, f_n, _ = px_prof[_lib.PROF_FLOW_FWD]
            px.append({"dtype": name, "value": world * args.B * args.M * args.steps / px_elapsed,
                       "ms_per_step": px_elapsed / args.steps * 1e3, "flow_bwd_avg_ms": b_ms / max(b_n, 1),
                       "flow_fwd_avg_ms": f_ms / max(f_n, 1),
                       "last_flow_fused": bool(px_prof[_lib.PROF_FLOW_FUSED][1]), "note": note})
        model.engine.precision = prec

    B, T, k, H, nh, nf, D, bn = args.B, args.M, args.k, 50, meta["nh"], meta["n_flows"], meta["D"], meta["bn"]
    kext = nf * k + D * T + D
    Lh = [(kext - i * k - k) // D for i in range(nf)]
    positions_per_launch = B * sum(Lh) / nf
    fwd_ms, fwd_n, _ = prof[_lib.PROF_FLOW_FWD]
    bwd_ms, bwd_n, _ = prof[_lib.PROF_FLOW_BWD]
    f_pos = flow_bwd_flops_per_position(k, H, nh, bn)
    flops_per_launch = positions_per_launch * f_pos
    avg_launch_s = bwd_ms / max(bwd_n, 1) / 1e3
    achieved = flops_per_launch / avg_launch_s / 1e12 if bwd_n else None
    peak = PEAKS_TFLOPS[args.precision]
    kernel = "flow5::bwd_kernel (bf16 matrix cores)" if args.precision != "fp32" else "flow4::bwd_kernel (fp32 matrix cores)"
    traffic = measured_traffic(args)
    t_step = elapsed / args.steps
    value = world * B * T * args.steps / elapsed
    mfma_peak = PEAKS_TFLOPS[args.precision] if args.precision != "fp32" else VALU_PEAK_TFLOPS
    bwd_roof_s = mixed_roof_s(positions_per_launch, k, H, nh, bn, mfma_peak, 2)
    # the backward launches by variant: flow 0 without du (its input is the base noise), the middle flows,
    # and (AR, bf16 / bf16x3) the last flow fused with its ELBO terms; each with the positions of its flow
    variants = {}
    has_nodu, has_fused = bool(prof[_lib.PROF_FLOW_BWD_NODU][1]), bool(prof[_lib.PROF_FLOW_FUSED][1])
    flows_of = {_lib.PROF_FLOW_BWD_NODU: [0], _lib.PROF_FLOW_FUSED: [nf - 1],
                _lib.PROF_FLOW_BWD_DU: [i for i in range(nf) if not (i == 0 and has_nodu)
                                        and not (i == nf - 1 and has_fused)]}
    for kind, key in ((_lib.PROF_FLOW_BWD_NODU, "first_flow_no_du"), (_lib.PROF_FLOW_BWD_DU, "middle_flows_du"),
                      (_lib.PROF_FLOW_FUSED, "last_flow_fused_elbo")):
        ms, n, _ = prof[kind]
        fl = flows_of[kind]
        if not n or not fl:
            continue
        pos = B * sum(Lh[i] for i in fl) / len(fl)
        a_ms = ms / n
        ach = pos * f_pos / (a_ms / 1e3) / 1e12
        variants[key] = {"avg_launch_ms": a_ms, "launches": n, "flows": fl, "achieved": ach, "frac": ach / peak,
                         "mixed_roof_frac": mixed_roof_s(pos, k, H, nh, bn, mfma_peak, 2) / (a_ms / 1e3)}
    res = {
        "metric": METRIC if args.model == "ar" else METRIC.replace("AR(1) T=5000", f"{args.model.upper()} T={T}"),
        "value": value,
        "unit": "transitions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_step * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": meta["data"],
        "config": {"workload": meta["workload"], "global_batch": B * world, "seq_len": args.T,
                   "parallelism": f"dp{world}", "hip_graph": bool(args.graph),
                   # gradient bytes SUM-all-reduced per step and rank (LV at >1 ranks: each flow's dC instead of
                   # its window-shared variables, vi_ssm.VISSMBase._shared_grad_plan)
                   "allreduce_bytes_per_step": int(getattr(model, "last_allreduce_bytes", 0)),
                   "last_flow_fused": bool(model.engine.fused_ok(model.batch_for(model.select_windows()), B))},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": (achieved / peak) if achieved else None, "traffic": traffic,
                     "kernel": kernel, "flops_per_launch": flops_per_launch,
                     "flops_accounting": "2 x F_fwd per (sample, head position), SURVEY.md §8(d); "
                                         "the recomputed forward is not counted",
                     "recompute_flops_per_launch": flops_per_launch / 2,
                     "avg_launch_ms": avg_launch_s * 1e3, "launches": bwd_n,
                     "variants": variants,
                     "mixed_roof_ms": bwd_roof_s * 1e3,
                     "mixed_roof_frac": bwd_roof_s / avg_launch_s if bwd_n else None,
                     "fwd_kernel_avg_ms": fwd_ms / max(fwd_n, 1)},
    }
    # the HBM-bound streaming kernels of the step: the algorithmic bytes each launch
    # states (libvissm records them with its HIP events: z read / dz written by the log-density kernels,
    # eps written by the base-noise kernel) over the live launch time, against the 8 TB/s HBM peak
    fused = bool(prof[_lib.PROF_FLOW_FUSED][1])
    names = {_lib.PROF_ELBO_FWD: ("elbo_fwd_kernel (reads z: the log-densities and their per-sample theta gradient in "
                                  "one pass, vissm_elbo_fwd_theta_grad)") if fused else
                                 "elbo_fwd_kernel (log-densities: reads z)",
             _lib.PROF_ELBO_BWD: ("elbo_bwd_kernel (reads z, writes the per-sample theta gradient only: the fused "
                                  "last flow differentiated through z itself)") if fused else
                                 ("elbo_onepass_kernel (values, dz and dtheta from one read of z: reads z, writes dz; "
                                  "vissm_elbo_fwd_grad)") if model.engine.onepass_ok() else
                                 "elbo_bwd_kernel (reads z, writes dz)",
             _lib.PROF_NORMAL: "normal_base_kernel (Philox base noise: writes eps)"}
    streaming = []
    for kind, name in names.items():
        ms, n, nb = prof[kind]
        if n and ms > 0:
            gbs = nb / (ms / 1e3) / 1e9
            streaming.append({"kernel": name, "bound": "hbm", "bytes_per_launch": nb / n, "avg_launch_ms": ms / n,
                              "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                              "launches": n})
    res["streaming_rooflines"] = streaming
    # SURVEY.md §8(d) step-level accounting: sum over the step's kernels of each one's t_min under its own
    # roof (flows: MFMA terms at the matrix-core peak + vector terms at 157.3 TF; streaming kernels: their
    # algorithmic bytes at 8 TB/s; Adamax: 32 B/param), divided by the measured step time
    terms = {
        "flow_fwd": mixed_roof_s(positions_per_launch, k, H, nh, bn, mfma_peak, 1) * nf,
        "flow_bwd": bwd_roof_s * nf,
        "adamax": 32.0 * model.store.numel / (HBM_PEAK_GBS * 1e9),
    }
    for kind, key in ((_lib.PROF_ELBO_FWD, "elbo_fwd"), (_lib.PROF_ELBO_BWD, "elbo_bwd"), (_lib.PROF_NORMAL, "base_noise")):
        ms, n, nb = prof[kind]
        terms[key] = (nb / args.steps) / (HBM_PEAK_GBS * 1e9)
    t_min = sum(terms.values())
    res["step_roofline"] = {"t_min_ms": t_min * 1e3, "t_step_ms": t_step * 1e3, "frac": t_min / t_step,
                            "terms_ms": {kk: v * 1e3 for kk, v in terms.items()},
                            "note": "sum of per-kernel t_min (SURVEY.md §8d) / measured step time"}
    if px is not None:
        res["parity_precision"] = px
    return res, model, meta


FAMILY_NOTE = ("the other model families of BASELINE.json configs[2-4] at their per-GPU shapes, timed in the same run "
               "the same way (warm-up, then exactly `steps` steps between barrier + synchronize, max over ranks): "
               "LV (lotka_volterra_partial.py:402-405) at every GPU count (B = 16384 per GPU: configs[3]'s 131072 "
               "over 8 GPUs), SV and FHN on one GPU; value = transitions/s of all ranks")


def family_lines(args, ctx, dev):
    """LV at every world size, SV and FHN at world 1: the families' step rates with their flow-backward
    roofline, per-variant launch times and streaming-kernel rooflines (north_star: throughput on AR(1) /
    Lotka-Volterra sequences at 1, 2, 4 and 8 GPUs)."""
    import torch
    out = []
    models = ["lv"] + (["sv", "fhn"] if ctx.world == 1 else [])
    for m in models:
        a = parse_args(["--model", m, "--steps", str(args.family_steps), "--warmup", "2",
                        "--precision", args.precision, "--cpu-baseline", "off", "--parity-line", "off"])
        r, model, _ = measure(a, ctx, dev, parity_line=False)
        rl = r["roofline"]
        out.append({"model": m, "value": r["value"], "unit": r["unit"], "ms_per_step": r["ms_per_step"],
                    "steps": a.steps, "warmup": a.warmup, "dtype": r["dtype"], "config": r["config"],
                    "data": r["data"],
                    "roofline": {k: rl[k] for k in ("bound", "achieved", "peak", "unit", "frac", "kernel",
                                                    "avg_launch_ms", "fwd_kernel_avg_ms", "mixed_roof_frac",
                                                    "variants")},
                    "streaming_rooflines": r["streaming_rooflines"], "step_roofline": r["step_roofline"]})
        del model
        torch.cuda.empty_cache()
    return out


def main():
    args = parse_args()

    import torch
    from viforssms_amd.launch import ensure_world, init_distributed

    # --gpus N without torchrun: launch N ranks (torchrun, 127.0.0.1) from here before any GPU call and exit with
    # their status; under torchrun the world must be N
    if args.gpus is not None:
        rc = ensure_world(args.gpus, os.path.abspath(__file__), sys.argv[1:])
        if rc is not None:
            sys.exit(rc)

    ctx = init_distributed()
    dev = torch.device("cuda", torch.cuda.current_device())
    res, model, meta = measure(args, ctx, dev, parity_line=args.parity_line == "auto")
    if args.cpu_baseline == "auto" and ctx.world == 1 and args.model == "ar" and ctx.rank == 0:
        res["cpu_baseline"] = cpu_baseline(args, *meta["ar_data"])
        res["cpu_baseline"]["ar_plumbing"] = cpu_baseline_ar_plumbing(args)
    else:
        res["cpu_baseline"] = None
    if args.families == "auto" and args.model == "ar" and not args.graph:
        del model
        torch.cuda.empty_cache()
        res["family_lines"] = family_lines(args, ctx, dev)
        res["family_lines_note"] = FAMILY_NOTE
    if ctx.rank == 0:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
