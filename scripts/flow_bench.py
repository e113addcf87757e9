"""Flow-kernel micro-benchmark: times vissm_flow_fwd / vissm_flow_bwd alone at a given shape,
interleaving implementations in one process (A/B), and cross-checks their outputs."""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from viforssms_amd import _lib  # noqa: E402
from viforssms_amd.ops import FlowShape, MAFlowFn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16384)
    ap.add_argument("--T", type=int, default=5000)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--H", type=int, default=50)
    ap.add_argument("--nh", type=int, default=1)
    ap.add_argument("--stride2", action="store_true")
    ap.add_argument("--impls", default="fp32,bf16", help="flow precisions to time: fp32, bf16, bf16x3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="", help="run only this impl (for PMC passes)")
    ap.add_argument("--fold", type=int, default=1, help="pass the theta branch's factors (theta_term = theta W + b, "
                    "rank 3): the two-sample AR kernels fold them into the layer-0 product, as the training step does")
    args = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    D = 2 if args.stride2 else 1
    L = 3 * args.k + D * args.T + D
    B, k, H, nh = args.B, args.k, args.H, args.nh
    sh = FlowShape(B=B, L=L, k=k, H=H, n_hidden=nh, bn=nh > 1, stride2=args.stride2, swap_out=False,
                   n_logsig=D * args.T, n_win=1)
    r = lambda *s, sc=1.0: (torch.randn(*s, generator=g, device=dev) * sc).contiguous()
    u = r(B, L)
    C = r(1, sh.Lh, H, sc=0.3)
    th3, wt3, bt3 = r(B, 3, sc=0.5), r(3, H, sc=0.2), r(H, sc=0.1)
    tt = torch.addmm(bt3, th3, wt3).contiguous()
    tf = (th3, wt3, bt3) if args.fold else None
    w_eps, w_hid, b_hid = r(k, H, sc=0.3), r(nh, H, H, sc=0.15), r(nh, H, sc=0.1)
    bn_g, bn_b = (1 + r(nh, H, sc=0.1), r(nh, H, sc=0.1)) if nh > 1 else (None, None)
    w_head, b_head = r(H, 2, sc=0.2), r(2, sc=0.1)
    gnext, gls = r(B, sh.Lout), r(B)
    # entries: an fp32 implementation number (1-4) or "bf16" / "bf16x3" (matrix-core bf16 kernels)
    PREC = {"fp32": _lib.VISSM_PREC_FP32, "bf16": _lib.VISSM_PREC_BF16, "bf16x3": _lib.VISSM_PREC_BF16X3,
            "bf16x2": _lib.VISSM_PREC_BF16X2}   # bf16x2: forward only (its backward runs bf16)
    impls = [x if x in PREC else "fp32" for x in (args.only or args.impls).split(",")]  # legacy 2/4 -> fp32
    import dataclasses
    res = {}
    outs = {}
    kern = {}  # kernel-only times (HIP events around the flow kernel launches, vissm_profile_*)

    def prof_read(which):
        tot, cnt = ctypes.c_double(), ctypes.c_int64()
        _lib.check(lib.vissm_profile_read(which, ctypes.byref(tot), ctypes.byref(cnt)), "profile_read")
        return tot.value, cnt.value

    for rd in range(args.rounds):
        for im in impls:
            lib.vissm_profile_reset()
            lib.vissm_profile_enable(1 if rd > 0 else 0)
            shp = dataclasses.replace(sh, precision=PREC[im],
                                      bwd_precision=_lib.VISSM_PREC_BF16 if im == "bf16x2" else None)
            ins = [t.clone().requires_grad_(True) for t in (u, C, tt, w_eps, w_hid, b_hid, w_head, b_head)]
            extra = [bn_g, bn_b]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            un, ls = MAFlowFn.apply(shp, None, ins[0], ins[1], ins[2], ins[3], ins[4], ins[5], extra[0], extra[1],
                                    ins[6], ins[7], tf)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            torch.autograd.backward([un, ls], [gnext, gls])
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            res.setdefault(im, []).append((t1 - t0, t2 - t1))
            lib.vissm_profile_enable(0)
            if rd > 0:
                (fk, fn), (bk, bn) = prof_read(_lib.PROF_FLOW_FWD), prof_read(_lib.PROF_FLOW_BWD)
                kern.setdefault(im, []).append((fk / max(fn, 1), bk / max(bn, 1)))
            if rd == 0:
                outs[im] = [un.detach(), ls.detach()] + [t.grad for t in ins]
    summary = {}
    for im, v in res.items():
        f = sorted(x[0] for x in v[1:] or v)
        b = sorted(x[1] for x in v[1:] or v)
        summary[im] = {"fwd_ms": 1e3 * f[len(f) // 2], "bwd_ms": 1e3 * b[len(b) // 2]}
        if im in kern:
            kf = sorted(x[0] for x in kern[im])
            kb = sorted(x[1] for x in kern[im])
            summary[im]["fwd_kernel_ms"] = kf[len(kf) // 2]
            summary[im]["bwd_kernel_ms"] = kb[len(kb) // 2]
    if len(outs) > 1:
        ks = sorted(outs, key=str)
        a0 = outs[ks[0]]
        names = ["u_next", "logsig", "du", "dC", "dtheta", "dw_eps", "dw_hid", "db_hid", "dw_head", "db_head"]
        for im in ks[1:]:
            errs = [float((x - y).norm() / (y.norm() + 1e-30)) for x, y in zip(outs[im], a0)]
            summary[im]["max_rel_diff_vs_%s" % ks[0]] = max(errs)
            summary[im]["rel_diff"] = dict(zip(names, errs))
    print(json.dumps({"shape": vars(args), "results": summary}))


if __name__ == "__main__":
    main()
