"""LV / SV / FHN log-density kernels alone (vissm_elbo_fwd / vissm_elbo_bwd) at the configs' per-GPU shapes:
average launch time over ROUNDS x 20 launches (HIP events) and the fraction of 8 TB/s for the algorithmic bytes
(fwd reads z: 4 D (M+1) B; bwd reads z and writes dz: 8 D (M+1) B).  Prints one JSON line."""
import ctypes
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from viforssms_amd import _lib  # noqa: E402
from viforssms_amd.ops import ElboDesc, ElboFeeds, check, ptr  # noqa: E402

SHAPES = {"lv": (16384, 5000, 2), "sv": (16384, 1508, 1), "fhn": (8192, 2000, 2)}


def case(model, B, M, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g, device=dev)
    if model == "lv":
        z = 100 + 10 * r(B, 2 * (M + 1))
        th = torch.stack([math.log(0.5) + 0.1 * r(B), math.log(0.0025) + 0.1 * r(B), math.log(0.3) + 0.1 * r(B)], 1)
        mask = torch.ones(1, 2, M + 1, device=dev)
        shift = torch.zeros(1, 2, M + 1, device=dev)
        mask[0, :, 0] = 0
        shift[0, :, 0] = 100
        obs = 100 + 10 * r(1, 2, M)
        obn = (torch.rand(1, 2, M, generator=g, device=dev) < 0.01).float()
        return z, th, ElboFeeds(obs=obs, obs_bin=obn, mask=mask, shift=shift), _lib.MODEL_LV, 0.1
    if model == "sv":
        z = -8 + r(B, M + 1)
        th = torch.stack([0.001 + 0.01 * r(B), -0.6 + 0.1 * r(B), math.log(0.08) + 0.1 * r(B),
                          math.log(0.5) + 0.1 * r(B)], 1)
        mask = torch.ones(1, M + 1, device=dev)
        shift = torch.zeros(1, M + 1, device=dev)
        d1 = 2 + 14 * torch.rand(1, M + 1, generator=g, device=dev)
        return z, th, ElboFeeds(mask=mask, shift=shift, dim_one=d1), _lib.MODEL_SV, 1.0
    z = r(B, 2 * (M + 1))
    th = torch.stack([math.log(2) + 0.1 * r(B), 1 + 0.1 * r(B), 1.5 + 0.1 * r(B), math.log(0.5) + 0.1 * r(B),
                      math.log(0.3) + 0.1 * r(B)], 1)
    obs = r(1, 2, M)
    obn = (torch.rand(1, 2, M, generator=g, device=dev) < 0.1).float()
    return z, th, ElboFeeds(obs=obs, obs_bin=obn), _lib.MODEL_FHN, 0.1


def main():
    dev = torch.device("cuda", 0)
    rounds = int(os.environ.get("ROUNDS", "3"))
    out = {}
    for model in os.environ.get("MODELS", "lv,sv,fhn").split(","):
        B, M, D = SHAPES[model]
        z, th, feeds, mid, dt = case(model, B, M, dev)
        lib = _lib.load()
        d = ElboDesc(mid, B, M, 1, float(dt), 1.0)
        data = feeds.cdata()
        pdata = None
        if feeds.mask is not None:   # the same feeds with the plain-span table (VissmElboData.plain_from)
            from dataclasses import replace
            from viforssms_amd.features import plain_from_table
            mk, sh = feeds.mask[0].double().cpu().numpy(), feeds.shift[0].double().cpu().numpy()
            pf = torch.as_tensor(plain_from_table(mk, sh, M), device=dev)
            pfeeds = replace(feeds, plain_from=pf)
            pdata = pfeeds.cdata()
        st = _lib.stream_handle(dev)
        sde, obs, ex = (torch.empty(B, device=dev) for _ in range(3))
        gs = torch.ones(B, device=dev)
        dz, dth = torch.empty_like(z), torch.empty_like(th)
        calls = {
            "fwd": lambda: check(lib.vissm_elbo_fwd(ctypes.byref(d), ctypes.byref(data), ptr(z), ptr(th), ptr(sde),
                                                    ptr(obs), ptr(ex), st), "fwd"),
            "bwd": lambda: check(lib.vissm_elbo_bwd(ctypes.byref(d), ctypes.byref(data), ptr(z), ptr(th), ptr(gs),
                                                    ptr(gs), ptr(gs), ptr(dz), ptr(dth), st), "bwd"),
            # the training step's one pass (vissm_elbo_fwd_grad): values, dz and dtheta from one read of z
            "one": lambda: check(lib.vissm_elbo_fwd_grad(ctypes.byref(d), ctypes.byref(data), ptr(z), ptr(th),
                                                         ptr(gs), ptr(gs), ptr(gs), ptr(sde), ptr(obs), ptr(ex),
                                                         ptr(dz), ptr(dth), st), "one"),
            "one_plain": lambda: check(lib.vissm_elbo_fwd_grad(ctypes.byref(d), ctypes.byref(pdata), ptr(z), ptr(th),
                                                               ptr(gs), ptr(gs), ptr(gs), ptr(sde), ptr(obs), ptr(ex),
                                                               ptr(dz), ptr(dth), st), "one_plain"),
        }
        kinds = ["fwd", "bwd"] + (["one"] if hasattr(lib, "vissm_elbo_fwd_grad") else [])
        kinds += ["one_plain"] if pdata is not None and "one" in kinds else []
        ts = {k: [] for k in kinds}
        for _ in range(rounds):
            for kind in kinds:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                calls[kind]()
                torch.cuda.synchronize()
                s.record()
                for _ in range(20):
                    calls[kind]()
                e.record()
                torch.cuda.synchronize()
                ts[kind].append(s.elapsed_time(e) / 20)
        zb = 4.0 * D * (M + 1) * B
        f, b = min(ts["fwd"]), min(ts["bwd"])
        out[model] = {"fwd_ms": round(f, 4), "bwd_ms": round(b, 4), "fwd_frac": round(zb / (f * 1e-3) / 8e12, 3),
                      "bwd_frac": round(2 * zb / (b * 1e-3) / 8e12, 3), "check": [float(sde.double().sum()), float(dz.double().abs().sum())]}
        if "one" in ts:
            o = min(ts["one"])
            out[model].update(one_ms=round(o, 4), one_frac=round(2 * zb / (o * 1e-3) / 8e12, 3),
                              two_launch_ms=round(f + b, 4))
        if "one_plain" in ts:
            o = min(ts["one_plain"])
            out[model].update(one_plain_ms=round(o, 4), one_plain_frac=round(2 * zb / (o * 1e-3) / 8e12, 3))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
