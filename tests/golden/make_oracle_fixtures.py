"""Generates tests/golden/oracle_cases.npz: committed golden vectors of the float64 oracle
(oracle/nma_oracle.py) for small cases of the four families — inputs (flat parameters, window
starts, injected eps and q(theta) base draws) and outputs (per-sample ELBO, d sum(-ELBO) / d flat
parameters).  tests/test_golden.py pins the oracle to them on the CPU; tests/test_gpu_golden.py
checks the HIP path against them.  Run from the repo root: python tests/golden/make_oracle_fixtures.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tests.parity_util import build_model, oracle_reference  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "oracle_cases.npz")
OUT_CFG = os.path.join(HERE, "oracle_cases_cfg.npz")
# name: (family, B, M, k, n_flows, H, n_layers, fw, T, starts)
CASES = {
    "ar_small": ("ar", 5, 24, 4, 2, 16, 3, 3, None, None),
    "ar_cfg_shape": ("ar", 4, 30, 8, 1, 50, 3, 10, None, None),  # the AR-cfg flow shape, one flow
    "ar_windows": ("ar", 6, 50, 10, 3, 32, 3, 10, 300, [0, 50, 100, 100, 250, 0]),
    "lv_small": ("lv", 4, 24, 4, 2, 16, 5, 3, None, None),
    "sv_small": ("sv", 4, 24, 6, 2, 16, 5, 3, None, None),
    "fhn_small": ("fhn", 4, 40, 6, 2, 24, 5, 3, 160, [120, 0, 40, 80]),
}
# BASELINE configs[1] at its own length (AR(1) T = M = 5000, impute 5, kernel_len 8, 3 flows, [50]*3),
# conditioned parameter draw (parity_util.build_model(condition=True)); a file of its own (~1 MB)
CFG_CASES = {
    "ar_cfg_length": ("ar", 4, 5000, 8, 3, 50, 3, 10, None, None),
}
CFG_OPTS = {"ar_cfg_length": dict(impute=5, condition=True)}


def case_arrays(name, cfg, seed=3):
    family, B, M, k, nf, H, nl, fw, T, starts = cfg
    opts = CFG_OPTS.get(name, {})
    model = build_model(family, B, M, k, nf, H, nl, fw, "cpu", T=T, seed=seed, **opts)
    md = model.mdef
    starts = np.zeros(B, dtype=np.int64) if starts is None else np.asarray(starts, dtype=np.int64)
    batch = model.engine.make_batch(starts)
    g = torch.Generator().manual_seed(seed + 11)
    # fp32-representable draws (stored as fp32; the GPU path consumes fp32)
    eps = torch.randn(B, md.kernel_ext, generator=g, dtype=torch.float64).float().double()
    x0 = (torch.randn(B, md.P_theta, generator=g, dtype=torch.float64) * md.theta_base[1]
          + md.theta_base[0]).float().double()
    elbo, grads = oracle_reference(model, batch, eps, x0)
    st = model.store
    gflat = np.concatenate([np.asarray(grads[n], dtype=np.float64).ravel() for n in st.names()])
    pre = name + "/"
    return {pre + "cfg": np.array([B, M, k, nf, H, nl, fw, -1 if T is None else T, opts.get("impute", 0),
                                   int(opts.get("condition", False))], dtype=np.int64),
            pre + "family": np.array(family), pre + "starts": starts,
            pre + "flat": st.flat.detach().cpu().numpy().astype(np.float32),
            pre + "eps": eps.numpy().astype(np.float32), pre + "x0": x0.numpy().astype(np.float32),
            pre + "elbo": elbo, pre + "grad": gflat.astype(np.float32)}


def write(path, cases):
    arrs = {}
    for name, cfg in cases.items():
        arrs.update(case_arrays(name, cfg))
    np.savez_compressed(path, names=np.array(list(cases)), **arrs)
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    which = sys.argv[1:] or ["small", "cfg"]
    if "small" in which:
        write(OUT, CASES)
    if "cfg" in which:
        write(OUT_CFG, CFG_CASES)


if __name__ == "__main__":
    main()
