"""Loader of the committed oracle golden vectors (tests/golden/oracle_cases.npz, written by
tests/golden/make_oracle_fixtures.py)."""
import os

import numpy as np
import torch

from tests.parity_util import build_model

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PATHS = [os.path.join(GOLDEN, "oracle_cases.npz"), os.path.join(GOLDEN, "oracle_cases_cfg.npz")]


def _file_of(name: str) -> str:
    for p in PATHS:
        if name in [str(n) for n in np.load(p)["names"]]:
            return p
    raise KeyError(name)


def cases():
    return [str(n) for p in PATHS for n in np.load(p)["names"]]


def load_case(name: str, device: str, precision: int = 0):
    """The case's model (fixture parameters loaded), batch, eps, x0 and expected outputs."""
    d = np.load(_file_of(name))
    g = lambda k: d[f"{name}/{k}"]
    cfg = [int(x) for x in g("cfg")]
    B, M, k, nf, H, nl, fw, T = cfg[:8]
    impute, condition = (cfg[8], bool(cfg[9])) if len(cfg) > 8 else (0, False)
    model = build_model(str(g("family")), B, M, k, nf, H, nl, fw, device, T=None if T < 0 else T,
                        precision=precision, seed=3, impute=impute or None, condition=condition)
    with torch.no_grad():
        model.store.flat.copy_(torch.as_tensor(g("flat"), device=model.store.flat.device))
    batch = model.engine.make_batch(g("starts"))
    eps = torch.as_tensor(g("eps").astype(np.float64))
    x0 = torch.as_tensor(g("x0").astype(np.float64))
    return model, batch, eps, x0, g("elbo"), g("grad").astype(np.float64)
