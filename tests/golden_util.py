"""Loader of the committed oracle golden vectors (tests/golden/oracle_cases.npz, written by
tests/golden/make_oracle_fixtures.py)."""
import os

import numpy as np
import torch

from tests.parity_util import build_model

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_cases.npz")


def cases():
    d = np.load(PATH)
    return [str(n) for n in d["names"]]


def load_case(name: str, device: str, precision: int = 0):
    """The case's model (fixture parameters loaded), batch, eps, x0 and expected outputs."""
    d = np.load(PATH)
    g = lambda k: d[f"{name}/{k}"]
    B, M, k, nf, H, nl, fw, T = (int(x) for x in g("cfg"))
    model = build_model(str(g("family")), B, M, k, nf, H, nl, fw, device, T=None if T < 0 else T,
                        precision=precision, seed=3)
    with torch.no_grad():
        model.store.flat.copy_(torch.as_tensor(g("flat"), device=model.store.flat.device))
    batch = model.engine.make_batch(g("starts"))
    eps = torch.as_tensor(g("eps").astype(np.float64))
    x0 = torch.as_tensor(g("x0").astype(np.float64))
    return model, batch, eps, x0, g("elbo"), g("grad").astype(np.float64)
