"""The rounding model the reduced-precision modes' GPU tolerances derive from (oracle/precision_model.py), on the
CPU: exact mode == the plain oracle, the modes' error ordering at the AR-cfg flow shape, and the committed
trajectory envelope (tests/golden/precision_drift.json) reproduced by its generator for the first steps."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import nma_oracle as O
from oracle.precision_model import emulate
from tests.parity_util import build_model, oracle_reference

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _case(B=6, M=40, k=8):
    m = build_model("ar", B, M, k, 3, 50, 3, 10, "cpu")
    md = m.mdef
    batch = m.engine.make_batch(np.zeros(B, dtype=np.int64))
    g = torch.Generator().manual_seed(14)
    eps = torch.randn(B, md.kernel_ext, generator=g, dtype=torch.float64)
    x0 = torch.randn(B, md.P_theta, generator=g, dtype=torch.float64) * md.theta_base[1] + md.theta_base[0]
    return m, batch, eps, x0


def _errs(ref, em):
    (e, gr), (e2, g2) = ref, em
    a = np.concatenate([gr[n].ravel() for n in gr])
    b = np.concatenate([g2[n].ravel() for n in gr])
    return float(np.max(np.abs(e2 - e) / np.abs(e))), float(np.linalg.norm(b - a) / np.linalg.norm(a))


def test_emulation_modes():
    m, batch, eps, x0 = _case()
    ref = oracle_reference(m, batch, eps, x0)
    with emulate(None):
        assert _errs(ref, oracle_reference(m, batch, eps, x0)) == (0.0, 0.0)
    assert O.iaf_flow.__name__ == "iaf_flow"            # restored on exit
    errs = {}
    for mode in ("bf16", "bf16x2f", "bf16x2"):
        with emulate(mode):
            errs[mode] = _errs(ref, oracle_reference(m, batch, eps, x0))
    print(errs)
    # split weights remove the weights' coherent rounding from the forward (ELBO) and the chain (gradient)
    assert errs["bf16x2f"][0] < errs["bf16"][0] and errs["bf16x2"][0] == errs["bf16x2f"][0]
    assert errs["bf16x2"][1] < errs["bf16x2f"][1] < errs["bf16"][1]
    assert all(0 < e < 2e-2 for v in errs.values() for e in v)
    # a scaled-domain realisation moves the errors, not their scale
    with emulate("bf16", realisation=1):
        ej = _errs(ref, oracle_reference(m, batch, eps, x0))
    assert ej != errs["bf16"] and 0.5 < ej[1] / errs["bf16"][1] < 2.0


def test_precision_drift_fixture_reproduces():
    """The first two steps of the committed fixture's plain realisation, regenerated
    (scripts/precision_drift_emul.py); the envelope is the maximum over the realisations."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import precision_drift_emul as P
    fix = json.load(open(os.path.join(ROOT, "tests", "golden", "precision_drift.json")))
    assert fix["K"] >= 20 and set(fix["modes"]) == {"bf16", "bf16x2f", "bf16x2"}
    res = P.run(K=2, realisations=1)
    for mode, reals in res["per_realisation"].items():
        for s in range(2):
            for key in ("dmean", "dsd", "elbo"):
                got, want = reals[0][s][key], fix["per_realisation"][mode][0][s][key]
                assert got == pytest.approx(want, rel=1e-6, abs=1e-12), (mode, s, key)
                assert fix["modes"][mode][s][key] == max(r[s][key] for r in fix["per_realisation"][mode])
