"""ELBO / gradient error of each training precision against the float64 oracle on one parity case (default: the
several-window AR case of tests/test_gpu_parity.py).  usage: python scripts/case_prec_errs.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.parity_util import run_parity_case  # noqa: E402
from viforssms_amd._lib import TRAIN_PRECISIONS as PREC  # noqa: E402

starts = [0, 50, 100, 100, 250, 0]
for seed in (3, 4, 5):
    for m in ("bf16", "bf16x2f", "bf16x2", "bf16x3", "fp32"):
        r = run_parity_case("ar", 6, 50, 10, 3, 32, 3, 10, device="cuda:0", T=300, starts=starts, precision=PREC[m],
                            seed=seed)
        per = sorted(r["per_param"].items(), key=lambda kv: -kv[1])[:3]
        print(json.dumps({"seed": seed, "mode": m, "elbo": r["elbo_rel_err"], "grad": r["grad_rel_err"],
                          "worst": per}), flush=True)
