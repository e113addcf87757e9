"""Per-sample ELBO and gradient error of each training precision against the float64 oracle at one AR shape
(default the AR-cfg length, B = 20, bench chunk geometry): which products limit the gradient.
usage: python scripts/grad_err_modes.py [M] [modes...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.parity_util import run_parity_case  # noqa: E402
from viforssms_amd._lib import TRAIN_PRECISIONS as PREC  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
modes = sys.argv[2:] or ["bf16", "bf16x2f", "bf16x3f", "bf16x3", "fp32"]
for m in modes:
    for step in (False, True):
        if step and m == "fp32":
            continue
        r = run_parity_case("ar", 20, M, 8, 3, 50, 3, 10, device="cuda:0", precision=PREC[m], impute=5, condition=True,
                            step_path=step, chunk_tiles=167 if M == 5000 else 0)
        per = sorted(r["per_param"].items(), key=lambda kv: -kv[1])[:4]
        print(json.dumps({"mode": m, "step_path": step, "fused": r["fused"], "elbo": r["elbo_rel_err"],
                          "grad": r["grad_rel_err"], "worst": per}), flush=True)
