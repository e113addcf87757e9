"""Parity of the bf16 / bf16x3 flow kernels against the float64 oracle (AR cases)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.parity_util import run_parity_case

CASES = [
    dict(family="lv", B=4, M=24, k=4, n_flows=2, H=16, n_layers=5, fw=3),
    dict(family="lv", B=3, M=50, k=20, n_flows=3, H=50, n_layers=5, fw=10),
    dict(family="sv", B=4, M=24, k=6, n_flows=2, H=16, n_layers=5, fw=3),
    dict(family="sv", B=3, M=52, k=50, n_flows=5, H=50, n_layers=5, fw=5),
    dict(family="fhn", B=3, M=50, k=20, n_flows=3, H=50, n_layers=5, fw=10),
    dict(family="fhn", B=5, M=40, k=6, n_flows=2, H=24, n_layers=5, fw=3, T=160, starts=[120, 0, 40, 40, 80]),
    dict(family="ar", B=4, M=24, k=4, n_flows=2, H=16, n_layers=3, fw=3),
    dict(family="ar", B=40, M=30, k=8, n_flows=3, H=50, n_layers=3, fw=10),
    dict(family="ar", B=3, M=50, k=50, n_flows=3, H=50, n_layers=3, fw=10),
    dict(family="ar", B=6, M=50, k=10, n_flows=3, H=32, n_layers=3, fw=10, T=300, starts=[0, 50, 100, 100, 250, 0]),
]
for c in CASES:
    for prec in ((1, 2) if c["family"] == "ar" else (1,)):
        try:
            r = run_parity_case(**c, device="cuda:0", precision=prec)
            print(json.dumps({"case": {k: v for k, v in c.items() if k != "starts"}, "prec": prec,
                              "elbo": r["elbo_rel_err"], "grad": r["grad_rel_err"], "worst": r["worst_param"],
                              "worst_err": r["grad_max_param_err"], "finite": r["finite"]}), flush=True)
        except Exception as e:  # noqa
            print(json.dumps({"case": c.get("k"), "prec": prec, "error": str(e)[:300]}), flush=True)
