"""Runs parity cases against the oracle with each flow implementation (A/B on correctness)."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.parity_util import run_parity_case
from viforssms_amd import _lib

CASES = [
    dict(family="lv", B=3, M=50, k=20, n_flows=3, H=50, n_layers=5, fw=10),
    dict(family="lv", B=3, M=50, k=20, n_flows=3, H=16, n_layers=5, fw=10),
    dict(family="lv", B=5, M=40, k=6, n_flows=2, H=24, n_layers=5, fw=3, T=160, starts=[0, 40, 80, 80, 120]),
    dict(family="sv", B=4, M=40, k=8, n_flows=2, H=24, n_layers=5, fw=3, T=160, starts=[0, 40, 120, 40]),
    dict(family="ar", B=6, M=50, k=10, n_flows=3, H=32, n_layers=3, fw=10, T=300, starts=[0, 50, 100, 100, 250, 0]),
]
lib = _lib.load()
impls = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4").split(",")]
for c in CASES:
    for im in impls:
        lib.vissm_flow_set_impl(im)
        r = run_parity_case(**c, device="cuda:0")
        print(json.dumps({"case": {k: v for k, v in c.items() if k != "starts"}, "impl": im,
                          "elbo": r["elbo_rel_err"], "grad": r["grad_rel_err"], "worst": r["worst_param"],
                          "worst_err": r["grad_max_param_err"], "finite": r["finite"],
                          "elbo_mean": r["elbo_ref_mean"]}), flush=True)
