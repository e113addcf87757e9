"""Per-parameter gradient errors of the bf16 family parity cases (tests/test_gpu_parity.py) under the library named by
VISSM_LIB (A/B of kernel builds): python scripts/sv_case_errs.py sv|lvfhn|sv50 [--all]  (--all: every variable's error)"""
import os, sys, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from tests.parity_util import run_parity_case
CASES = {"sv": [("sv", 3, 52, 50, 5, 50, 5, 5), ("sv", 4, 80, 64, 2, 50, 5, 5), ("sv", 5, 60, 33, 2, 50, 5, 5),
                ("sv", 20, 1508, 50, 5, 50, 5, 5)],
         "lvfhn": [("lv", 3, 50, 20, 3, 50, 5, 10), ("fhn", 3, 50, 20, 3, 50, 5, 10), ("lv", 5, 40, 24, 2, 32, 5, 3),
                   ("lv", 4, 24, 4, 2, 16, 5, 3), ("fhn", 20, 2000, 20, 3, 50, 5, 10)],
         "sv50": [("sv", 3, 52, 50, 5, 50, 5, 5), ("sv", 3, 52, 50, 1, 50, 5, 5)]}
for args in CASES[sys.argv[1] if len(sys.argv) > 1 else "sv"]:
    res = run_parity_case(*args, device="cuda:0", precision=1, condition=args[2] > 1000)
    pp = res.get("per_param", {})
    top = sorted(pp.items(), key=lambda kv: -kv[1])[:None if "--all" in sys.argv else 4] if isinstance(pp, dict) else None
    print(os.environ.get("VISSM_LIB", "tree").split("/")[-1], args, {k: (round(v, 5) if isinstance(v, float) else v) for k, v in res.items() if k in ("elbo_rel_err", "grad_rel_err", "grad_max_param_err", "worst_param")}, top, flush=True)
