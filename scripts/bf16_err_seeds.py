"""bf16 rounding error against the float64 oracle over several seeds (AR-cfg flow shape):
separates a systematic change of a kernel's numerics from the rounding lottery of one seed.
Library under test: VISSM_LIB (default: the in-tree build)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.parity_util import run_parity_case

prec = int(sys.argv[1]) if len(sys.argv) > 1 else 1
e, g = [], []
for seed in range(1, 9):
    r = run_parity_case("ar", 40, 30, 8, 3, 50, 3, 10, device="cuda:0", precision=prec, seed=seed)
    e.append(r["elbo_rel_err"])
    g.append(r["grad_rel_err"])
print(json.dumps({"lib": os.environ.get("VISSM_LIB", "in-tree"), "prec": prec, "elbo_rel_err": e,
                  "elbo_mean": float(np.mean(e)), "grad_mean": float(np.mean(g)), "grad_max": float(np.max(g))}))
