import sys, json
sys.path.insert(0, ".")
from tests.parity_util import run_parity_case
from viforssms_amd import _lib
for prec in (1, _lib.VISSM_PREC_BF16X2F, 2):
    for sp in (False, True):
        for seed in (3, 4, 5):
            r = run_parity_case("ar", 6, 30, 5, 2, 20, 3, 4, device="cuda:0", T=150, starts=[0, 30, 60, 60, 120, 0],
                                precision=prec, step_path=sp, seed=seed)
            print(prec, sp, seed, r["fused"], "%.2e" % r["elbo_rel_err"], "%.2e" % r["grad_rel_err"], flush=True)
