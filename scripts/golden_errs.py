"""Errors of the HIP path against the committed oracle golden vectors, per case and precision."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.golden_util import cases
from tests.test_gpu_golden import _run

for name in cases():
    for prec in (0, 2, 1):
        elbo, er, g, gr = _run(name, prec)
        print(json.dumps({"case": name, "prec": prec, "elbo_max_rel": float(np.max(np.abs(elbo - er) / np.abs(er))),
                          "grad_rel_l2": float(np.linalg.norm(g - gr) / np.linalg.norm(gr))}), flush=True)
