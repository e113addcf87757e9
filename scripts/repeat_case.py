"""Run one bf16 parity case twice in one process under VISSM_LIB and report whether the gradients are bitwise equal
(a race shows as run-to-run differences) and their errors against the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.parity_util import run_parity_case  # noqa: E402

args = tuple(int(a) if a.isdigit() else a for a in sys.argv[1].split(","))
r1 = run_parity_case(*args, device="cuda:0", precision=1)
r2 = run_parity_case(*args, device="cuda:0", precision=1)
k = [x for x in r1 if x.startswith("grad") or x.startswith("elbo")]
print(os.environ.get("VISSM_LIB", "tree").split("/")[-1], args, {x: r1[x] for x in k if not isinstance(r1[x], dict)},
      "same errors twice:", all(r1[x] == r2[x] for x in k if not isinstance(r1[x], dict)), flush=True)
