#!/bin/bash
# Paper-shape fp32 recovery runs (scripts/ar_recovery.py, 10,000 ELBO steps after pre-training) over several Philox
# seeds of the eps / q(theta) base draws, for each theta-branch form: torch (library GEMMs), assoc (the torch form,
# collapsed weights associated the other way: a rounding-only change), 1 (the HIP theta-branch kernels).  Each run
# once, with optimiser / flow diagnostics every 250 steps.  SEEDS / MODES override the lists.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/recs; mkdir -p "$OUT"; export TMPDIR=/tmp
for s in ${SEEDS:-1 2 3 4}; do
  for mode in ${MODES:-torch assoc 1}; do
    unset VISSM_THETA_BRANCH_ASSOC; export VISSM_THETA_BRANCH_KERNEL=0
    if [ $mode = assoc ]; then export VISSM_THETA_BRANCH_ASSOC=1
    elif [ $mode != torch ]; then export VISSM_THETA_BRANCH_KERNEL=$mode; fi
    echo "== $mode seed $s"
    timeout -k 10 300 python3 scripts/ar_recovery.py --steps ${STEPS:-10000} --every 250 --seed $s --diag \
      > "$OUT/${mode}_s$s.log" 2>&1 || exit 3
    python3 -c "
import json
for l in open('$OUT/${mode}_s$s.log'):
    if l.startswith('{'):
        d=json.loads(l)
        if d['step'] % 1000 == 0: print(d['step'], [round(x,3) for x in d['mean']], [round(x,3) for x in d['sd']])"
  done
done
