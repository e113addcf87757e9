#!/bin/bash
# The paper-shape recovery run (scripts/ar_recovery.py, fp32, 10,000 steps) with the theta-branch kernels opt-in
# (VISSM_THETA_BRANCH_KERNEL = 1: forward and backward kernels, the default from round 6; bwd: backward kernel only) and
# with the torch form (=0) (assoc: the torch form with the collapsed weights in the other association order, a rounding-only
# change): which direction moves the posterior sd, and how far rounding alone moves it.  MODES / RUNS override the lists.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/rec; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in ${RUNS:-1}; do
  for mode in ${MODES:-torch bwd 1}; do
    unset VISSM_THETA_BRANCH_ASSOC
    if [ $mode = torch ]; then export VISSM_THETA_BRANCH_KERNEL=0
    elif [ $mode = assoc ]; then export VISSM_THETA_BRANCH_KERNEL=0; export VISSM_THETA_BRANCH_ASSOC=1
    else export VISSM_THETA_BRANCH_KERNEL=$mode; fi
    echo "== $mode run $r"
    timeout -k 10 200 python3 scripts/ar_recovery.py --steps 10000 --every 1000 > "$OUT/${mode}_$r.log" 2>&1 || exit 3
    python3 -c "
import json
for l in open('$OUT/${mode}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['step'], [round(x,3) for x in d['mean']], [round(x,3) for x in d['sd']])"
  done
done
