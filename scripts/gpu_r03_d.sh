#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== A/B"; date
bash scripts/ab_step.sh || exit $?
echo "== pmc bwd2"; date
TAG=r03_bwd2_pmc IMPL=bf16 B=16384 bash scripts/gpu_pmc.sh > "$OUT/r03_bwd2_pmc.txt" 2>&1 || { tail -5 "$OUT/r03_bwd2_pmc.txt"; exit 3; }
tail -40 "$OUT/r03_bwd2_pmc.txt"
echo "== posterior"; date
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_posterior.py > "$OUT/r03_posterior.log" 2>&1
rc=$?; grep -E "worst|passed|failed" "$OUT/r03_posterior.log" | tail -5
date
