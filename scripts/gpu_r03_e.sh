#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== A/B"; date
bash scripts/ab_step.sh || exit $?
echo "== pmc bwd2"; date
TAG=r03_bwd2_pmc IMPL=bf16 B=16384 bash scripts/gpu_pmc.sh > "$OUT/r03_bwd2_pmc.txt" 2>&1 || { tail -5 "$OUT/r03_bwd2_pmc.txt"; exit 3; }
grep -A40 bwd2 "$OUT/r03_bwd2_pmc.txt" | head -42
echo "== posterior bf16x2f"; date
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_posterior.py::test_ar_posterior_trajectory_matches_oracle[bf16x2f]" > "$OUT/r03_posterior_x2.log" 2>&1
grep -E "^step|worst|passed|failed" "$OUT/r03_posterior_x2.log" | tail -25
echo "== pmc elbo"; date
bash scripts/gpu_pmc_elbo.sh > "$OUT/r03_elbo_pmc.txt" 2>&1; tail -60 "$OUT/r03_elbo_pmc.txt"
date
