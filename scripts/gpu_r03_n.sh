#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_elbo_models.py tests/test_gpu_parity.py -k "elbo or lv" > "$OUT/r03_n_tests.log" 2>&1 || { tail -20 "$OUT/r03_n_tests.log"; exit 3; }; tail -1 "$OUT/r03_n_tests.log"
for r in 1 2; do for v in base bf; do
  echo -n "$v "; VISSM_LIB=$ROOT/abl/lib_$v.so ROUNDS=3 timeout -k 10 120 python -u scripts/elbo_models_bench.py || exit 4
done; done
