#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
VISSM_LIB=$ROOT/abl/lib_lag.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_config_parity.py tests/test_gpu_fused.py -k "ar or fused" > "$OUT/r03_p_tests.log" 2>&1
rc=$?; tail -2 "$OUT/r03_p_tests.log"; [ $rc -eq 0 ] || exit 3
ROUNDS=2 STEPS=6 bash scripts/ab_step.sh
