#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
VISSM_LIB=$ROOT/abl/lib_both.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_fused.py tests/test_gpu_config_parity.py tests/test_gpu_fullsize.py -k "fused or ar_cfg or fullsize or full" > "$OUT/r03_v_tests.log" 2>&1
rc=$?; tail -1 "$OUT/r03_v_tests.log"; [ $rc -eq 0 ] || { tail -30 "$OUT/r03_v_tests.log"; exit 3; }
ROUNDS=2 STEPS=5 bash scripts/ab_step.sh
