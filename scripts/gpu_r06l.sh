#!/bin/bash
# Round-6 session l: the bf16 GEMM with K steps of 64 (VISSM_GEMM_BK=64: half the barriers, 2 blocks per CU) against 32:
# GEMM / LV-branch parity with it, then the LV step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06l; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
VISSM_LIB=$ROOT/abl/lib_bk64.so timeout -k 10 300 $PT tests/test_gpu_lvfeat.py > "$OUT/pytest_bk64.log" 2>&1; rc=$?
tail -n 2 "$OUT/pytest_bk64.log"; [ $rc -eq 0 ] || exit $rc
OUT=$OUT ROUNDS=2 STEPS=6 EXTRA="--model lv" bash scripts/ab_step.sh abl/lib_cur.so abl/lib_bk64.so
date
