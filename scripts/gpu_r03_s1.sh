#!/bin/bash
# Round-3 session c, first call: GPU suite on the rebuilt tree, then the feature-GEMM A/B (gpu_r03_z.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/s1_pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/s1_pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_r03_z.sh
