#!/bin/bash
# dC slab groups padded to 8 elements + the 16-byte bf16 reduce: reduce / flow parity tests, then the AR-cfg step
# against the previous build (abl/lib_base.so), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_reduce.py tests/test_gpu_fused.py tests/test_gpu_config_parity.py tests/test_gpu_fullsize.py tests/test_gpu_pitch.py > "$OUT/pytest_red8.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_red8.log"; [ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash scripts/ab_step.sh abl/lib_red8.so abl/lib_base.so || exit 4
