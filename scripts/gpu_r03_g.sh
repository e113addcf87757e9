#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== fwd2 parity"; date
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_config_parity.py tests/test_gpu_parity.py > "$OUT/r03_g_tests.log" 2>&1
rc=$?; tail -3 "$OUT/r03_g_tests.log"; [ $rc -le 1 ] || exit $rc
echo "== A/B"; date
bash scripts/ab_step.sh || exit $?
