#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== bwd2n parity (lv / fhn / sv / loop / dist / golden)"; date
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_config_parity.py tests/test_gpu_golden.py tests/test_gpu_loop.py \
  tests/test_gpu_dist.py tests/test_gpu_graph.py > "$OUT/r03_h_tests.log" 2>&1
rc=$?; tail -5 "$OUT/r03_h_tests.log"; [ $rc -le 1 ] || exit $rc
echo "== A/B lv"; date
EXTRA="--model lv" STEPS=5 bash scripts/ab_step.sh || exit $?
echo "== A/B fhn"; date
EXTRA="--model fhn" STEPS=5 bash scripts/ab_step.sh || exit $?
