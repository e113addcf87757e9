#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== bwd2n parity"; date
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_config_parity.py tests/test_gpu_golden.py tests/test_gpu_loop.py > "$OUT/r03_i_tests.log" 2>&1
rc=$?; tail -3 "$OUT/r03_i_tests.log"; [ $rc -le 1 ] || exit $rc
echo "== A/B lv"; date
EXTRA="--model lv" STEPS=5 bash scripts/ab_step.sh || exit $?
echo "== rocprof lv step"; date
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/r03_prof_lv" -o lv --output-format csv -- python "$ROOT/bench.py" --model lv --steps 3 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/r03_prof_lv.log" 2>&1 || { tail -5 "$OUT/r03_prof_lv.log"; exit 4; }
cd "$ROOT"; head -25 $(find "$OUT/r03_prof_lv" -name "*kernel_stats.csv" | head -1) | cut -c1-160
