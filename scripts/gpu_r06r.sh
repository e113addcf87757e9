#!/bin/bash
# Round-6 session r: LV GEMM split-K, third pass -- (VISSM_LV_SPLIT for G / dWc, VISSM_LV_SPLIT_W3 for dW3 / dH3)
# at (5, 8) (5, 16) (6, 16) (4, 16); the LV feature tests at (6, 16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06r; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
VISSM_LV_SPLIT=6 VISSM_LV_SPLIT_W3=16 timeout -k 10 300 $PT tests/test_gpu_lvfeat.py > "$OUT/pytest_split616.log" 2>&1; rc=$?
tail -n 1 "$OUT/pytest_split616.log"; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --model lv --steps 8 --warmup 2 --cpu-baseline off --parity-line off --families off"
for r in 1 2; do for cfg in 5:8 5:16 6:16 4:16; do
  a=${cfg%:*}; b=${cfg#*:}
  VISSM_LV_SPLIT=$a VISSM_LV_SPLIT_W3=$b timeout -k 10 300 $B > "$OUT/bench_${a}_${b}_$r.json" 2> "$OUT/bench_${a}_${b}_$r.err" || exit 5
  python -c "import json; print('split $a $b', round(json.loads(open('$OUT/bench_${a}_${b}_$r.json').read().strip().splitlines()[-1])['ms_per_step'], 2))"
done; done
date
