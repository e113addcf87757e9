#!/bin/bash
# bench.py on each model config (1 GPU); small steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for M in ${MODELS:-sv fhn lv}; do
  echo "== $M"
  timeout -k 10 600 python bench.py --model $M --steps ${STEPS:-3} --warmup 1 --cpu-baseline off $EXTRA > $OUT/bench_$M.log 2>&1 || { tail -20 $OUT/bench_$M.log; exit 3; }
  tail -1 $OUT/bench_$M.log | cut -c1-900
done
