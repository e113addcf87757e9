#!/bin/bash
# Round validation of the current tree: parity tests + smoke + full bench + rocprofv3 kernel
# trace + the two HBM-traffic PMC passes (scripts/gpu_round.sh), then the per-model bench lines.
# Each GPU step has its own limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
bash scripts/gpu_round.sh || exit $?
for m in lv sv fhn; do
  echo "== bench $m"
  timeout -k 10 300 python bench.py --model $m --steps 3 --warmup 1 --cpu-baseline off > "$OUT/bench_$m.log" 2>&1 || { tail -5 "$OUT/bench_$m.log"; exit 6; }
  tail -1 "$OUT/bench_$m.log" | cut -c1-300
done
