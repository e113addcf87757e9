#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
for m in lv sv; do
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$m" -o $m --output-format csv -- python3 "$ROOT/bench.py" --model $m --steps 4 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/prof_$m.log" 2>&1 || exit 4
f=$(find "$OUT/prof_$m" -name "*kernel_stats.csv" | head -1); python3 - "$f" << 'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 5e6
print("total per step (5 steps incl. warmup) %.2f ms" % tot)
for r in rows[:14]: print("%-60s %5s %8.3f ms/step" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"]) / 5e6))
PY
done
