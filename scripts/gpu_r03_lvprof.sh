#!/bin/bash
# LV-cfg step kernel breakdown (rocprofv3 kernel trace, full kernel names).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/lvprof" -o lv --output-format csv -- python3 "$ROOT/bench.py" --model lv --steps 4 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/lvprof.log" 2>&1 || { tail -5 "$OUT/lvprof.log"; exit 4; }
f=$(find "$OUT/lvprof" -name "*kernel_stats.csv" | head -1); python3 - "$f" << 'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 5e6
print("total per step (5 steps incl. warmup) %.2f ms" % tot)
for r in rows[:22]: print("%-100s %5s %8.3f ms/step" % (r["Name"][:100], r["Calls"], float(r["TotalDurationNs"]) / 5e6))
PY
