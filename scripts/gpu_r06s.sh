#!/bin/bash
# Round-6 session s: where the step's small torch kernels come from (scripts/prof_glue.py) for SV, LV and AR.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06s; mkdir -p "$OUT"; export TMPDIR=/tmp
for m in sv lv ar; do
  timeout -k 10 300 python -u scripts/prof_glue.py --model $m > "$OUT/glue_$m.txt" 2> "$OUT/glue_$m.err" || { tail -20 "$OUT/glue_$m.err"; exit 4; }
  head -12 "$OUT/glue_$m.txt"
done
date
