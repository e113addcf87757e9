#!/bin/bash
# Kernel trace of the LV-cfg step (bench.py --model lv): where the step's time goes outside the flow kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/prof_lv; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o lv --output-format csv -- python3 "$ROOT/bench.py" --model lv --steps 3 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/prof.log" 2>&1; rc=$?
head -25 "$OUT/lv_kernel_stats.csv" | cut -c1-160
exit $rc
