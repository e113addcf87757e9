#!/bin/bash
# Round-6 session v: FHN-cfg kernel trace (library kernels left in its step) and the SV step's torch glue after the
# gradient hand-off change.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06v; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_fhn" -o fhn --output-format csv -- python "$ROOT/bench.py" --model fhn --steps 3 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/prof_fhn.log" 2>&1 || exit 4
cd "$ROOT" && timeout -k 10 300 python -u scripts/prof_glue.py --model sv > "$OUT/glue_sv_release.txt" 2> "$OUT/glue_sv_release.err" || exit 5
head -12 "$OUT/glue_sv_release.txt"; grep -c Cijk "$OUT/prof_fhn/fhn_kernel_stats.csv" || true
date
