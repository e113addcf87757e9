#!/bin/bash
# Round-6 session m: the bf16 slab reduction (dC partials) with 8 / 16 / 32 rows in flight per thread
# (VISSM_REDUCE_DEPTH): its bit-exactness test, then the AR-cfg step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06m; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
VISSM_LIB=$ROOT/abl/lib_red32.so timeout -k 10 300 $PT tests/test_gpu_reduce.py > "$OUT/pytest_red32.log" 2>&1; rc=$?
tail -n 1 "$OUT/pytest_red32.log"; [ $rc -eq 0 ] || exit $rc
OUT=$OUT ROUNDS=2 STEPS=10 bash scripts/ab_step.sh abl/lib_cur.so abl/lib_red16.so abl/lib_red32.so
cd /tmp && for L in cur red32; do VISSM_LIB=$ROOT/abl/lib_$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_$L" -o ar --output-format csv -- python "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/prof_$L.log" 2>&1 || exit 4; grep -h reduce_rows_bf16 "$OUT/prof_$L/ar_kernel_stats.csv" | cut -d, -f1-4; done
date
