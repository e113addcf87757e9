#!/bin/bash
# Quick GPU iteration: the GPU tests (or a subset via TESTS=...), then one bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== pytest ${TESTS:-tests}"
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -15 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
echo "== bench"
timeout -k 10 600 python bench.py --cpu-baseline off $BENCH_ARGS > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 3; }
tail -1 "$OUT/bench.log"
