#!/bin/bash
# Round GPU session: parity tests, smoke, full bench (with CPU baseline), rocprofv3 kernel-trace
# summary of the bench, and the two HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs).
# Each GPU step has its own limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
fault() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping: rc=$rc"; exit "$rc"; fi; }
SKIP_TESTS=${SKIP_TESTS:-0}
if [ "$SKIP_TESTS" = 0 ]; then
echo "== pytest -m gpu"; date
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
tail -4 "$OUT/pytest_gpu.log"; fault $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
tail -2 "$OUT/smoke.log"; fault $rc
fi
echo "== bench full"; date
timeout -k 10 900 python bench.py $BENCH_ARGS > "$OUT/bench_full.log" 2>&1 || { tail -20 "$OUT/bench_full.log"; exit 3; }
tail -1 "$OUT/bench_full.log"
echo "== rocprofv3 kernel trace"; date
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o bench --output-format csv -- python "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-baseline off --parity-line off --families off $BENCH_ARGS > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 4; }
tail -1 "$OUT/prof.log"
for C in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $C"; date
  cd /tmp && timeout -k 10 900 rocprofv3 --pmc $C --kernel-trace --stats -T --kernel-include-regex "bwd" -d "$OUT/pmc_$C" -o pmc --output-format csv -- python "$ROOT/bench.py" --steps 1 --warmup 0 --cpu-baseline off --parity-line off --families off $BENCH_ARGS > "$OUT/pmc_$C.log" 2>&1 || { tail -20 "$OUT/pmc_$C.log"; exit 5; }
done
date
cd "$ROOT" && python scripts/traffic_from_pmc.py ${PREC:-bf16} 65536 5000 8
