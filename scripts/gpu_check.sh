#!/bin/bash
# One GPU session: parity tests, smoke, bench (small then full), rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_on_fault() {  # pytest returns 1 for test failures; anything else (crash, timeout) stops the run
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping: rc=$rc"; exit "$rc"; fi
}
echo "== pytest -m gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"; stop_on_fault $rc
echo "== smoke"; date
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -3 "$OUT/smoke.log"; stop_on_fault $rc
echo "== bench small"; date
timeout -k 10 300 python bench.py --B 4096 --steps 3 --warmup 1 --cpu-baseline off > "$OUT/bench_small.log" 2>&1 || { tail -20 "$OUT/bench_small.log"; exit 3; }
tail -1 "$OUT/bench_small.log"
echo "== bench full"; date
timeout -k 10 900 python bench.py > "$OUT/bench_full.log" 2>&1 || { tail -20 "$OUT/bench_full.log"; exit 4; }
tail -1 "$OUT/bench_full.log"
echo "== rocprofv3 kernel trace"; date
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o bench --output-format csv -- python "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-baseline off > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 5; }
tail -1 "$OUT/prof.log"
find "$OUT/prof" -name "*stats*" | head
date
