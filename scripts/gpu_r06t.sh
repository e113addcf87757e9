#!/bin/bash
# Round-6 session t: the gradient hand-off without per-variable adds (ParamStore.release_grads, VISSM_GRAD_RELEASE):
# the driver's GPU test command, then SV / LV / AR steps with it on and off (alternating).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06t; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_driver.log" 2>&1; rc=$?
tail -n 2 "$OUT/pytest_driver.log"; [ $rc -eq 0 ] || exit $rc
for m in sv lv ar; do for r in 1 2; do for rel in 0 1; do
  VISSM_GRAD_RELEASE=$rel timeout -k 10 300 python -u bench.py --model $m --steps 8 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/bench_${m}_rel${rel}_$r.json" 2> "$OUT/bench_${m}_rel${rel}_$r.err" || exit 5
  python -c "import json; print('$m release $rel', round(json.loads(open('$OUT/bench_${m}_rel${rel}_$r.json').read().strip().splitlines()[-1])['ms_per_step'], 2))"
done; done; done
date
