#!/bin/bash
# The driver's GPU test command (scripts/gpu_driver_suite.sh), then smoke(); a fault / abort / time limit ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
bash scripts/gpu_driver_suite.sh; rc=$?
[ $rc -eq 0 ] || { echo "stopping: suite rc=$rc"; exit $rc; }
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
tail -3 "$OUT/smoke.log"; exit $rc
