#!/bin/bash
# The 20-step posterior trajectories of the reduced modes with the float32 oracle run beside them (the fp32 case's
# yardstick printed per step), for the tolerance analysis of DESIGN.md §5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/traj; mkdir -p "$OUT"; export TMPDIR=/tmp
VISSM_TRAJ_FP32_YARDSTICK=1 timeout -k 10 900 python3 -m pytest tests/test_gpu_posterior.py -k "trajectory and (bf16x2 or bf16)" -s -q -p no:cacheprovider > "$OUT/traj.log" 2>&1; rc=$?
grep -E "step|worst|passed|failed|Error" "$OUT/traj.log" | tail -80
exit $rc
