#!/bin/bash
# A/B of library builds in abl/*.so on the full training step (bench.py, alternating, same box);
# BENCH_ARGS pass through (e.g. "--fuse off")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do for L in abl/*.so; do
  echo -n "$L ${TAG:-} "
  VISSM_LIB=$PWD/$L timeout -k 10 300 python bench.py --cpu-baseline off --parity-line off --steps 5 $BENCH_ARGS 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), round(r['fwd_kernel_avg_ms'],2))"
done; done
