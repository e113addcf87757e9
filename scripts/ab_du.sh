#!/bin/bash
# A/B: the first flow's backward with and without du (same library; VISSM_FORCE_DU=1 computes it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do for F in 1 0; do
  echo -n "force_du=$F "
  VISSM_FORCE_DU=$F timeout -k 10 300 python bench.py --cpu-baseline off --parity-line off --steps 5 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), round(r['fwd_kernel_avg_ms'],2))"
done; done
