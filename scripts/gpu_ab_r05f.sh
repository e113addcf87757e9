#!/bin/bash
# Round-5 session f: the theta-branch backward kernel (vissm_theta_branch_bwd) -- its test and the q(theta) / flow
# tests, then the step A/B against the torch form (VISSM_THETA_BRANCH_TORCH=1, same library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r05f; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python3 -m pytest tests/test_gpu_theta.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_graph.py -x -q -m gpu -p no:cacheprovider > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" "$OUT/pytest.log" | head -20; exit $rc; }
for r in 1 2 3; do
  for mode in kernel torch; do
    if [ $mode = torch ]; then export VISSM_THETA_BRANCH_TORCH=1; else unset VISSM_THETA_BRANCH_TORCH; fi
    timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/ab.json" 2>"$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 4; }
    python3 -c "import json;d=json.load(open('$OUT/ab.json'));print('$mode', round(d['ms_per_step'],2))"
  done
done
