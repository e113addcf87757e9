#!/bin/bash
# Round-6 session p: split-K of LV's two K = 10,061 GEMMs (G = D^T Wc and dWc = D dG, 632 tiles each: 2.47 blocks
# per CU) -- VISSM_LV_SPLIT 1 / 2 / 3: the LV feature tests at split 2, the LV-cfg step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06p; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
VISSM_LV_SPLIT=2 timeout -k 10 300 $PT tests/test_gpu_lvfeat.py > "$OUT/pytest_split2.log" 2>&1; rc=$?
tail -n 1 "$OUT/pytest_split2.log"; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --model lv --steps 8 --warmup 2 --cpu-baseline off --parity-line off --families off"
for r in 1 2; do for sk in 1 2 3; do
  VISSM_LV_SPLIT=$sk timeout -k 10 300 $B > "$OUT/bench_s${sk}_$r.json" 2> "$OUT/bench_s${sk}_$r.err" || exit 5
  python -c "import json; print('split $sk', round(json.loads(open('$OUT/bench_s${sk}_$r.json').read().strip().splitlines()[-1])['ms_per_step'], 2))"
done; done
date
