#!/bin/bash
# Round-6 session u: LV's feature branch at the parity precisions on the split-bf16 GEMM (vissm_gemm_bf16x3 with hi / lo
# bf16 epilogues): the GEMM / feature tests, every LV GPU test, then the LV-cfg step at bf16x2f against the torch
# form (VISSM_LV_FEAT=torch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06u; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 400 $PT tests/test_gpu_svfeat.py tests/test_gpu_lvfeat.py > "$OUT/pytest_feat.log" 2>&1; rc=$?
tail -n 1 "$OUT/pytest_feat.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 $PT tests/ -k "lv" > "$OUT/pytest_lv.log" 2>&1; rc=$?
tail -n 1 "$OUT/pytest_lv.log"; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --model lv --precision bf16x2f --steps 6 --warmup 2 --cpu-baseline off --parity-line off --families off"
for r in 1 2; do for f in torch hip; do
  VISSM_LV_FEAT=$f timeout -k 10 300 $B > "$OUT/bench_x2f_${f}_${r}.json" 2> "$OUT/bench_x2f_${f}_$r.err" || exit 5
  python -c "import json; print('lv bf16x2f $f', round(json.loads(open('$OUT/bench_x2f_${f}_${r}.json').read().strip().splitlines()[-1])['ms_per_step'], 2))"
done; done
date
