#!/bin/bash
# Round-6 session o: the GEMM's register prefetch depth (VISSM_GEMM_PF 1 / 2) and register bound (VISSM_GEMM_MINB):
# GEMM / feature-branch tests per build, the LV-cfg step A/B, and per-build GEMM kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06o; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
for L in pf2 pf2b3; do
  VISSM_LIB=$ROOT/abl/lib_$L.so timeout -k 10 300 $PT tests/test_gpu_lvfeat.py tests/test_gpu_svfeat.py > "$OUT/pytest_$L.log" 2>&1; rc=$?
  tail -n 1 "$OUT/pytest_$L.log"; [ $rc -eq 0 ] || exit $rc
done
OUT=$OUT ROUNDS=2 STEPS=8 EXTRA="--model lv" bash scripts/ab_step.sh abl/lib_pf1.so abl/lib_pf2.so abl/lib_pf2b3.so || exit 4
cd /tmp && for L in pf1 pf2 pf2b3; do VISSM_LIB=$ROOT/abl/lib_$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_$L" -o lv --output-format csv -- python "$ROOT/bench.py" --model lv --steps 2 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/prof_$L.log" 2>&1 || exit 5; done
date
