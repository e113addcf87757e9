#!/bin/bash
# A/B of abl/*.so on the AR-cfg step, then the bench-geometry fused parity case on each variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
ROUNDS=2 bash scripts/ab_step.sh || exit $?
for L in abl/*.so; do n=$(basename $L .so)
  VISSM_LIB=$ROOT/$L timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_fused.py -k "bench_geometry or theta_fold" > "$OUT/s3_par_$n.log" 2>&1; rc=$?
  echo "$n parity rc=$rc $(tail -1 $OUT/s3_par_$n.log)"; [ $rc -gt 1 ] && exit $rc
done; exit 0
