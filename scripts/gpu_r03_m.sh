#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_elbo_models.py tests/test_gpu_dist.py tests/test_gpu_parity.py -k "elbo or dist or lv or sv or fhn" > "$OUT/r03_m_tests.log" 2>&1
rc=$?; grep -E "FAIL|passed|failed" "$OUT/r03_m_tests.log" | tail -8; [ $rc -le 1 ] || exit $rc
for r in 1 2; do for v in seg1 seg2 seg4; do
  echo -n "$v "; VISSM_LIB=$ROOT/abl/lib_$v.so ROUNDS=3 timeout -k 10 120 python -u scripts/elbo_models_bench.py || exit 4
done; done
