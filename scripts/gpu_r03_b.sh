#!/bin/bash
# Round 3 session b: full GPU suite (new posterior / save_paths / bench-geometry cases included; the long
# recovery test deselected), the AR posterior recovery trajectory, and the default bench (family lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== posterior trajectory"; date
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_posterior.py::test_ar_posterior_trajectory_matches_oracle" > "$OUT/r03_posterior_traj.log" 2>&1
rc=$?; tail -5 "$OUT/r03_posterior_traj.log"; [ $rc -le 1 ] || exit $rc
echo "== recovery"; date
timeout -k 10 400 python -u scripts/ar_recovery.py --steps 30000 --every 1000 > "$OUT/r03_recovery.log" 2>&1
rc=$?; tail -3 "$OUT/r03_recovery.log"; [ $rc -eq 0 ] || exit $rc
echo "== bench"; date
timeout -k 10 600 python -u bench.py > "$OUT/r03_bench_b.log" 2>&1
rc=$?; tail -c 600 "$OUT/r03_bench_b.log"; [ $rc -eq 0 ] || exit $rc
echo "== suite"; date
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_posterior.py::test_ar_posterior_recovers_generating_theta \
  --deselect tests/test_gpu_posterior.py::test_ar_posterior_trajectory_matches_oracle > "$OUT/r03_suite_b.log" 2>&1
rc=$?; tail -5 "$OUT/r03_suite_b.log"
date
exit $rc
