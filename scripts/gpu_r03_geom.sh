#!/bin/bash
# Round 3, first GPU session: the bench-geometry / full-size / reduction parity tests, then the SQ counter
# passes of the current flow backward (AR-cfg middle flow shape, B = 16384) and of the nh = 3 (LV) shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== tests"; date
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_reduce.py tests/test_gpu_fullsize.py \
  "tests/test_gpu_config_parity.py::test_ar_cfg_bench_geometry" \
  "tests/test_gpu_fused.py::test_fused_step_ar_cfg_bench_geometry" \
  "tests/test_gpu_fused.py::test_fused_step_matches_oracle" > "$OUT/r03_geom_tests.log" 2>&1
rc=$?; tail -30 "$OUT/r03_geom_tests.log"; [ $rc -le 1 ] || exit $rc
echo "== pmc AR"; date
TAG=r03_ar_pmc IMPL=bf16 B=16384 bash scripts/gpu_pmc.sh > "$OUT/r03_ar_pmc.txt" 2>&1 || { tail -5 "$OUT/r03_ar_pmc.txt"; exit 3; }
echo "== pmc LV nh3"; date
TAG=r03_lv_pmc IMPL=bf16 B=4096 EXTRA="--k 20 --nh 3 --stride2" bash scripts/gpu_pmc.sh > "$OUT/r03_lv_pmc.txt" 2>&1 || { tail -5 "$OUT/r03_lv_pmc.txt"; exit 4; }
date
