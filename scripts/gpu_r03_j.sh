#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== lv parity"; date
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_config_parity.py -k "lv" tests/test_gpu_parity.py tests/test_gpu_golden.py > "$OUT/r03_j_tests.log" 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" "$OUT/r03_j_tests.log" | tail -8; [ $rc -le 1 ] || exit $rc
echo "== lv step"; date
for r in 1 2; do timeout -k 10 300 python -u bench.py --model lv --steps 5 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/r03_j_lv.json" 2>"$OUT/r03_j_lv.err" || { tail -5 "$OUT/r03_j_lv.err"; exit 4; }
python -c "import json;d=json.load(open('$OUT/r03_j_lv.json'));r=d['roofline'];print('lv', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), round(r['fwd_kernel_avg_ms'],2), '%.3e' % d['value'])"; done
