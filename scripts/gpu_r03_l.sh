#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_split.py tests/test_gpu_config_parity.py -k "split or lv_cfg" > "$OUT/r03_l_tests.log" 2>&1 || { tail -30 "$OUT/r03_l_tests.log"; exit 3; }
tail -1 "$OUT/r03_l_tests.log"
for r in 1 2; do timeout -k 10 300 python -u bench.py --model lv --steps 5 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/r03_l_lv.json" 2>"$OUT/r03_l_lv.err" || { tail -5 "$OUT/r03_l_lv.err"; exit 4; }
python -c "import json;d=json.load(open('$OUT/r03_l_lv.json'));r=d['roofline'];print('lv', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), round(r['fwd_kernel_avg_ms'],2), '%.3e' % d['value'])"; done
