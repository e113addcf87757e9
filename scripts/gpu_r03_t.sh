#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_config_parity.py tests/test_gpu_golden.py tests/test_gpu_loop.py tests/test_gpu_dist.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py -k "sv or lv or fhn or matrix_core" > "$OUT/r03_t_tests.log" 2>&1
rc=$?; grep -E "FAIL|passed|failed" "$OUT/r03_t_tests.log" | tail -6; [ $rc -eq 0 ] || exit 3
for m in sv lv fhn; do timeout -k 10 300 python -u bench.py --model $m --steps 4 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/r03_t_$m.json" 2>"$OUT/r03_t_$m.err" || { tail -5 "$OUT/r03_t_$m.err"; exit 4; }
python -c "import json;d=json.load(open('$OUT/r03_t_$m.json'));r=d['roofline'];print('$m', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), {k:round(v['avg_launch_ms'],2) for k,v in r['variants'].items()}, 'fwd', round(r['fwd_kernel_avg_ms'],2), '%.3e' % d['value'])"; done
