#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in new newnoslp; do
VISSM_LIB=$ROOT/abl/lib_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_config_parity.py tests/test_gpu_golden.py tests/test_gpu_loop.py -k "sv" > "$OUT/r03_s_tests_$v.log" 2>&1
rc=$?; echo "$v: $(tail -1 $OUT/r03_s_tests_$v.log)"; [ $rc -eq 0 ] || { tail -30 "$OUT/r03_s_tests_$v.log"; exit 3; }
done
for r in 1 2; do for v in old new newnoslp; do
VISSM_LIB=$ROOT/abl/lib_$v.so timeout -k 10 300 python -u bench.py --model sv --steps 4 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/r03_s_sv.json" 2>"$OUT/r03_s_sv.err" || { tail -5 "$OUT/r03_s_sv.err"; exit 4; }
python -c "import json;d=json.load(open('$OUT/r03_s_sv.json'));r=d['roofline'];print('$v sv', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), {k:round(v['avg_launch_ms'],2) for k,v in r['variants'].items()}, 'fwd', round(r['fwd_kernel_avg_ms'],2), '%.3e' % d['value'])"; done; done
