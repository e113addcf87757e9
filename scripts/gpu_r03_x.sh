#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
VISSM_LIB=$ROOT/abl/lib_hwlog.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_config_parity.py tests/test_gpu_parity.py -k "ar_cfg or lv or matrix_core" > "$OUT/r03_x_tests.log" 2>&1
rc=$?; tail -1 "$OUT/r03_x_tests.log"; [ $rc -eq 0 ] || { tail -30 "$OUT/r03_x_tests.log"; exit 3; }
ROUNDS=3 STEPS=5 bash scripts/ab_step.sh || exit 4
for r in 1 2; do for v in base hwlog; do VISSM_LIB=$ROOT/abl/lib_$v.so timeout -k 10 300 python -u bench.py --model lv --steps 3 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/x_lv.json" 2>/dev/null || exit 4
python -c "import json;d=json.load(open('$OUT/x_lv.json'));r=d['roofline'];print('$v lv', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), round(r['fwd_kernel_avg_ms'],3))"; done; done
