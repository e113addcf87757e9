#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
VISSM_FEATURE_GEMM=bf16 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_config_parity.py tests/test_gpu_parity.py tests/test_gpu_golden.py -k "lv" > "$OUT/r03_z_tests.log" 2>&1
echo "bf16 feature GEMM parity rc=$?: $(tail -1 $OUT/r03_z_tests.log)"; grep -E "FAIL|Error|assert" "$OUT/r03_z_tests.log" | head -5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_split.py > "$OUT/r03_z_split.log" 2>&1; echo "split rc=$?: $(tail -1 $OUT/r03_z_split.log)"
for r in 1 2; do for v in x3 bf16; do VISSM_FEATURE_GEMM=$v timeout -k 10 300 python -u bench.py --model lv --steps 4 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/z_lv.json" 2>/dev/null || exit 4
python -c "import json;d=json.load(open('$OUT/z_lv.json'));r=d['roofline'];print('$v lv', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), round(r['fwd_kernel_avg_ms'],3))"; done; done
bash scripts/gpu_r03_y.sh
