#!/bin/bash
# LV at bf16 with single-bf16 feature GEMMs (the default now): the LV GPU cases, then the LV step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_config_parity.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_dist.py tests/test_gpu_graph.py tests/test_gpu_loop.py tests/test_gpu_split.py -k "lv or LV or split" > "$OUT/s8_lv.log" 2>&1; rc=$?
tail -3 "$OUT/s8_lv.log"; grep -E "^FAILED|Error" "$OUT/s8_lv.log" | head -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --model lv --steps 4 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/s8_lv.json" 2>/dev/null || exit 4
python -c "import json;d=json.load(open('$OUT/s8_lv.json'));r=d['roofline'];print('lv', round(d['ms_per_step'],2), '%.3e' % d['value'], round(r['avg_launch_ms'],2), round(r['fwd_kernel_avg_ms'],3))"
