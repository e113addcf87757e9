#!/bin/bash
# bf16x2 forward on the two-sample kernel: the bf16x2f parity cases, then the bench's parity-precision lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_config_parity.py tests/test_gpu_parity.py tests/test_gpu_posterior.py tests/test_gpu_fused.py -k "x2f or X2F or 29 or theta_fold" > "$OUT/s5_x2f.log" 2>&1; rc=$?
tail -3 "$OUT/s5_x2f.log"; grep -E "FAIL|Error" "$OUT/s5_x2f.log" | head -5; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --cpu-baseline off --families off > "$OUT/s5_bench.json" 2> "$OUT/s5_bench.err" || { tail -5 "$OUT/s5_bench.err"; exit 4; }
python -c "import json;d=json.load(open('$OUT/s5_bench.json'));print(round(d['ms_per_step'],2), [(p['dtype'], round(p['ms_per_step'],2), p['value'], round(p['flow_fwd_avg_ms'],2), round(p['flow_bwd_avg_ms'],2)) for p in d['parity_precision']])"
