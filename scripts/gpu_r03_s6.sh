#!/bin/bash
# two-sample forward at the three-hidden-layer shapes: LV / FHN / SV parity, then the family steps A/B (abl/*.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_config_parity.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_loop.py tests/test_gpu_graph.py -k "lv or fhn or sv or LV or FHN or SV" > "$OUT/s6_par.log" 2>&1; rc=$?
tail -3 "$OUT/s6_par.log"; grep -E "^FAILED|Error" "$OUT/s6_par.log" | head -5; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for L in abl/*.so; do n=$(basename $L .so); for m in lv fhn; do
  VISSM_LIB=$ROOT/$L timeout -k 10 300 python -u bench.py --model $m --steps 4 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/s6_$n_$m.json" 2>/dev/null || exit 4
  python -c "import json;d=json.load(open('$OUT/s6_$n_$m.json'));r=d['roofline'];print('$n $m', round(d['ms_per_step'],2), 'bwd', round(r['avg_launch_ms'],2), 'fwd', round(r['fwd_kernel_avg_ms'],3))"
done; done; done
