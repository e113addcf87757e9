#!/bin/bash
# bf16x2f with the last flow fused (split-weight recompute), SV forward on the two-sample kernel: parity, then A/B
# of the AR headline + parity-precision lines and the SV step over abl/*.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_config_parity.py tests/test_gpu_posterior.py tests/test_gpu_parity.py tests/test_gpu_golden.py -k "fused or theta_fold or x2f or X2F or 17 or sv or SV" > "$OUT/s7_par.log" 2>&1; rc=$?
tail -3 "$OUT/s7_par.log"; grep -E "^FAILED|Error" "$OUT/s7_par.log" | head -8; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for L in abl/*.so; do n=$(basename $L .so)
  VISSM_LIB=$ROOT/$L timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline off --families off > "$OUT/s7_$n.json" 2>/dev/null || exit 4
  python -c "import json;d=json.load(open('$OUT/s7_$n.json'));r=d['roofline'];print('$n', round(d['ms_per_step'],2), 'fwd', round(r['fwd_kernel_avg_ms'],2), [(p['dtype'], round(p['ms_per_step'],2), '%.3e' % p['value']) for p in d['parity_precision']])"
  VISSM_LIB=$ROOT/$L timeout -k 10 300 python -u bench.py --model sv --steps 4 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/s7_sv.json" 2>/dev/null || exit 4
  python -c "import json;d=json.load(open('$OUT/s7_sv.json'));r=d['roofline'];print('$n sv', round(d['ms_per_step'],2), 'bwd', round(r['avg_launch_ms'],2), 'fwd', round(r['fwd_kernel_avg_ms'],3))"
done; done
