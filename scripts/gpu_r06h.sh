#!/bin/bash
# Round-6 session h: the adopted tree (lofold for the split-weight kernels, VISSM_DERIV16 = 2, flow_v5 / flow_v5f
# without SLP): parity of the flow kernels and the posterior trajectories, then the AR-cfg step at bf16 and bf16x2f and
# the LV / FHN steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06h; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
echo "== parity"; date
timeout -k 10 900 $PT tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_config_parity.py \
  tests/test_gpu_parity.py tests/test_gpu_fullsize_lv.py tests/test_gpu_vgpr_form.py tests/test_gpu_posterior.py \
  -k "not recover" > "$OUT/pytest.log" 2>&1; rc=$?
tail -n 3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
echo "== steps"; date
for spec in "ar bf16" "ar bf16x2f" "lv bf16" "fhn bf16" "ar bf16" "ar bf16x2f"; do
  set -- $spec
  timeout -k 10 300 python bench.py --model $1 --precision $2 --steps 8 --warmup 2 --cpu-baseline off --parity-line off \
    --families off > "$OUT/bench_$1_$2.json" 2> "$OUT/bench_$1_$2.err" || { tail -5 "$OUT/bench_$1_$2.err"; exit 3; }
  python -c "import json;d=json.load(open('$OUT/bench_$1_$2.json'));r=d['roofline'];print('$1 $2', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), {k:round(v['avg_launch_ms'],2) for k,v in r['variants'].items()}, 'fwd', round(r['fwd_kernel_avg_ms'],2))"
done
date
