#!/bin/bash
# Round-6 session k: the bf16 GEMM (vissm_gemm_bf16) and LV's feature branch on it (VISSM_LV_FEAT=hip): kernel
# parity, the LV config / full-size parity cases through it, then the LV step hip vs torch form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06k; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
echo "== gemm + lv feature parity"; date
timeout -k 10 600 $PT tests/test_gpu_lvfeat.py > "$OUT/pytest_lvfeat.log" 2>&1; rc=$?
tail -n 15 "$OUT/pytest_lvfeat.log"; [ $rc -eq 0 ] || exit $rc
echo "== LV parity cases through the HIP feature branch"; date
VISSM_LV_FEAT=hip timeout -k 10 600 $PT tests/test_gpu_config_parity.py tests/test_gpu_fullsize_lv.py -k "lv or LV" \
  > "$OUT/pytest_lv_hip.log" 2>&1; rc=$?
tail -n 4 "$OUT/pytest_lv_hip.log"; [ $rc -eq 0 ] || exit $rc
echo "== LV step"; date
for rep in 1 2; do for f in torch hip; do
  VISSM_LV_FEAT=$f timeout -k 10 300 python bench.py --model lv --steps 6 --warmup 2 --cpu-baseline off \
    --parity-line off --families off > "$OUT/lv_$f.json" 2> "$OUT/lv_$f.err" || { tail -5 "$OUT/lv_$f.err"; exit 3; }
  python -c "import json;d=json.load(open('$OUT/lv_$f.json'));r=d['roofline'];print('lv $f', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), 'fwd', round(r['fwd_kernel_avg_ms'],2))"
done; done
echo "== kernel trace, LV step with the HIP feature branch"; date
cd /tmp && VISSM_LV_FEAT=hip timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o lv --output-format csv -- python "$ROOT/bench.py" --model lv --steps 3 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 4; }
date
