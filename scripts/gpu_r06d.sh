#!/bin/bash
# Round-6 session d: flow_v5n.hip (VGPR form) against the default-form build of the same kernels; the fused feature kernels (vissm_feat_fwd / _bwd) at FHN's kernel_len 20 (stride 2) and SV's 50
# (its diff-augmented input) against the torch + hipBLASLt form they lost to at 32 positions per block (round 4):
# correctness at 8 positions per block, then the FHN / SV steps, alternating.  Each step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06d; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== flow_v5n (VGPR form) vs the default-form build at the shipped shapes"; date
timeout -k 10 400 python -u -m pytest tests/test_gpu_vgpr_form.py -m gpu -q -s -p no:cacheprovider --timeout 300 \
  --timeout-method thread > "$OUT/pytest_vgpr_form.log" 2>&1; rc=$?
grep -E "worst|passed|failed" "$OUT/pytest_vgpr_form.log" | cut -c1-200; [ $rc -eq 0 ] || exit $rc
echo "== feature kernels at 8 positions per block vs torch"; date
VISSM_FEAT_KT=8 VISSM_FEAT_KT_BWD=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_feat.py -m gpu -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_feat_kt8.log" 2>&1; rc=$?
tail -n 2 "$OUT/pytest_feat_kt8.log"; [ $rc -eq 0 ] || exit $rc
echo "== FHN / SV config parity through the feature kernels"; date
VISSM_FEAT_MAX_K=64 timeout -k 10 600 python -u -m pytest tests/test_gpu_config_parity.py -m gpu -q -k "sv or fhn" \
  -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_cfg_feat.log" 2>&1; rc=$?
tail -n 2 "$OUT/pytest_cfg_feat.log"; [ $rc -eq 0 ] || exit $rc
run() {  # name, "VAR=value ..." (environment), bench args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 python bench.py --cpu-baseline off --parity-line off --families off "$@" \
    > "$OUT/$name.log" 2>&1 || { echo "FAILED $name"; tail -n 5 "$OUT/$name.log"; exit 3; }
  python3 -c "
import json; d = json.loads(open('$OUT/$name.log').read().strip().split(chr(10))[-1])
print('$name', round(d['ms_per_step'], 2), 'ms', 'bwd', round(d['roofline']['avg_launch_ms'], 2), flush=True)"
}
for rep in 1 2; do
  for m in fhn sv; do
    run ${m}_torch_$rep "VISSM_FEAT_MAX_K=16" --model $m --steps 6 --warmup 2
    run ${m}_hip_auto_$rep "VISSM_FEAT_MAX_K=64" --model $m --steps 6 --warmup 2
    run ${m}_hip_kt8_$rep "VISSM_FEAT_MAX_K=64 VISSM_FEAT_KT=8 VISSM_FEAT_KT_BWD=8" --model $m --steps 6 --warmup 2
    run ${m}_hip_kt16_$rep "VISSM_FEAT_MAX_K=64 VISSM_FEAT_KT=16 VISSM_FEAT_KT_BWD=16" --model $m --steps 6 --warmup 2
  done
done
date
