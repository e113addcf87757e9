#!/bin/bash
# Round-6 session e: elu' as f16 pairs from the recompute's clamped exponential, applied by v_fma_mix_f32
# (VISSM_DERIV16) in bwd2_kernel: parity of the production build (DERIV16, SLP on) and of the no-SLP build, then the
# AR-cfg step A/B over base (DERIV16=0) / d16 / d16ns (no SLP in flow_v5 + flow_v5f) / ns.  Each step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06e; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
echo "== parity, production build"; date
timeout -k 10 600 $PT tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_config_parity.py \
  tests/test_gpu_parity.py tests/test_gpu_pitch.py tests/test_gpu_reduce.py tests/test_gpu_fullsize_lv.py \
  tests/test_gpu_vgpr_form.py > "$OUT/pytest_d16.log" 2>&1; rc=$?
tail -n 3 "$OUT/pytest_d16.log"; [ $rc -eq 0 ] || exit $rc
echo "== parity, split-weight modes (lofold) and posterior trajectories"; date
timeout -k 10 600 $PT tests/test_gpu_posterior.py -k "not recover" tests/test_gpu_split.py > "$OUT/pytest_x2.log" 2>&1; rc=$?
tail -n 3 "$OUT/pytest_x2.log"; [ $rc -eq 0 ] || exit $rc
echo "== parity, no-SLP build"; date
VISSM_LIB=$ROOT/abl/lib_d16ns.so timeout -k 10 400 $PT tests/test_gpu_fused.py tests/test_gpu_config_parity.py -k "ar or AR" \
  > "$OUT/pytest_d16ns.log" 2>&1; rc=$?
tail -n 3 "$OUT/pytest_d16ns.log"; [ $rc -eq 0 ] || exit $rc
echo "== A/B"; date
OUT=$OUT ROUNDS=2 STEPS=10 bash scripts/ab_step.sh abl/lib_base.so abl/lib_d16.so abl/lib_d16ns.so abl/lib_ns.so
echo "== A/B LV / FHN (bwd2n: flow_v5n, DERIV16 on / off)"; date
OUT=$OUT/lv ROUNDS=2 STEPS=6 EXTRA="--model lv" bash scripts/ab_step.sh abl/lib_base.so abl/lib_d16.so
OUT=$OUT/fhn ROUNDS=2 STEPS=6 EXTRA="--model fhn" bash scripts/ab_step.sh abl/lib_base.so abl/lib_d16.so
OUT=$OUT/x2f ROUNDS=1 STEPS=6 EXTRA="--precision bf16x2f" bash scripts/ab_step.sh abl/lib_base.so abl/lib_nolof.so \
  abl/lib_d16.so abl/lib_nwf4.so
date
