#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== fused parity"; date
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fused.py tests/test_gpu_fullsize.py > "$OUT/r03_f_tests.log" 2>&1
rc=$?; tail -3 "$OUT/r03_f_tests.log"; [ $rc -le 1 ] || exit $rc
echo "== A/B"; date
bash scripts/ab_step.sh || exit $?
for M in lv sv fhn; do MODELS=$M TAG=elbo_pmc_$M bash scripts/gpu_pmc_elbo.sh > "$OUT/r03_elbo_pmc_$M.txt" 2>&1 || exit 5; done
for M in lv sv fhn; do echo "== $M"; grep -E "kernel|INSTS_VALU|ACTIVE_INST_VALU|WAVE_CYCLES|GRBM_GUI|SQ_BUSY|WAIT" "$OUT/r03_elbo_pmc_$M.txt" | head -30; done
