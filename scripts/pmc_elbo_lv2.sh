#!/bin/bash
# LV one-pass kernel after the rates rewrite: VALU / transcendental / wait counters (one pass) over the LV kernels alone
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_lv2; mkdir -p "$OUT"; export TMPDIR=/tmp
MODELS=lv ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/p1" -o run -- python3 scripts/elbo_models_bench.py > "$OUT/p1.log" 2>&1
echo "p1 rc=$?"
