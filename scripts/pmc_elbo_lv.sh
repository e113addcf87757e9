#!/bin/bash
# LV one-pass ELBO instruction mix: the counters available, then SQ instruction / cycle counters over the LV kernels
# alone (scripts/elbo_models_bench.py, MODELS=lv, one round)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_lv; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
grep -oE "SQ_[A-Z0-9_]+" "$OUT/avail.txt" | sort -u > "$OUT/sq_counters.txt" || true
cd "$ROOT"
MODELS=lv ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/p1" -o run -- python3 scripts/elbo_models_bench.py > "$OUT/p1.log" 2>&1
echo "p1 rc=$?"
ls -R "$OUT" | head -20
