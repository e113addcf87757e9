#!/bin/bash
# Round-3 session c, final evidence on the committed build: GPU suite, smoke, full bench, rocprofv3 kernel-trace
# summary and the two HBM-traffic PMC passes (gpu_round.sh), then SQ counters of the two-sample kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit $?
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
i=0
for SET in "$P1" "$P2"; do i=$((i+1))
  cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $SET --kernel-trace --stats -T --kernel-include-regex "bwd2|fwd2" -d "$OUT/sq_$i" -o pmc --output-format csv -- python "$ROOT/scripts/flow_bench.py" --B 16384 --only bf16 --rounds 2 > "$OUT/sq_$i.log" 2>&1 || { tail -20 "$OUT/sq_$i.log"; exit 3; }
done
cd "$ROOT" && python scripts/pmc_summary.py "$OUT/sq_1" "$OUT/sq_2" > "$OUT/sq_summary.txt" 2>&1; head -3 "$OUT/sq_summary.txt"
