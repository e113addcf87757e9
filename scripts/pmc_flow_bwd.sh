#!/bin/bash
# SQ counters of the AR-cfg step's kernels (bench.py, one warmup + one timed step), three PMC passes of their own
# (at most 8 SQ counters each); summarised per kernel by scripts/pmc_sq_table.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_sq; mkdir -p "$OUT"; export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 1 --cpu-baseline off --parity-line off --families off"
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY" \
           "SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- $B > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
python3 scripts/pmc_sq_table.py "$OUT"/p*/run_counter_collection.csv > "$OUT/sq_table.txt" && cat "$OUT/sq_table.txt"
