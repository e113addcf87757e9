#!/bin/bash
# PMC counter passes (separate runs, kernel trace only) on the flow micro-benchmark.
# usage: IMPL=bf16 B=16384 bash scripts/gpu_pmc.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
IMPL=${IMPL:-bf16}; B=${B:-16384}; TAG=${TAG:-pmc}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P3="SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_DATA_FIFO_FULL"
P4="TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE"
i=0
for SET in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  echo "== pass $i"
  cd /tmp && timeout -k 10 600 rocprofv3 --pmc $SET --kernel-trace --stats -T --kernel-include-regex "bwd|fwd" -d "$OUT/${TAG}_$i" -o pmc --output-format csv -- python "$ROOT/scripts/flow_bench.py" --B $B --only $IMPL --rounds 2 ${EXTRA} > "$OUT/${TAG}_$i.log" 2>&1 || { tail -20 "$OUT/${TAG}_$i.log"; exit 3; }
done
cd "$ROOT" && python scripts/pmc_summary.py "$OUT/${TAG}_1" "$OUT/${TAG}_2" "$OUT/${TAG}_3" "$OUT/${TAG}_4"
