#!/bin/bash
# SQ counter passes (separate runs, kernel trace only) of the LV / SV / FHN streaming log-density kernels at
# the configs' per-GPU shapes (scripts/elbo_models_bench.py): VALU busy vs wave cycles says whether a kernel
# below half the HBM roof is vector-bound.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
TAG=${TAG:-elbo_pmc}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM"
P2="SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for SET in "$P1" "$P2"; do
  i=$((i+1))
  echo "== pass $i"
  cd /tmp && timeout -k 10 300 rocprofv3 --pmc $SET --kernel-trace --stats -T --kernel-include-regex "stream_|elbo" -d "$OUT/${TAG}_$i" -o pmc --output-format csv -- python "$ROOT/scripts/elbo_models_bench.py" > "$OUT/${TAG}_$i.log" 2>&1 || { tail -20 "$OUT/${TAG}_$i.log"; exit 3; }
done
cd "$ROOT" && python scripts/pmc_summary.py "$OUT/${TAG}_1" "$OUT/${TAG}_2"
