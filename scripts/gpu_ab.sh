#!/bin/bash
# GPU session: parity (default impl), flow A/B micro-bench, PMC counters, full bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
fault() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping: rc=$rc"; exit "$rc"; fi; }
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_gpu.log"; fault $rc
echo "== flow A/B (AR cfg)"; timeout -k 10 600 python scripts/flow_bench.py --B 65536 --impls 2,4 > "$OUT/flow_ab_ar.log" 2>&1 || { tail -20 "$OUT/flow_ab_ar.log"; exit 3; }; tail -1 "$OUT/flow_ab_ar.log"
echo "== flow A/B (LV-like)"; timeout -k 10 600 python scripts/flow_bench.py --B 4096 --k 20 --nh 3 --stride2 --impls 2,4 > "$OUT/flow_ab_lv.log" 2>&1 || { tail -20 "$OUT/flow_ab_lv.log"; exit 4; }; tail -1 "$OUT/flow_ab_lv.log"
echo "== bench full"; timeout -k 10 900 python bench.py --cpu-baseline off > "$OUT/bench_full.log" 2>&1 || { tail -20 "$OUT/bench_full.log"; exit 5; }; tail -1 "$OUT/bench_full.log"
echo "== counters"; cd /tmp && timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "rc=$?"; grep -c . "$OUT/counters.txt"
echo "== pmc"; cd /tmp && timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F32 --kernel-trace --stats -T --kernel-include-regex "bwd_kernel|fwd_kernel" -d "$OUT/pmc1" -o pmc --output-format csv -- python "$ROOT/scripts/flow_bench.py" --B 16384 --only 4 --rounds 2 > "$OUT/pmc1.log" 2>&1; echo "pmc rc=$?"; tail -3 "$OUT/pmc1.log"
date
