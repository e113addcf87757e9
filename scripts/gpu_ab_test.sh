#!/bin/bash
# A/B of abl/*.so on the full step (scripts/ab_bench.sh), then the GPU suite and one FETCH_SIZE /
# WRITE_SIZE pass on the in-tree library (TESTS=0 / PMC=0 skip those).  Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== A/B ${TAG:-}"; bash scripts/ab_bench.sh || exit 3
if [ "${TESTS:-1}" = 1 ]; then
  echo "== pytest -m gpu"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu_ab.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_gpu_ab.log"; [ $rc = 0 ] || exit $rc
fi
if [ "${PMC:-1}" = 1 ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== pmc $C"
    cd /tmp && timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --stats -T --kernel-include-regex "bwd_kernel" \
      -d "$OUT/pmc_$C" -o pmc --output-format csv -- python "$ROOT/bench.py" --steps 1 --warmup 0 --cpu-baseline off \
      --parity-line off > "$OUT/pmc_$C.log" 2>&1 || { tail -20 "$OUT/pmc_$C.log"; exit 5; }
  done
  cd "$ROOT" && python scripts/traffic_from_pmc.py bf16 65536 5000 8
fi
