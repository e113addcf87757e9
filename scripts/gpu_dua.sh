#!/bin/bash
# Fused last flow with aligned du blocks (DUA): fused / pitch parity tests, step A/B against the previous build
# (abl/lib_base.so), WRITE_SIZE of the flow backward launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_pitch.py tests/test_gpu_fused.py tests/test_gpu_posterior.py tests/test_gpu_fullsize.py > "$OUT/pytest_dua.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_dua.log"; [ $rc -eq 0 ] || exit $rc
ROUNDS=2 bash scripts/ab_step.sh abl/lib_dua.so abl/lib_base.so || exit 4
cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -T --kernel-include-regex "bwd2" -d "$OUT/pmcw_dua" -o pmc --output-format csv -- python "$ROOT/bench.py" --steps 1 --warmup 0 --cpu-baseline off --parity-line off --families off > "$OUT/pmcw_dua.log" 2>&1 || { tail -20 "$OUT/pmcw_dua.log"; exit 5; }
cd "$ROOT" && python - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/pmcw_dua/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r["Kernel_Name"][:60], "WRITE_SIZE GB", round(float(r["Counter_Value"]) * 1024 / 1e9, 3))
PY
