#!/bin/bash
# Row-pitch change: the pitch parity tests, the flow / fused / family parity suites, then the bench with padded rows
# against dense rows (VISSM_ROW_PAD=0) and the WRITE_SIZE pass of the flow backward at both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_pitch.py tests/test_gpu_fused.py tests/test_gpu_config_parity.py tests/test_gpu_parity.py > "$OUT/pytest_pitch.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_pitch.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for pad in 1 0; do
  VISSM_ROW_PAD=$pad timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/bench_pad$pad.json" 2>"$OUT/bench_pad$pad.err" || { tail -5 "$OUT/bench_pad$pad.err"; exit 3; }
  python -c "import json;d=json.load(open('$OUT/bench_pad$pad.json'));print('pad $pad', round(d['ms_per_step'],3), d['roofline']['achieved'], d.get('kernel_ms'))"
done; done
for pad in 1 0; do
  cd /tmp && VISSM_ROW_PAD=$pad timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -T --kernel-include-regex "bwd" -d "$OUT/pmcw_pad$pad" -o pmc --output-format csv -- python "$ROOT/bench.py" --steps 1 --warmup 0 --cpu-baseline off --parity-line off --families off > "$OUT/pmcw_pad$pad.log" 2>&1 || { tail -20 "$OUT/pmcw_pad$pad.log"; exit 5; }
done
cd "$ROOT" && python - <<'PY'
import csv, glob
for pad in (1, 0):
    for f in glob.glob(f"gpurun_out/pmcw_pad{pad}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            print("pad", pad, r["Kernel_Name"][:60], "WRITE_SIZE GB", round(float(r["Counter_Value"]) * 1024 / 1e9, 3))
PY
