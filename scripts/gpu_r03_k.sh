#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
PYTHONPATH=$ROOT timeout -k 10 200 python -u scripts/mm_x3_micro.py && timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_split.py > "$OUT/r03_k_split.log" 2>&1 || { tail -30 "$OUT/r03_k_split.log"; exit 3; }
tail -2 "$OUT/r03_k_split.log"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_lv_x3" -o lv --output-format csv -- python3 "$ROOT/bench.py" --model lv --steps 4 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/prof_lv_x3.log" 2>&1 || exit 4
f=$(find "$OUT/prof_lv_x3" -name "*kernel_stats.csv" | head -1); python3 - "$f" << 'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]: print("%-60s %5s %10.3f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_config_parity.py -k "lv" tests/test_gpu_parity.py -k "lv" tests/test_gpu_loop.py > "$OUT/r03_k_tests.log" 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" "$OUT/r03_k_tests.log" | tail -12; [ $rc -le 1 ] || exit $rc
for r in 1 2; do timeout -k 10 300 python -u bench.py --model lv --steps 5 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/r03_k_lv.json" 2>"$OUT/r03_k_lv.err" || { tail -5 "$OUT/r03_k_lv.err"; exit 4; }
python -c "import json;d=json.load(open('$OUT/r03_k_lv.json'));r=d['roofline'];print('lv', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), round(r['fwd_kernel_avg_ms'],2), '%.3e' % d['value'])"; done
