#!/bin/bash
# GPU suite + default bench (family lines, CPU baseline) on the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/s4_pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/s4_pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > "$OUT/s4_bench.json" 2> "$OUT/s4_bench.err" || { tail -5 "$OUT/s4_bench.err"; exit 4; }
python -c "import json;d=json.load(open('$OUT/s4_bench.json'));r=d['roofline'];print(d['value'], round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), {k:round(v['avg_launch_ms'],2) for k,v in r['variants'].items()}, round(r['frac'],4), [(f['model'], round(f['ms_per_step'],2)) for f in d.get('family_lines',[])])"
