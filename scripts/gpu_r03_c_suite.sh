#!/bin/bash
# final GPU suite + smoke + default bench on the committed tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/final_pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/final_pytest_gpu.log"; grep -E "^FAILED" "$OUT/final_pytest_gpu.log" | head; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/final_smoke.log" 2>&1 || { tail -5 "$OUT/final_smoke.log"; exit 2; }
timeout -k 10 900 python -u bench.py > "$OUT/final_bench.json" 2> "$OUT/final_bench.err" || { tail -5 "$OUT/final_bench.err"; exit 4; }
python -c "import json;d=json.load(open('$OUT/final_bench.json'));r=d['roofline'];print(d['value'], round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), round(r['frac'],4), [(p['dtype'], round(p['ms_per_step'],2)) for p in d['parity_precision']], [(f['model'], round(f['ms_per_step'],2), '%.3e' % f['value']) for f in d['family_lines']])"
