#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
ROUNDS=2 STEPS=6 bash scripts/ab_step.sh || exit 4
for r in 1 2; do for v in base noslp; do
  echo -n "$v "; VISSM_LIB=$ROOT/abl/lib_$v.so timeout -k 10 300 python -u bench.py --model lv --steps 3 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/q_lv.json" 2>"$OUT/q_lv.err" || { tail -5 "$OUT/q_lv.err"; exit 4; }
  python -c "import json;d=json.load(open('$OUT/q_lv.json'));r=d['roofline'];print('lv', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), round(r['fwd_kernel_avg_ms'],2))"
done; done
