#!/bin/bash
# A/B of the full AR-cfg training step over the library builds given as arguments (default abl/*.so; alternating,
# ROUNDS rounds):
# ms per step, backward per launch (average and per variant), roofline fraction.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=${OUT:-$ROOT/gpurun_out}; mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do for L in ${@:-abl/*.so}; do
  n=$(basename $L .so)
  VISSM_LIB=$ROOT/$L timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 2 --cpu-baseline off \
    --parity-line off --families off $EXTRA > "$OUT/ab_$n.json" 2>"$OUT/ab_$n.err" || { tail -5 "$OUT/ab_$n.err"; exit 4; }
  python -c "import json;d=json.load(open('$OUT/ab_$n.json'));r=d['roofline'];print('$n', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), {k:round(v['avg_launch_ms'],2) for k,v in r['variants'].items()}, 'fwd', round(r['fwd_kernel_avg_ms'],2), round(r['frac'],4))"
done; done
