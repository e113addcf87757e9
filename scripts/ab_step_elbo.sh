#!/bin/bash
# A/B of the one-pass log-density kernel inside the family steps (bench.py --model M): its in-step launch time and HBM
# fraction (streaming_rooflines) per library build given as arguments (alternating, ROUNDS rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=${OUT:-$ROOT/gpurun_out}; mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do for L in "$@"; do for model in ${MODELS:-sv}; do
  n=$(basename $L .so)
  VISSM_LIB=$ROOT/$L timeout -k 10 300 python -u bench.py --model $model --steps ${STEPS:-6} --warmup 2 --cpu-baseline off \
    --parity-line off --families off > "$OUT/ab_se.json" 2>"$OUT/ab_se.err" || { tail -5 "$OUT/ab_se.err"; exit 4; }
  python -c "import json;d=json.load(open('$OUT/ab_se.json'));s=[x for x in d['streaming_rooflines'] if 'onepass' in x['kernel'] or 'elbo' in x['kernel']][0];print('$n', '$model', round(d['ms_per_step'],2), 'elbo', round(s['avg_launch_ms'],4), round(s['frac'],3))"
done; done; done
