#!/bin/bash
# A/B of the LV / FHN / SV family steps (bench.py --model) across library builds given as arguments (alternating,
# ROUNDS rounds, default 2), after their bf16 bench-geometry parity cases (tests/test_gpu_config_parity.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
for L in "$@"; do
  n=$(basename $L .so)
  VISSM_LIB=$ROOT/$L timeout -k 10 600 python -u -m pytest tests/test_gpu_config_parity.py -k "family_cfg_bench_geometry and bf16" -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/ab_fam_$n.pytest.log" 2>&1
  rc=$?; echo "$n parity rc=$rc $(tail -1 $OUT/ab_fam_$n.pytest.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
for r in $(seq 1 ${ROUNDS:-2}); do for L in "$@"; do for model in ${MODELS:-lv fhn sv}; do
  n=$(basename $L .so)
  VISSM_LIB=$ROOT/$L timeout -k 10 300 python -u bench.py --model $model --steps ${STEPS:-5} --warmup 2 --cpu-baseline off \
    --parity-line off --families off > "$OUT/ab_fam.json" 2>"$OUT/ab_fam.err" || { tail -5 "$OUT/ab_fam.err"; exit 4; }
  python -c "import json;d=json.load(open('$OUT/ab_fam.json'));r=d['roofline'];print('$n', '$model', round(d['ms_per_step'],2), 'bwd', round(r['avg_launch_ms'],3), {k:round(v['avg_launch_ms'],3) for k,v in r['variants'].items()}, 'fwd', round(r['fwd_kernel_avg_ms'],3))"
done; done; done
