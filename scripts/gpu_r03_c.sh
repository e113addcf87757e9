#!/bin/bash
# Round 3 session c: two-sample backward (bwd2) correctness first, then the A/B step time against the
# one-sample kernel, then session b's posterior / recovery / bench / suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== bwd2 parity"; date
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fused.py tests/test_gpu_fullsize.py "tests/test_gpu_config_parity.py::test_ar_cfg_bench_geometry" \
  "tests/test_gpu_config_parity.py::test_ar_cfg_length" tests/test_gpu_parity.py > "$OUT/r03_bwd2_tests.log" 2>&1
rc=$?; tail -5 "$OUT/r03_bwd2_tests.log"; [ $rc -le 1 ] || exit $rc
echo "== A/B step"; date
for r in 1 2; do for L in old new; do
  VISSM_LIB=$ROOT/abl/lib_$L.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off \
    --parity-line off --families off > "$OUT/r03_ab_$L.json" 2>"$OUT/r03_ab_$L.err" || { tail -5 "$OUT/r03_ab_$L.err"; exit 4; }
  python -c "import json;d=json.load(open('$OUT/r03_ab_$L.json'));r=d['roofline'];print('$L', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), {k:round(v['avg_launch_ms'],2) for k,v in r['variants'].items()}, round(r['frac'],4))"
done; done
[ "${AB_ONLY:-0}" = 1 ] && exit 0
bash scripts/gpu_r03_b.sh
