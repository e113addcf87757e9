#!/bin/bash
# Round-3 session c: GPU suite on the theta-fold build, then the fold A/B on the AR-cfg step
# (VISSM_THETA_FOLD=1 / 0: the same library, the host passes the theta factors or not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_fused.py > "$OUT/s2_fused.log" 2>&1; rc=$?
tail -3 "$OUT/s2_fused.log"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for f in 1 0; do
  VISSM_THETA_FOLD=$f timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/s2_ab_$f.json" 2>"$OUT/s2_ab_$f.err" || { tail -5 "$OUT/s2_ab_$f.err"; exit 4; }
  python -c "import json;d=json.load(open('$OUT/s2_ab_$f.json'));r=d['roofline'];print('fold=$f', round(d['ms_per_step'],2), round(r['avg_launch_ms'],2), {k:round(v['avg_launch_ms'],2) for k,v in r['variants'].items()}, 'fwd', round(r['fwd_kernel_avg_ms'],2))"
done; done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/s2_pytest_gpu.log" 2>&1; rc=$?
tail -3 "$OUT/s2_pytest_gpu.log"; exit $rc
