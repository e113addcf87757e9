#!/bin/bash
# One-pass AR ELBO values + theta gradient (vissm_elbo_fwd_theta_grad): ELBO / fused / posterior tests, then the
# AR-cfg step against the two-pass form (VISSM_ELBO_TWO_PASS=1), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_elbo.py tests/test_gpu_fused.py tests/test_gpu_posterior.py tests/test_gpu_fullsize.py > "$OUT/pytest_elbo1.log" 2>&1; rc=$?; tail -3 "$OUT/pytest_elbo1.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do for tp in 0 1; do
  VISSM_ELBO_TWO_PASS=$tp timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/b_tp$tp.json" 2>"$OUT/b_tp$tp.err" || { tail -5 "$OUT/b_tp$tp.err"; exit 3; }
  python -c "import json;d=json.load(open('$OUT/b_tp$tp.json'));s=[x for x in d['streaming_rooflines'] if 'elbo' in x['kernel']];print('two_pass $tp', round(d['ms_per_step'],3), [(x['kernel'][:16], round(x['avg_launch_ms'],3)) for x in s])"
done; done
