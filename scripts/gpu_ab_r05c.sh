#!/bin/bash
# Round-5 session c: the plain-span one-pass ELBO (VissmElboData.plain_from) -- parity (the ELBO model tests incl.
# the plain-span cases), the kernels alone (one pass with and without the plain-span table), the LV / SV steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r05c; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== elbo parity"; date
timeout -k 10 600 python3 -m pytest tests/test_gpu_elbo_models.py -x -q -m gpu -p no:cacheprovider > "$OUT/pytest_elbo_models.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_elbo_models.log"
[ $rc -eq 0 ] || { grep -E "^E |Error" "$OUT/pytest_elbo_models.log" | head -20; exit $rc; }
echo "== elbo kernels"; date
for r in 1 2; do timeout -k 10 120 python3 scripts/elbo_models_bench.py >> "$OUT/elbo_kernels.log" 2>&1 || { tail -20 "$OUT/elbo_kernels.log"; exit 2; }; done
cat "$OUT/elbo_kernels.log"
echo "== lv / sv steps"; date
for m in lv sv; do
  timeout -k 10 300 python3 bench.py --model $m --steps 5 --warmup 2 --cpu-baseline off --parity-line off --families off > "$OUT/step_$m.json" 2> "$OUT/step_$m.err" || { tail -20 "$OUT/step_$m.err"; exit 3; }
  cat "$OUT/step_$m.json"
done
date
