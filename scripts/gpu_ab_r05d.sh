#!/bin/bash
# Round-5 session d: one-pass ELBO chunk width and residency per model -- parity of the production build,
# then the kernels alone across the variant builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r05d; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== elbo parity"; date
timeout -k 10 600 python3 -m pytest tests/test_gpu_elbo_models.py -x -q -m gpu -p no:cacheprovider > "$OUT/pytest_elbo_models.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_elbo_models.log"
[ $rc -eq 0 ] || { grep -E "^E |Error" "$OUT/pytest_elbo_models.log" | head -20; exit $rc; }
echo "== elbo A/B"; date
ROUNDS=2 timeout -k 10 400 bash scripts/ab_elbo.sh abl/lib_base.so abl/lib_lvkv4w4.so abl/lib_lvkv4w1.so abl/lib_sv1.so > "$OUT/ab_elbo.log" 2>&1 || { tail -20 "$OUT/ab_elbo.log"; exit 2; }
cat "$OUT/ab_elbo.log"
date
