#!/bin/bash
# Round-5 session b: the neighbour-exchange one-pass ELBO kernel (stream_onepass_kernel) -- parity (the one-pass
# tests against the two launches and the oracle), then A/B against the chunk-local one-pass (VISSM_ELBO_ONEPASS_NB=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r05b; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== one-pass parity"; date
timeout -k 10 600 python3 -m pytest tests/test_gpu_elbo_models.py -x -q -m gpu -p no:cacheprovider > "$OUT/pytest_elbo_models.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_elbo_models.log"
[ $rc -eq 0 ] || { grep -E "^E |Error" "$OUT/pytest_elbo_models.log" | head -20; exit $rc; }
echo "== elbo A/B"; date
ROUNDS=2 timeout -k 10 400 bash scripts/ab_elbo.sh abl/lib_base.so abl/lib_chunk.so > "$OUT/ab_elbo.log" 2>&1 || { tail -20 "$OUT/ab_elbo.log"; exit 2; }
cat "$OUT/ab_elbo.log"
date
