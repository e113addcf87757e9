#!/bin/bash
# A/B of abl/*.so on the LV / SV / FHN log-density kernels alone (scripts/elbo_models_bench.py), ROUNDS rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 ${ROUNDS:-2}); do for L in abl/*.so; do
  echo -n "$L "
  VISSM_LIB=$PWD/$L timeout -k 10 200 python scripts/elbo_models_bench.py 2>/dev/null | tail -1 || exit 3
done; done
