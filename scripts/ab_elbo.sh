#!/bin/bash
# A/B timing of the streaming log-density kernels (scripts/elbo_models_bench.py) across library builds
# given as arguments (alternating, ROUNDS rounds, default 2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 ${ROUNDS:-2}); do for L in "$@"; do
  echo -n "$L "
  VISSM_LIB=$PWD/$L timeout -k 10 120 python scripts/elbo_models_bench.py || exit 1
done; done
