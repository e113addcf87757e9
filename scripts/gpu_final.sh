#!/bin/bash
# Final session of a round: the driver's GPU test command and smoke (scripts/gpu_suite_smoke.sh), then the bench,
# its kernel trace and the PMC traffic passes (scripts/gpu_round.sh without its own tests).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_suite_smoke.sh || { rc=$?; echo "stopping: suite/smoke rc=$rc"; exit $rc; }
SKIP_TESTS=1 bash scripts/gpu_round.sh
