#!/bin/bash
# One box, several sessions (each script keeps its own limits): the driver's test command, then the scripts named in
# COMBO (default: the round-5 A/B session).  A fault / abort / time limit in any step ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_driver_suite.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: suite rc=$rc"; exit $rc; fi
for s in ${COMBO:-scripts/gpu_ab_r05a.sh}; do
  bash "$s" || { rc=$?; echo "stopping: $s rc=$rc"; exit $rc; }
done
