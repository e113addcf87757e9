#!/bin/bash
# The driver's round-end GPU check, verbatim (python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider, no --timeout),
# under an outer time limit; the conftest hook names each test on stderr with its start time, and a fatal signal's
# Python stack goes to gpurun_out/faulthandler.log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
date
timeout -k 10 ${TLIM:-1000} python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider ${PYTEST_ARGS} \
    > "$OUT/pytest_driver.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 "$OUT/pytest_driver.log"; date
exit $rc
