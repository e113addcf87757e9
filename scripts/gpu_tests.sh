#!/bin/bash
# Run a selection of GPU tests (TESTS, pytest node ids / -k expressions via PYTEST_ARGS) under a time limit,
# then optional extra commands (EXTRA, one shell line; each of its GPU steps carries its own timeout).
# Output under gpurun_out/; a crash or timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
LOG=${LOG:-pytest_sel}
if [ -n "$TESTS" ]; then
  echo "== pytest $TESTS $PYTEST_ARGS"; date
  timeout -k 10 ${TLIM:-900} python -u -m pytest $TESTS $PYTEST_ARGS -m gpu -v -p no:cacheprovider --timeout 400 \
      --timeout-method thread > "$OUT/$LOG.log" 2>&1; rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/$LOG.log" | tail -40
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc=$rc"; exit $rc; fi
fi
if [ -n "$EXTRA" ]; then echo "== extra"; date; bash -o pipefail -c "$EXTRA"; fi
date
