#!/bin/bash
# Round-6 session w: the training-step GPU tests after sync_grads restores the views of gradient-less variables.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06w; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_gpu_loop.py tests/test_gpu_graph.py tests/test_gpu_dist.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_optim.py > "$OUT/pytest_step.log" 2>&1; rc=$?
tail -n 2 "$OUT/pytest_step.log"; exit $rc
