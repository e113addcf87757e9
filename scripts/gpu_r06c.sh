#!/bin/bash
# Round-6 session c: SV's k = 50 gradients under -amdgpu-mfma-vgpr-form=1 -- the plain flagged build and two padded
# ones (-amdgpu-snop-padding=15: an s_nop 15 before every instruction; -amdgpu-mfma-padding-ratio=100: the whole MFMA
# latency as s_nops between neighbouring MFMAs) -- which tells a wait-state hazard from a register-allocation fault;
# then the posterior tests (the multi-seed recovery criterion).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06c; mkdir -p "$OUT"; export TMPDIR=/tmp
for v in sv5vgpr svpad svmpad; do
  echo "== $v"; date
  VISSM_LIB=$ROOT/abl/lib_$v.so timeout -k 10 400 python3 scripts/sv_case_errs.py sv50 > "$OUT/$v.log" 2>&1 \
    || { echo "FAILED $v"; tail -n 5 "$OUT/$v.log"; exit 3; }
  grep -v "^\[vissm" "$OUT/$v.log" | cut -c1-260
done
echo "== posterior"; date
timeout -k 10 900 python -u -m pytest tests/test_gpu_posterior.py -m gpu -q -p no:cacheprovider -s --timeout 600 \
  --timeout-method thread > "$OUT/pytest_posterior.log" 2>&1; rc=$?
grep -E "seed|passed|failed" "$OUT/pytest_posterior.log" | cut -c1-200 | tail -n 12
date; exit $rc
