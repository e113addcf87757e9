#!/bin/bash
# Round-5 session e: the fused last flow from its own translation unit (flow_v5f.hip, scheduler register-pressure
# trackers) -- the fused-flow parity tests on the production build, then the step A/B against the flow_v5.hip build
# of the fused kernels (VISSM_FUSED_TU=0), bf16 and bf16x2f.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r05e; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== fused parity"; date
timeout -k 10 900 python3 -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_pitch.py tests/test_gpu_config_parity.py -x -q -m gpu -p no:cacheprovider > "$OUT/pytest_fused.log" 2>&1; rc=$?
tail -3 "$OUT/pytest_fused.log"
[ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" "$OUT/pytest_fused.log" | head -20; exit $rc; }
echo "== step A/B"; date
OUT=$OUT ROUNDS=2 timeout -k 10 600 bash scripts/ab_step.sh abl/lib_fz.so abl/lib_nofz.so || exit 2
OUT=$OUT ROUNDS=1 EXTRA="--precision bf16x2f" timeout -k 10 600 bash scripts/ab_step.sh abl/lib_fz.so abl/lib_nofz.so || exit 3
date
