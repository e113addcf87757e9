#!/bin/bash
# SV's k = 50 parity cases (5 flows and 1 flow) with every variable's gradient error, on the tree's library and on
# abl/lib_sv5vgpr.so (flow_v5s.hip built with -mllvm -amdgpu-mfma-vgpr-form=1): which gradients the flag breaks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/svflag; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/sv_case_errs.py sv50 --all > "$OUT/tree.log" 2>&1 || exit 3
VISSM_LIB=$(pwd)/abl/lib_sv5vgpr.so timeout -k 10 300 python3 scripts/sv_case_errs.py sv50 --all > "$OUT/vgpr.log" 2>&1 || exit 4
tail -n 3 "$OUT/tree.log"; tail -n 3 "$OUT/vgpr.log"
