#!/bin/bash
# Round-6 session j: the split-weight forward (bf16x2f) with the hidden layer's hi planes register-resident in its
# 8-wave blocks (VISSM_X2_HIDREG) against the all-LDS form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06j; mkdir -p "$OUT"; export TMPDIR=/tmp
date
OUT=$OUT ROUNDS=3 STEPS=6 EXTRA="--precision bf16x2f" bash scripts/ab_step.sh abl/lib_cur.so abl/lib_hidreg.so
date
