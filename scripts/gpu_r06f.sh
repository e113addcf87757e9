#!/bin/bash
# Round-6 session f: AR-cfg step A/B -- base (the production build: no f16 derivatives), ns (flow_v5 / flow_v5f
# without the SLP vectorizer), d1 / d1ns (elu'(A0) as f16 pairs, VISSM_DERIV16=1, with / without SLP).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06f; mkdir -p "$OUT"; export TMPDIR=/tmp
date
OUT=$OUT ROUNDS=2 STEPS=10 bash scripts/ab_step.sh abl/lib_base.so abl/lib_ns.so abl/lib_d1.so abl/lib_d1ns.so
date
