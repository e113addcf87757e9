#!/bin/bash
# Round-6 session g: the f16-derivative variants with the pairs pinned where they are computed (pin_pair): AR-cfg
# step A/B base / d1p / d1pns / d2pns, then LV and FHN base / d2pns.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06g; mkdir -p "$OUT"; export TMPDIR=/tmp
date
OUT=$OUT ROUNDS=2 STEPS=10 bash scripts/ab_step.sh abl/lib_base.so abl/lib_d1p.so abl/lib_d1pns.so abl/lib_d2pns.so
OUT=$OUT/lv ROUNDS=2 STEPS=6 EXTRA="--model lv" bash scripts/ab_step.sh abl/lib_base.so abl/lib_d2pns.so
OUT=$OUT/fhn ROUNDS=2 STEPS=6 EXTRA="--model fhn" bash scripts/ab_step.sh abl/lib_base.so abl/lib_d2pns.so
date
