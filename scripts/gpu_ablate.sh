#!/bin/bash
# Phase ablation timing of the v5 backward (results are wrong by construction; timing only).
# Masks are compile-time (scripts/build_ablate.sh -> abl_mask/lib_abl<mask>.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for L in viforssms_amd/libvissm.so abl_mask/lib_abl*.so viforssms_amd/libvissm.so; do
  echo -n "$L "
  VISSM_LIB=$PWD/$L timeout -k 10 300 python scripts/flow_bench.py --B 65536 --only bf16 --rounds 3 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['results']['bf16'])"
done
