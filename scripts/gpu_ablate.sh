#!/bin/bash
# Phase ablation timing of the v5 backward (results are wrong by construction; timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for A in 0 1 2 4 8 16 31; do
  echo -n "abl=$A "
  VISSM_V5_ABLATE=$A timeout -k 10 300 python scripts/flow_bench.py --B 65536 --only bf16 --rounds 3 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['results']['bf16'])"
done
