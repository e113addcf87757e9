#!/bin/bash
# A/B timing of library builds in abl/*.so (alternating, same box; ROUNDS rounds, default 2); IMPL picks the
# flow precision (default bf16); extra env passes through
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 ${ROUNDS:-2}); do for L in abl/*.so; do
  echo -n "$L ${TAG:-} "
  VISSM_LIB=$PWD/$L timeout -k 10 300 python scripts/flow_bench.py --B 65536 --only ${IMPL:-bf16} --rounds 3 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['results']['${IMPL:-bf16}'])"
done; done
