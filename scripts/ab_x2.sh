#!/bin/bash
# forward-kernel A/B of the bf16x2 (split-weight) variants in abl/*.so against bf16 / bf16x3 (flow micro-benchmark)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do for L in abl/*.so; do
  echo -n "$L "
  VISSM_LIB=$PWD/$L timeout -k 10 300 python scripts/flow_bench.py --B 65536 --impls bf16,bf16x2,bf16x3 --rounds 3 | python -c "import sys,json; d=json.loads(sys.stdin.read())['results']; print({k: (round(v['fwd_kernel_ms'],2), round(v['bwd_kernel_ms'],2), v.get('max_rel_diff_vs_bf16')) for k, v in d.items()})"
done; done
