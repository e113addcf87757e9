#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -1 "$OUT/$name.log" | cut -c1-1500; if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi; }
run q_small python scripts/flow_bench.py --B 64 --T 200 --k 8 --nh 1 --impls 4,bf16,bf16x3 --rounds 2
run q_small_s2 python scripts/flow_bench.py --B 48 --T 150 --k 6 --nh 1 --stride2 --impls 4,bf16,bf16x3 --rounds 2
run q_ar_cfg python scripts/flow_bench.py --B 65536 --impls 4,bf16,bf16x3 --rounds 3 ${EXTRA}
