#!/bin/bash
# bf16 flow kernels: cross-check vs fp32 kernels, parity vs oracle, timing at the AR config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -3 "$OUT/$name.log"; if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi; }
run v5_small python scripts/flow_bench.py --B 64 --T 200 --k 8 --nh 1 --impls 4,bf16,bf16x3 --rounds 2
run v5_small_s2 python scripts/flow_bench.py --B 48 --T 150 --k 6 --nh 1 --stride2 --impls 4,bf16,bf16x3 --rounds 2
run v5_k50 python scripts/flow_bench.py --B 40 --T 120 --k 50 --nh 1 --impls 4,bf16 --rounds 2
run v5_parity python scripts/parity_prec.py
run v5_ar_cfg python scripts/flow_bench.py --B 65536 --impls 4,bf16,bf16x3 --rounds 3
