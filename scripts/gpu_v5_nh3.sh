#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -12 "$OUT/$name.log" | cut -c1-700; if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi; }
run n3_small python scripts/flow_bench.py --B 48 --T 150 --k 6 --nh 3 --stride2 --impls 2,bf16 --rounds 2
run n3_k20 python scripts/flow_bench.py --B 40 --T 200 --k 20 --nh 3 --stride2 --impls 2,bf16 --rounds 2
run n3_k50 python scripts/flow_bench.py --B 40 --T 120 --k 50 --nh 3 --impls 2,bf16 --rounds 2
run parity python scripts/parity_prec.py
run n3_lv python scripts/flow_bench.py --B 4096 --k 20 --nh 3 --stride2 --impls 2,bf16 --rounds 3
run ar_cfg python scripts/flow_bench.py --B 65536 --impls 4,bf16 --rounds 3
