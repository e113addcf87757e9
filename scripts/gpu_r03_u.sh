#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench (both ranks on the one GPU of this box, gloo instead of RCCL)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
VISSM_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --B 8192 --cpu-baseline off --family-steps 2 > "$OUT/dist2_r03.log" 2>&1 || { tail -30 "$OUT/dist2_r03.log"; exit 3; }
grep '^{' "$OUT/dist2_r03.log" | python -c "
import json,sys
d=json.loads(sys.stdin.readline()); print('ar', d['n_gpus'], round(d['ms_per_step'],2), '%.3e'%d['value'], d['config']['parallelism'])
for f in d.get('family_lines', []): print(f['model'], round(f['ms_per_step'],2), '%.3e'%f['value'], f['config']['parallelism'], f['config']['global_batch'])
"
