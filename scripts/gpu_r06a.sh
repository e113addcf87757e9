#!/bin/bash
# Round-6 session a: the files the round-6 changes touch (observation list, feature kernels at 16 positions per block,
# theta-branch kernels on by default), then the full bench with its family lines.  Each step has its own limit; a
# fault ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06a; mkdir -p "$OUT"; export TMPDIR=/tmp
fault() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping: rc=$rc"; exit "$rc"; fi; }
echo "== pytest (changed areas)"; date
timeout -k 10 900 python -u -m pytest tests/test_gpu_elbo_models.py tests/test_gpu_feat.py tests/test_gpu_theta.py \
  tests/test_gpu_config_parity.py tests/test_gpu_fused.py tests/test_gpu_loop.py -m gpu -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
tail -4 "$OUT/pytest.log"; fault $rc
echo "== bench full"; date
timeout -k 10 900 python bench.py > "$OUT/bench_full.log" 2>&1 || { tail -20 "$OUT/bench_full.log"; exit 3; }
tail -1 "$OUT/bench_full.log" | cut -c1-400
echo "== rocprofv3 kernel trace (AR step, LV / FHN steps)"; date
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o bench --output-format csv -- python "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 4; }
date
echo "== rocprofv3 kernel trace, bf16x2f step"; date
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_x2f" -o bench --output-format csv -- python "$ROOT/bench.py" --steps 3 --warmup 1 --precision bf16x2f --cpu-baseline off --parity-line off --families off > "$OUT/prof_x2f.log" 2>&1 || { tail -20 "$OUT/prof_x2f.log"; exit 5; }
date
