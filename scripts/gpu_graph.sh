#!/bin/bash
# Captured-graph step: GPU test against the eager step, then the paper-size AR bench eager vs graph.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
fault() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping: rc=$rc"; exit "$rc"; fi; }
timeout -k 10 300 python -m pytest tests/test_gpu_graph.py -x -q > $OUT/graph_pytest.log 2>&1; rc=$?
tail -30 $OUT/graph_pytest.log; fault $rc
for G in "" "--graph"; do
  timeout -k 10 200 python bench.py --B 50 --M 50 --k 50 --steps 50 --warmup 5 --precision bf16 --cpu-baseline off $G > $OUT/paper_graph.log 2>&1; rc=$?
  tail -1 $OUT/paper_graph.log | cut -c1-400; fault $rc
done
D=$(mktemp -d); cp -r dat hyperparameters.txt $D/ 2>/dev/null; chmod -R u+w $D; R=$PWD
(cd $D && timeout -k 10 300 python $R/main.py hyperparameters.txt --steps 200 --no-pretrain --precision bf16 --graph --log-every 50 > $R/$OUT/main_graph.log 2>&1); rc=$?
tail -3 $OUT/main_graph.log; fault $rc
