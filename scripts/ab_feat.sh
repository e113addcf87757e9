cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_feat.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_feat.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_feat.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
for m in 0 1 0 1; do
  for model in ar fhn sv; do
    VISSM_FEAT_TORCH=$m timeout -k 10 300 python bench.py --model $model --steps 10 --warmup 2 --cpu-baseline off --parity-line off --families off > gpurun_out/feat_ab.json 2>gpurun_out/feat_ab.err || { tail -5 gpurun_out/feat_ab.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/feat_ab.json'));print('torch' if '$m'=='1' else 'hip', '$model', round(d['ms_per_step'],3), d['value'])" >> gpurun_out/feat_ab.log
  done
done
cat gpurun_out/feat_ab.log
