#!/bin/bash
# FHN (k = 20, stride 2) step with the fused feature branch forced on (VISSM_FEAT_MAX_K=32) against the torch form,
# after the feature-kernel parity cases
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_feat.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_feat2.log 2>&1; tail -1 gpurun_out/pytest_feat2.log
for r in 1 2; do for mode in hip torch; do
  if [ $mode = hip ]; then e="VISSM_FEAT_MAX_K=32"; else e="VISSM_FEAT_TORCH=1"; fi
  env $e timeout -k 10 300 python bench.py --model fhn --steps 10 --warmup 2 --cpu-baseline off --parity-line off --families off > gpurun_out/feat_fhn.json 2>gpurun_out/feat_fhn.err || { tail -5 gpurun_out/feat_fhn.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/feat_fhn.json'));print('$mode fhn', round(d['ms_per_step'],3))"
done; done
