#!/bin/bash
# Round-6 session n: SV's hand-written feature branch (ops.SvFeatConvFn: vissm_lv_mlp_* at four layers with the
# first-difference input, the conv as a split-bf16 GEMM, vissm_gemm_bf16x3): its tests, the SV / LV parity cases,
# then the SV-cfg step against the torch form (VISSM_SV_FEAT=torch) and a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06n; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 400 $PT tests/test_gpu_svfeat.py tests/test_gpu_lvfeat.py > "$OUT/pytest_feat.log" 2>&1; rc=$?
tail -n 3 "$OUT/pytest_feat.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $PT tests/test_gpu_config_parity.py tests/test_gpu_parity.py tests/test_gpu_feat.py -k "sv" > "$OUT/pytest_sv.log" 2>&1; rc=$?
tail -n 3 "$OUT/pytest_sv.log"; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --model sv --steps 10 --warmup 2 --cpu-baseline off --parity-line off --families off"
for r in 1 2; do
  VISSM_SV_FEAT=torch timeout -k 10 300 $B > "$OUT/bench_torch_$r.json" 2> "$OUT/bench_torch_$r.err" || exit 5
  timeout -k 10 300 $B > "$OUT/bench_hip_$r.json" 2> "$OUT/bench_hip_$r.err" || exit 6
  python -c "import json,sys; [print(f, json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step']) for f in sys.argv[1:]]" "$OUT/bench_torch_$r.json" "$OUT/bench_hip_$r.json"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_sv" -o sv --output-format csv -- python "$ROOT/bench.py" --model sv --steps 3 --warmup 1 --cpu-baseline off --parity-line off --families off > "$OUT/prof_sv.log" 2>&1 || exit 7
date
