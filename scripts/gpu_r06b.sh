#!/bin/bash
# Round-6 session b: same-box A/B of the round-5 tree (abl/r05tree: git worktree of 5cee78d with its own library)
# against this tree -- the AR step twice each, alternating; the fused feature kernels' positions per block
# (VISSM_FEAT_KT / _BWD); LV / FHN steps with and without the observation list (VISSM_ELBO_OBS_LIST); then SV's
# k = 50 gradients under -amdgpu-mfma-vgpr-form=1 (scripts/gpu_sv_flag.sh).  Each step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06b; mkdir -p "$OUT"; export TMPDIR=/tmp
A=$ROOT/abl/r05tree
run() {  # name, dir, args...
  local name=$1 dir=$2; shift 2
  (cd "$dir" && timeout -k 10 300 python bench.py --cpu-baseline off --parity-line off --families off "$@") \
    > "$OUT/$name.log" 2>&1 || { echo "FAILED $name"; tail -5 "$OUT/$name.log"; exit 3; }
  python3 - "$OUT/$name.log" "$name" << 'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
r = d.get("roofline", {})
s = [(x["kernel"][:22], round(x["avg_launch_ms"], 4), round(x["frac"], 3)) for x in d.get("streaming_rooflines", [])]
print(sys.argv[2], round(d["ms_per_step"], 2), "ms", "bwd", round(r.get("avg_launch_ms", 0), 2), "fwd",
      round(r.get("fwd_kernel_avg_ms", 0), 2), s, flush=True)
PY
}
for rep in 1 2; do
  run r05_ar_$rep "$A" --steps 8 --warmup 2
  run cur_ar_$rep "$ROOT" --steps 8 --warmup 2
done
for kt in 8 16 32; do VISSM_FEAT_KT_BWD=$kt run cur_ar_ktb$kt "$ROOT" --steps 8 --warmup 2; done
VISSM_FEAT_KT=32 run cur_ar_ktf32 "$ROOT" --steps 8 --warmup 2
for m in lv fhn; do
  run r05_$m "$A" --model $m --steps 5 --warmup 2
  VISSM_ELBO_OBS_LIST=1 run cur_${m}_ol1 "$ROOT" --model $m --steps 5 --warmup 2
  VISSM_ELBO_OBS_LIST=0 run cur_${m}_ol0 "$ROOT" --model $m --steps 5 --warmup 2
done
bash scripts/gpu_sv_flag.sh || exit 4
date
