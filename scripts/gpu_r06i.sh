#!/bin/bash
# Round-6 session i: the LV / SV / FHN one-pass ELBO kernel with several waves per trajectory (stream_onepass_kernel
# NWV, VISSM_ELBO_NWV): parity at NWV = 2 and 4 against the two-launch form and the oracle, then each family's step at
# NWV = 1 / 2 / 4 (the kernel's live HBM fraction); the split-weight forward in 8- vs 4-wave blocks (bf16x2f).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r06i; mkdir -p "$OUT"; export TMPDIR=/tmp
PT="python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu"
for n in 2 4; do
  echo "== one-pass parity, NWV=$n"; date
  VISSM_ELBO_NWV=$n timeout -k 10 600 $PT tests/test_gpu_elbo_models.py -k "one_pass and not obs_list" > "$OUT/pytest_nwv$n.log" 2>&1; rc=$?
  tail -n 2 "$OUT/pytest_nwv$n.log"; [ $rc -eq 0 ] || exit $rc
done
echo "== family steps"; date
for rep in 1 2; do for m in sv fhn lv; do for n in 1 2 4; do
  VISSM_ELBO_NWV=$n timeout -k 10 300 python bench.py --model $m --steps 6 --warmup 2 --cpu-baseline off --parity-line off \
    --families off > "$OUT/b_${m}_$n.json" 2> "$OUT/b_${m}_$n.err" || { tail -5 "$OUT/b_${m}_$n.err"; exit 3; }
  python -c "
import json; d=json.load(open('$OUT/b_${m}_$n.json'))
s=[x for x in d['streaming_rooflines'] if 'onepass' in x['kernel']][0]
print('$m nwv=$n', round(d['ms_per_step'],2), 'elbo', round(s['avg_launch_ms']*1e3,1), 'us', round(s['frac'],3))"
done; done; done
echo "== bf16x2f forward blocks"; date
OUT=$OUT/x2f ROUNDS=2 STEPS=6 EXTRA="--precision bf16x2f" bash scripts/ab_step.sh abl/lib_cur.so abl/lib_nwf8.so
date
