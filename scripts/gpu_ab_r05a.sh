#!/bin/bash
# Round-5 A/B session: (1) the streaming log-density kernels (two launches vs the one-pass vissm_elbo_fwd_grad;
# default build vs -fno-slp-vectorize), (2) per-buffer attribution of the AR backward's PMC WRITE_SIZE (timing-only
# builds without the fused flow's x / du stores or the dC slab stores, and dword du stores instead of 16-byte ones),
# one bench step per variant.  Each GPU step has its own limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/r05a; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "== elbo A/B"; date
ROUNDS=2 timeout -k 10 400 bash scripts/ab_elbo.sh abl/lib_base.so abl/lib_noslp.so abl/lib_kv8.so abl/lib_kv8noslp.so > "$OUT/ab_elbo.log" 2>&1 || { tail -20 "$OUT/ab_elbo.log"; exit 2; }
cat "$OUT/ab_elbo.log"
echo "== step A/B: shared head backward (base) vs per-sample (hs0), 16-byte du stores vs dword (dux4off)"; date
OUT=$OUT ROUNDS=2 STEPS=8 timeout -k 10 900 bash scripts/ab_step.sh abl/lib_base.so abl/lib_hs0.so abl/lib_dux4off.so \
    > "$OUT/ab_step.log" 2>&1 || { tail -20 "$OUT/ab_step.log"; exit 4; }
cat "$OUT/ab_step.log"
for v in base dux4off nox nodu nodc; do
  echo "== WRITE_SIZE $v"; date
  cd /tmp && VISSM_LIB=$ROOT/abl/lib_$v.so timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -T \
      --kernel-include-regex "bwd" -d "$OUT/pmcw_$v" -o pmc --output-format csv -- python3 "$ROOT/bench.py" --steps 1 \
      --warmup 0 --cpu-baseline off --parity-line off --families off > "$OUT/pmcw_$v.log" 2>&1 \
      || { tail -20 "$OUT/pmcw_$v.log"; exit 3; }
  cd "$ROOT"
done
python3 scripts/pmc_write_table.py "$OUT" base dux4off nox nodu nodc
date
