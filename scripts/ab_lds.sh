#!/bin/bash
# LDS bank-conflict counters (one PMC pass per library, flow micro-benchmark) for abl/*.so, then the
# full-step A/B of the same libraries (scripts/ab_bench.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
for L in abl/*.so; do
  n=$(basename "$L" .so)
  echo "== pmc $n"
  cd /tmp && VISSM_LIB=$ROOT/$L timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --kernel-trace -T --kernel-include-regex "bwd_kernel|fwd_kernel" -d "$OUT/lds_$n" -o pmc --output-format csv -- python "$ROOT/scripts/flow_bench.py" --B 16384 --only bf16 --rounds 1 > "$OUT/lds_$n.log" 2>&1 || { tail -20 "$OUT/lds_$n.log"; exit 3; }
  cd "$ROOT" && python - "$OUT/lds_$n" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = "bwd" if "bwd_kernel" in r["Kernel_Name"] else "fwd"
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: "%.3e" % (sum(v) / len(v)) for c, v in d.items()})
PY
done
bash scripts/ab_bench.sh
