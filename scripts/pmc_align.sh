#!/bin/bash
# WRITE_SIZE of the bf16 flow kernels at an unaligned row length (T = 5000: L = 5025) and a 16-float-aligned one
# (T = 4999: L = 5024), flow micro-benchmark, one PMC pass per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
B=${B:-16384}
for T in 5000 4999; do
  cd /tmp && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -T --kernel-include-regex "bwd|fwd" -d "$OUT/align_$T" -o pmc --output-format csv -- python "$ROOT/scripts/flow_bench.py" --B $B --T $T --only bf16 --rounds 2 > "$OUT/align_$T.log" 2>&1 || { tail -20 "$OUT/align_$T.log"; exit 3; }
done
cd "$ROOT" && python - <<'PY'
import csv, glob
for T in (5000, 4999):
    rows = {}
    for f in glob.glob(f"gpurun_out/align_{T}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.setdefault(r["Kernel_Name"][:40], []).append(float(r["Counter_Value"]))
    for n, v in rows.items():
        print(T, n, "WRITE_SIZE KiB per launch", sum(v) / len(v), "launches", len(v))
PY
