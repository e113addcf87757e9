"""Summarise rocprofv3 PMC counter CSVs: per kernel, mean of each counter over dispatches."""
import csv, glob, os, sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            acc[row["Kernel_Name"][:60]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k)
    for c in sorted(m):
        print(f"   {c:28s} {m[c]:.4g}")
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VMEM", "SQ_VALU_MFMA_BUSY_CYCLES"):
            if c in m:
                print(f"   {c + '/WAVE_CYCLES':40s} {m[c] / wc:.3f}")
