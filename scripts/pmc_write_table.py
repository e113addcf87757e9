"""WRITE_SIZE per flow-backward dispatch for each variant directory of scripts/gpu_ab_r05a.sh:
usage: python scripts/pmc_write_table.py OUTDIR VARIANT ...  (reads OUTDIR/pmcw_VARIANT/**/*counter_collection.csv)"""
import csv
import glob
import json
import os
import re
import sys

out, variants = sys.argv[1], sys.argv[2:]
table = {}
for v in variants:
    rows = []
    for f in glob.glob(os.path.join(out, f"pmcw_{v}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "WRITE_SIZE" or "bwd" not in r["Kernel_Name"]:
                continue
            n = r["Kernel_Name"]
            m = re.search(r"bwd2_kernel<(\w+), (\w+)", n)
            tag = ("fused" if m.group(1) == "true" else ("du" if m.group(2) == "true" else "no_du")) if m else n[:40]
            rows.append((int(r.get("Dispatch_Id", 0) or 0), tag, float(r["Counter_Value"]) * 1024 / 1e9))
    rows.sort()
    table[v] = [(t, round(gb, 3)) for _, t, gb in rows]
    print(v, table[v])
json.dump(table, open(os.path.join(out, "write_table.json"), "w"), indent=1)
