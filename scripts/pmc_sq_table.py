"""Per-kernel averages of SQ counters from rocprofv3 --pmc CSVs (one or more passes), with the derived issue times:
VALU (4 cycles per wave64 instruction), MFMA busy, LDS, on 1024 SIMDs at 2.4 GHz.  usage: pmc_sq_table.py CSV..."""
import collections
import csv
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        m = re.search(r"(\w+_kernel)(<[^(]*>)?", name)
        key = (m.group(1) + (m.group(2) or "")) if m else name[:50]
        per[(int(r["Dispatch_Id"]), key)][r["Counter_Name"]] = float(r["Counter_Value"])
    for (_, key), cs in per.items():
        for c, v in cs.items():
            acc[key][c].append(v)
rows = []
for key, cs in acc.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    n = max(len(v) for v in cs.values())
    t = avg.get("GRBM_GUI_ACTIVE", 0) / 8 / 2.4e9 * 1e3
    rows.append((t * n, key, n, avg, t))
rows.sort(reverse=True)
for _, key, n, avg, t in rows[:12]:
    print(f"{key}  launches={n}  gui_active_ms~{t:.3f}")
    for c in sorted(avg):
        print(f"    {c:28s} {avg[c]:.4g}")
    if "SQ_INSTS_VALU" in avg:
        v = avg["SQ_INSTS_VALU"] * 4 / (1024 * 2.4e9) * 1e3
        mf = avg.get("SQ_INSTS_MFMA", 0)
        print(f"    -> VALU issue {v:.3f} ms; VALU/MFMA {avg['SQ_INSTS_VALU'] / max(mf, 1):.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        print(f"    -> MFMA busy {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * 2.4e9) * 1e3:.3f} ms (if per-SIMD cycles summed)")
