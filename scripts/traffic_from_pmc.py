"""HBM traffic per launch of the flow backward kernel from the FETCH_SIZE and WRITE_SIZE
rocprofv3 passes (gpurun_out/pmc_FETCH_SIZE, gpurun_out/pmc_WRITE_SIZE) -> profiles/traffic.json.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the bytes of wide
streaming reads (MI355X_MICROARCH.md, HBM section): it is doubled here.
usage: python scripts/traffic_from_pmc.py PRECISION B T k"""
import csv, glob, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prec, B, T, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])


def per_launch(counter):
    vals = []
    for f in glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{counter}", "**", "*counter_collection.csv"),
                       recursive=True):
        for row in csv.DictReader(open(f)):
            n = row["Kernel_Name"]
            flow_bwd = n.startswith(("bwd_kernel", "bwd2_kernel", "bwd2n_kernel")) or ("flow5" in n and "bwd" in n)
            if flow_bwd and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None, len(vals)


fetch, nf = per_launch("FETCH_SIZE")
write, nw = per_launch("WRITE_SIZE")
if fetch is None or write is None:
    sys.exit("no bwd_kernel counter rows found")
bytes_per_launch = (2.0 * fetch + write) * 1024.0
path = os.path.join(ROOT, "profiles", "traffic.json")
d = json.load(open(path)) if os.path.exists(path) else {}
d[prec] = {"B": B, "T": T, "k": k, "bytes_per_launch": bytes_per_launch, "fetch_kib_raw": fetch,
           "write_kib": write, "launches": [nf, nw],
           "note": "flow backward (bwd2_kernel at the AR shapes); FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, "
                   "mean over the step's launches"}
json.dump(d, open(path, "w"), indent=1)
print(json.dumps(d[prec]))
