"""Instruction mix per basic block of one kernel in a hipcc --save-temps .s file (CPU-side analysis:
which blocks carry the per-unit work and how many VALU / MFMA / LDS / SALU / VMEM instructions they issue).
usage: python scripts/asm_mix.py file.s kernel_substring [min_block_insts]"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if re.match(r"^_Z\w*:", l) and name in l:
            start = i
            break
    if start is None:
        sys.exit("kernel not found")
    blocks, cur, label = [], Counter(), "entry"
    ops = {}
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            blocks.append((label, cur, ops))
            cur, label, ops = Counter(), m.group(1), {}
            continue
        t = l.strip()
        if not t or t.startswith((";", ".", "//")):
            continue
        op = t.split()[0]
        c = classify(op)
        cur[c] += 1
        ops[op] = ops.get(op, 0) + 1
    blocks.append((label, cur, ops))
    tot = Counter()
    for label, c, ops in blocks:
        n = sum(c.values())
        tot += c
        if n >= mn:
            print(f"{label:24s} n={n:5d} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
            if "-v" in sys.argv:
                for op, v in sorted(ops.items(), key=lambda x: -x[1])[:40]:
                    print(f"      {op:36s} {v}")
    print("TOTAL", sum(tot.values()), dict(tot))


if __name__ == "__main__":
    main()
