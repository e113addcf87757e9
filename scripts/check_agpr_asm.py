"""Hazard audit of the inline-asm accumulator MFMAs (flow_v5.hip mfma32_a* / agpr_drain4): hipcc pads no hazard for an
asm statement, so every instruction the COMPILER emits that touches an AGPR an asm MFMA writes must be reachable from
an asm MFMA only through a drain statement (its 12 wait states), never directly.

usage: python scripts/check_agpr_asm.py [file.s ...]
With no argument it compiles viforssms_amd/csrc/flow_v5n.hip (the translation unit whose kernels carry asm MFMAs) to
device assembly with the Makefile's flags and audits every kernel that contains one.  Exit status 1 on a violation."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "viforssms_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=fast", "--offload-arch=gfx950", "--cuda-device-only", "-S"]
SOURCES = {"flow_v5n.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form=1"]}   # the TU with asm MFMAs


def agprs(tok):
    m = re.match(r"a\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"a(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def kernels(text):
    cur, out = None, {}
    for line in text.split("\n"):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is not None:
            t = line.strip()
            if t.startswith(".Lfunc_end"):
                cur = None
                continue
            out[cur].append(t)
    return out


def audit(name, body):
    """(n asm MFMA statements, violations): over the kernel's control-flow graph, a compiler instruction that reads or
    writes an AGPR which an asm MFMA wrote fewer than 12 wait states earlier on some path (no drain in between)."""
    # instructions as (kind, text): kind asm_mfma / drain / compiler / label / branch
    items, inasm, block = [], False, []
    for t in body:
        if t.startswith(";;#ASMSTART"):
            inasm, block = True, []
            continue
        if t.startswith(";;#ASMEND"):
            inasm = False
            if any(x.startswith("v_mfma") for x in block):
                items.append(("asm_mfma", block))
            elif any(x.startswith("s_nop 7") for x in block):
                items.append(("drain", block))
            continue
        if inasm:
            block.append(t)
            continue
        if not t or t.startswith(";") or (t.startswith(".") and not re.match(r"^\.LBB\w+:", t)):
            continue
        m = re.match(r"^(\.LBB\w+):", t)
        items.append(("label", m.group(1)) if m else ("compiler", t))
    owned = set()
    for k, v in items:
        if k == "asm_mfma":
            for x in v:
                if x.startswith("v_mfma"):
                    owned |= agprs(x.split()[1].rstrip(","))
    n_asm = sum(1 for k, _ in items if k == "asm_mfma")
    if not n_asm:
        return 0, []
    # basic blocks
    blocks, cur = [], {"label": None, "items": []}
    for k, v in items:
        if k == "label":
            blocks.append(cur)
            cur = {"label": v, "items": []}
            continue
        cur["items"].append((k, v))
        if k == "compiler" and (v.startswith("s_branch") or v.startswith("s_cbranch") or v.startswith("s_endpgm")):
            blocks.append(cur)
            cur = {"label": None, "items": []}
    blocks.append(cur)
    blocks = [b for b in blocks if b["label"] is not None or b["items"]]
    index = {b["label"]: i for i, b in enumerate(blocks) if b["label"]}
    succ = []
    for i, b in enumerate(blocks):
        s = []
        last = b["items"][-1][1] if b["items"] and b["items"][-1][0] == "compiler" else ""
        if last.startswith("s_branch"):
            s.append(index[last.split()[1]])
        elif last.startswith("s_endpgm"):
            pass
        else:
            if last.startswith("s_cbranch"):
                s.append(index[last.split()[1]])
            if i + 1 < len(blocks):
                s.append(i + 1)
        succ.append(s)
    pred = [[] for _ in blocks]
    for i, ss in enumerate(succ):
        for j in ss:
            pred[j].append(i)

    def states(k, v):
        if k != "compiler":
            return 1
        m = re.match(r"s_nop (\d+)", v)
        return int(m.group(1)) + 1 if m else 1

    def written(k, v):
        if k != "asm_mfma":
            return set()
        out = set()
        for x in v:
            if x.startswith("v_mfma"):
                out |= agprs(x.split()[1].rstrip(","))
        return out

    def recent_mfma_writes(bi, pos, regs, budget):
        """True if an asm MFMA writing one of regs lies within `budget` wait states before item pos of block bi
        (a drain statement ends the search: its nops cover every MFMA before it)."""
        stack, seen = [(bi, pos, budget)], set()
        while stack:
            b, p, left = stack.pop()
            items = blocks[b]["items"]
            q = p - 1
            while q >= 0 and left > 0:
                k, v = items[q]
                if k == "drain":
                    break
                if written(k, v) & regs:
                    return True
                left -= states(k, v)
                q -= 1
            else:
                if left > 0 and q < 0:
                    for pb in pred[b]:
                        if (pb, left) not in seen:
                            seen.add((pb, left))
                            stack.append((pb, len(blocks[pb]["items"]), left))
        return False

    bad = []
    for bi, b in enumerate(blocks):
        for pos, (k, v) in enumerate(b["items"]):
            if k != "compiler":
                continue
            used = set()
            for x in v.split()[1:]:
                used |= agprs(x.rstrip(","))
            # an 8-pass MFMA's D: 12 wait states before any other reader / writer (the asm's own next MFMA aside)
            if used & owned and recent_mfma_writes(bi, pos, used, 12):
                bad.append(v)
    return n_asm, bad


def main():
    files = sys.argv[1:]
    tmp = None
    if not files:
        tmp = tempfile.mkdtemp()
        for src, extra in SOURCES.items():
            out = os.path.join(tmp, src.replace(".hip", ".s"))
            subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-I" + os.path.join(ROOT, "include"), "-o", out,
                            os.path.join(CSRC, src)], check=True, cwd=CSRC)
            files.append(out)
    ok = True
    for f in files:
        for name, body in kernels(open(f).read()).items():
            n, bad = audit(name, body)
            if n:
                print(f"{os.path.basename(f)} {name[:70]}: {n} asm MFMA statements, {len(bad)} unpadded compiler "
                      f"accesses to their AGPRs")
                for v in bad[:10]:
                    print("    ", v)
                ok = ok and not bad
    print("OK" if ok else "VIOLATIONS")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
