"""Instruction mix of one kernel's basic blocks in a --save-temps / -S assembly file, largest blocks first.
usage: isa_mix.py FILE.s MANGLED_NAME [min_block_len]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 100
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
blocks, cur = [], None
for line in s[i:j].split("\n"):
    t = line.strip()
    if re.match(r"^\.LBB\d+_\d+:", t) or t == name + ":":
        cur = [t.split(":")[0], [], line]
        blocks.append(cur)
        continue
    if cur is not None and t and not t.startswith((";", ".")):
        cur[1].append(t)


def cls(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if re.match(r"v_(exp|log|rcp|sqrt|rsq|sin|cos)_f32", op):
        return "trans"
    if op.startswith("v_cvt"):
        return "cvt"
    if op.startswith(("v_mov", "v_accvgpr")):
        return "mov"
    if op.startswith("v_pk_"):
        return "pk"
    if op.startswith(("v_cndmask", "v_med3", "v_max", "v_min")):
        return "select"
    if op.startswith(("v_perm", "v_lshl_or", "v_and_or", "v_bfi", "v_alignbit", "v_lshlrev", "v_lshrrev", "v_and_b", "v_or_b", "v_xor")):
        return "bitops"
    if op.startswith(("v_add_u", "v_add_co", "v_sub_u", "v_mad_u", "v_mul_lo", "v_lshl_add", "v_add3", "v_mad_i", "v_mul_hi", "v_add_i", "v_sub_i", "v_addc")):
        return "int"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "cmp"
    if op.startswith("v_"):
        return "valu_other_f"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


tot = collections.Counter()
for b in sorted(blocks, key=lambda b: -len(b[1])):
    if len(b[1]) < minlen:
        continue
    c = collections.Counter(cls(x.split()[0]) for x in b[1])
    tot += c
    print(b[0], len(b[1]), b[2].strip()[len(b[0]) + 1:].strip()[:60], dict(c.most_common()))
print("total of listed blocks", dict(tot.most_common()))
