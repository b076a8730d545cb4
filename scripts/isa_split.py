"""The certified bounce walk's per-step VALU by what it does (a CPU study): the hot basic blocks of
k_bounce_trav<false, 2, false, false, true, false> (the certified 4-wide walk) in the assembly hipcc writes with -S,
their VALU by opcode class.  The QNode step is one block (the four slack tests, the margins, the sort, the pushes),
the leaf test another; .loc lines are not used (inlining and scheduling blur them).

usage: python scripts/isa_split.py <trace.s> [kernel-symbol-prefix] [min-VALU]"""
import re
import sys
from collections import Counter

CLASSES = [
    ("plane bytes -> float (v_cvt_f32_ubyte*)", lambda o: o.startswith("v_cvt_f32_ubyte")),
    ("fma / mul / add (slab distances, margins, triangle test)", lambda o: re.match(r"v_(pk_)?(fma|fmac|fmamk|fmaak|mul|add|sub|subrev|mad)_f32", o)),
    ("max3 / min3 / max / min", lambda o: re.match(r"v_(max3|min3|max|min|med3)_f32", o)),
    ("compares (v_cmp*)", lambda o: o.startswith("v_cmp")),
    ("selects (v_cndmask)", lambda o: o.startswith("v_cndmask")),
    ("integer / bit ops (ids, keys, addresses)", lambda o: re.match(r"v_(and|or|xor|lshl|lshr|ashr|bfe|bfi|alignbit|perm|add_u32|add_co|addc|sub_u32|sub_co|subb|mul_lo|mul_hi|mad_u|lshl_add|lshl_or|and_or|or3|add3|not|bcnt|mbcnt|ffbh|ffbl|min_u|max_u|min_i|max_i|cvt_u32|cvt_i32|cvt_f32_u32|cvt_f32_i32)", o)),
    ("moves / lane ops (v_mov, readlane, writelane, readfirstlane)", lambda o: re.match(r"v_(mov|readlane|writelane|readfirstlane|accvgpr)", o)),
    ("reciprocal / division helpers", lambda o: re.match(r"v_(rcp|div_|frexp|ldexp|rsq|sqrt)", o)),
]


def classify(op):
    for name, f in CLASSES:
        if f(op):
            return name
    return "other VALU"


def main(asm, prefix="_ZN5rtbvh12_GLOBAL__N_113k_bounce_travILb0ELi2ELb0ELb0ELb1ELb0E", minv=10):
    s = open(asm).read().split("\n")
    start = next(i for i, l in enumerate(s) if l.startswith(prefix) and l.split(";")[0].rstrip().endswith(":"))
    end = next(i for i in range(start, len(s)) if s[i].strip().startswith(".Lfunc_end"))
    blocks, cur, name, note = [], None, "entry", ""
    for l in s[start:end]:
        m = re.match(r"^(\.LBB\S+):(.*)$", l) or re.match(r"^; (%bb\.\d+):(.*)$", l)
        if m:
            cur = Counter()
            blocks.append((m.group(1), m.group(2).strip(), cur))
            continue
        t = l.strip()
        if cur is not None and t.startswith("v_"):
            cur[classify(t.split()[0])] += 1
    for b, note, c in blocks:
        v = sum(c.values())
        if v >= minv:
            print("%-12s %4d VALU  %s" % (b, v, note[:60]))
            for k, n in c.most_common():
                print("      %-62s %4d" % (k, n))


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []), *([int(sys.argv[3])] if len(sys.argv) > 3 else []))
