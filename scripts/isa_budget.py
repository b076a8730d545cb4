"""Static instruction budget of one kernel's basic blocks (a CPU study, not part of the library).

Usage: python scripts/isa_budget.py <file.s> <kernel-symbol-substring> [--blocks]

Compiles nothing: reads the assembly hipcc writes with -save-temps (see DESIGN.md 7.3 for the
recipe) and prints, per basic block of the kernel, its VALU / SALU / VMEM / LDS / branch counts,
with the source lines that block came from when the file carries .loc directives.  The per-step
budget in DESIGN.md 7.3 is these block counts grouped by what the block does.
"""
import re
import sys
from collections import OrderedDict


def classify(op):
    if op.startswith(("v_", )):
        return "valu"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_nop", "s_endpgm", "s_barrier", "s_sleep", "s_setprio")):
        return "other"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = None
    for i, l in enumerate(lines):
        if l.startswith(sym) or (sym in l and l.endswith(":") and l.startswith("_Z")):
            if sym in l.split(":")[0]:
                start = i
                break
    if start is None:
        sys.exit(f"kernel {sym} not found")
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = {"valu": 0, "salu": 0, "smem": 0, "vmem": 0, "lds": 0, "branch": 0, "other": 0, "locs": set(),
                   "loop": ""}
    loc = None
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end") or l.startswith("\t.section"):
            break
        m = re.match(r"^(\.LBB\w+|; %bb\.\d+):?\s*(;.*)?$", l)
        if m:
            cur = m.group(1)
            blocks[cur] = {"valu": 0, "salu": 0, "smem": 0, "vmem": 0, "lds": 0, "branch": 0, "other": 0,
                           "locs": set(), "loop": (m.group(2) or "").strip("; ")}
            continue
        m = re.match(r"^\s*\.loc\s+\d+\s+(\d+)", l)
        if m:
            loc = int(m.group(1))
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        k = classify(op)
        blocks[cur][k] += 1
        if loc is not None:
            blocks[cur]["locs"].add(loc)
    tot = {k: 0 for k in ("valu", "salu", "smem", "vmem", "lds", "branch")}
    print(f"{'block':<14} {'valu':>5} {'salu':>5} {'vmem':>5} {'lds':>4} {'br':>3}  loop / source lines")
    for b, c in blocks.items():
        for k in tot:
            tot[k] += c[k]
        locs = sorted(c["locs"])
        lr = f"{locs[0]}-{locs[-1]}" if locs else ""
        print(f"{b:<14} {c['valu']:>5} {c['salu']:>5} {c['vmem']:>5} {c['lds']:>4} {c['branch']:>3}  "
              f"{c['loop'][:40]} {lr}")
    print("total", tot)


if __name__ == "__main__":
    main()
