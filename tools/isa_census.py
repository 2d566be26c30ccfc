"""Instruction census of one kernel in a device assembly file, per basic block.

usage: python tools/isa_census.py <file.s> <symbol-substring>
Prints every basic block with its VALU / SALU / LDS / VMEM counts (and the
LDS atomics), then the totals; the loop blocks are marked with their branch
target.  Used for the pass-A VALU census in DESIGN.md.
"""
from __future__ import annotations

import re
import sys


def blocks(path: str, sym: str):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(sym.split()[-1] + "E") is False or (l.startswith("_Z") and sym in l and ":" in l))
    out, cur, name = [], [], "entry"
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            out.append((name, cur))
            name, cur = m.group(1), []
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        cur.append(t.split(";")[0].strip())
    out.append((name, cur))
    return out


def classify(ins: str) -> str:
    op = ins.split()[0]
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path: str, sym: str) -> None:
    tot = {"valu": 0, "salu": 0, "lds": 0, "vmem": 0, "other": 0}
    for name, ins in blocks(path, sym):
        c = {k: 0 for k in tot}
        atom = 0
        br = ""
        for i in ins:
            c[classify(i)] += 1
            if i.startswith("ds_add"):
                atom += 1
            if i.startswith("s_cbranch") or i.startswith("s_branch"):
                br = i.split()[-1]
        for k in tot:
            tot[k] += c[k]
        print(f"{name:12s} n={len(ins):4d} valu={c['valu']:4d} salu={c['salu']:3d} lds={c['lds']:3d} (atomic {atom:2d}) "
              f"vmem={c['vmem']:3d} -> {br}")
    print("total", tot)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
