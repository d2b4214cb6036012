"""Instruction mix of one kernel in a hipcc -save-temps gfx950 .s file, per basic block.

usage: python tools/isa_stats.py <file.s> <kernel-name-substring> [--loop] [--ops]
Prints, for every basic block (or only the hottest loop body with --loop: the block with the most MFMAs),
the count of each opcode class: mfma, valu, salu, lds, vmem, waitcnt, nop.
"""
from __future__ import annotations

import re
import sys
from collections import Counter, OrderedDict


def kernel_lines(path: str, sub: str) -> list[str]:
    lines = open(path).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", ln) and sub in ln.split(":")[0]:
            start = i
            continue
        if start is not None and (ln.startswith("\t.size") or re.match(r"^\.Lfunc_end", ln)):
            return lines[start:i]
    raise SystemExit(f"kernel matching {sub!r} not found")


def classify(op: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "accmov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op == "s_waitcnt":
        return "waitcnt"
    if op == "s_nop":
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def blocks(lines: list[str]) -> "OrderedDict[str, list[str]]":
    out: "OrderedDict[str, list[str]]" = OrderedDict()
    cur = "entry"
    out[cur] = []
    for ln in lines:
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        s = ln.strip()
        if not s or s.startswith((";", ".")):
            continue
        out[cur].append(s.split()[0])
    return out


def main() -> None:
    path, sub = sys.argv[1], sys.argv[2]
    bl = blocks(kernel_lines(path, sub))
    stats = {name: (Counter(classify(o) for o in ops), Counter(ops)) for name, ops in bl.items()}
    if "--loop" in sys.argv:
        name = max(stats, key=lambda k: stats[k][0]["mfma"])
        stats = {name: stats[name]}
    for name, (cls, ops) in stats.items():
        if not ops:
            continue
        print(f"{name}: " + " ".join(f"{k}={v}" for k, v in sorted(cls.items())))
        if "--loop" in sys.argv or "--ops" in sys.argv:
            for op, c in ops.most_common():
                print(f"    {op:32s} {c}")


if __name__ == "__main__":
    main()
