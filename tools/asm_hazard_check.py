"""Inline-asm VALU -> MFMA hazard check on a hipcc -save-temps gfx950 .s file.

LLVM's hazard recognizer does not look inside inline asm: a VALU instruction written as inline asm whose result is
read by an MFMA (srcA / srcB / srcC) within 2 wait states gets no s_nop, and the MFMA reads the stale register
(found in round 2: the 16x16x32 inference kernel's second 16-query group read a half-converted encoder operand).
This scans every kernel for such pairs: for each MFMA it walks back over the previous instructions, counting wait
states (1 per instruction, N + 1 per s_nop N), and reports an inline-asm VALU def of one of its source registers
found within 2 wait states.

    python tools/asm_hazard_check.py <file.s> [<kernel-substring>]   # exit 1 if any hazard is found
"""
from __future__ import annotations

import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
WAIT_STATES = 2


def regs(text: str) -> set[tuple[str, int]]:
    out = set()
    for m in REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out.update((kind, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def scan(path: str, sub: str = "") -> list[str]:
    lines = open(path).read().splitlines()
    found = []
    kernel = None
    window: list[tuple[bool, str, int]] = []  # (from inline asm, instruction text, wait states it takes)
    in_asm = False
    for ln in lines:
        s = ln.strip()
        if re.match(r"^_Z\S*:", ln) or re.match(r"^[A-Za-z_]\w*:$", ln) and not ln.startswith("."):
            kernel = ln[:-1]
            window = []
            continue
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            if s.endswith(":"):
                window = []  # a label: predecessors unknown, be conservative only within a block
            continue
        if kernel is None or (sub and sub not in kernel):
            continue
        op = s.split()[0]
        if op.startswith("v_mfma"):
            operands = s[len(op):].split(",")
            srcs = regs(",".join(operands[1:]))
            ws = 0
            for is_asm, text, w in reversed(window):
                if ws >= WAIT_STATES:
                    break
                tok = text.split()
                if is_asm and tok and tok[0].startswith("v_"):
                    dst = regs(text[len(tok[0]):].split(",")[0])
                    if dst & srcs:
                        found.append(f"{kernel}: '{text}' -> '{s}' after {ws} wait state(s)")
                ws += w
        w = 1
        if op == "s_nop":
            w = int(s.split()[1], 0) + 1
        window.append((in_asm, s, w))
        window = window[-16:]
    return found


def main() -> None:
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    found = scan(path, sub)
    for f in found:
        print(f)
    print(f"{len(found)} inline-asm VALU -> MFMA hazard(s)")
    sys.exit(1 if found else 0)


if __name__ == "__main__":
    main()
