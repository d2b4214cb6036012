"""ISA hazard checks on a hipcc -save-temps / --cuda-device-only -S gfx950 .s file. Three rules:

1. Inline-asm VALU -> MFMA (`scan`). LLVM's hazard recognizer does not look inside inline asm: a VALU instruction
   written as inline asm whose result is read by an MFMA (srcA / srcB / srcC) within 2 wait states gets no s_nop, and
   the MFMA reads the stale register (found in round 2: the 16x16x32 inference kernel's second 16-query group read a
   half-converted encoder operand). For each MFMA walk back over the previous instructions, counting wait states
   (1 per instruction, N + 1 per s_nop N), and report an inline-asm VALU def of one of its source registers found
   within 2 wait states.

2. Inline-asm vector-memory loads (`scan_loads`). The compiler does not know that an inline-asm `global_load` /
   `buffer_load` is still in flight after the asm statement: it treats the destination VGPRs as written, so it may
   read them (a copy, a spill) or reuse them (as an address, a temporary) before the data lands, and the data then
   overwrites whatever the registers hold by then (found in round 3: a timing ablation of the Hash feature pass faulted
   the GPU). For every inline-asm load this walks forward in program order to the first `s_waitcnt vmcnt(N)` that
   covers it (N <= the vector-memory instructions issued after it: at most N are outstanding, the N youngest,
   as loads return in order) and reports any instruction
   in that window that reads or writes one of its destination VGPRs, and any label or branch in the window (the walk
   does not follow control flow, so a window that crosses one is reported as unverifiable).

3. Scalar-branch prefetch + exec-masked store region in one loop (`scan_branch_store_loops`). The round-1 Hash
   inference shape corrupted whole 32-query tiles when one loop of a wave held both a global load under a scalar
   branch (s_cbranch_scc*/s_cbranch_vcc*) and a global store under a modified exec mask (s_and_saveexec / s_cbranch_execz
   region); either alone was clean (five GPU probes). The cause was never isolated, so no product
   kernel may contain that combination: for every natural loop of the control-flow graph (a back edge to a dominating
   block), report it if a scalar conditional branch (s_cbranch_scc*/vcc*) inside it leads to a block holding a
   vector-memory load and an s_cbranch_execz inside it falls through to a block holding a vector-memory store (the
   exec-masked region the compiler emits for a divergent `if`).

    python tools/asm_hazard_check.py <file.s> [<kernel-substring>]   # exit 1 if any rule reports
"""
from __future__ import annotations

import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
WAIT_STATES = 2
VMEM_PREFIX = ("global_", "buffer_", "flat_", "scratch_")


def regs(text: str) -> set[tuple[str, int]]:
    out = set()
    for m in REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out.update((kind, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _strip_comment(s: str) -> str:
    i = s.find(";")
    return s[:i].rstrip() if i >= 0 else s


def kernels(path: str) -> dict[str, list[tuple[bool, str]]]:
    """Per function: its instructions and labels in order as (from inline asm, text); labels keep their trailing ':'."""
    out: dict[str, list[tuple[bool, str]]] = {}
    cur = None
    in_asm = False
    for ln in open(path).read().splitlines():
        s = ln.strip()
        if re.match(r"^_Z\S*:", ln) or (re.match(r"^[A-Za-z_]\w*:$", ln) and not ln.startswith(".")):
            cur = ln.strip()[:-1]
            out[cur] = []
            continue
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if cur is None or not s or s.startswith((";", ".")) and not s.startswith(".LBB"):
            continue
        if s.startswith(".Lfunc_end"):
            cur = None
            continue
        s = _strip_comment(s)
        if s:
            out[cur].append((in_asm, s))
    return out


def scan(path: str, sub: str = "") -> list[str]:
    """Rule 1: inline-asm VALU -> MFMA within 2 wait states."""
    found = []
    for kernel, body in kernels(path).items():
        if sub and sub not in kernel:
            continue
        window: list[tuple[bool, str, int]] = []  # (from inline asm, instruction text, wait states it takes)
        for in_asm, s in body:
            if s.endswith(":"):
                window = []  # a label: predecessors unknown, be conservative only within a block
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


def _is_vmem(op: str) -> bool:
    return op.startswith(VMEM_PREFIX)


def _vmcnt(s: str) -> int | None:
    if not s.startswith("s_waitcnt"):
        return None
    m = re.search(r"vmcnt\((\d+)\)", s)
    if m:
        return int(m.group(1))
    if re.fullmatch(r"s_waitcnt\s+0", s):
        return 0
    return None


def scan_loads(path: str, sub: str = "") -> tuple[list[str], int]:
    """Rule 2: returns (findings, number of inline-asm loads checked)."""
    found = []
    checked = 0
    for kernel, body in kernels(path).items():
        if sub and sub not in kernel:
            continue
        for i, (in_asm, s) in enumerate(body):
            if not in_asm or s.endswith(":"):
                continue
            op = s.split()[0]
            if not (op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")) and "lds" not in op):
                continue
            checked += 1
            dst = regs(s[len(op):].split(",")[0])
            younger = 0
            covered = False
            for _, t in body[i + 1:]:
                if t.endswith(":"):
                    found.append(f"{kernel}: '{s}': label {t} before the covering s_waitcnt")
                    break
                top = t.split()[0]
                n = _vmcnt(t)
                if n is not None and younger >= n:  # at most n outstanding = the n youngest: this one has landed
                    covered = True
                    break
                if top.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
                    found.append(f"{kernel}: '{s}': '{t}' before the covering s_waitcnt")
                    break
                if regs(t[len(top):]) & dst:
                    found.append(f"{kernel}: '{s}': '{t}' touches its destination while the load is in flight")
                if _is_vmem(top):
                    younger += 1
            else:
                if not covered:
                    found.append(f"{kernel}: '{s}': no covering s_waitcnt before the end of the function")
    return found, checked


def _blocks(body: list[tuple[bool, str]]):
    """Basic blocks of one function: (instructions, successor block indices, terminator)."""
    starts = [0]
    for k, (_, t) in enumerate(body):
        if t.endswith(":") and k:
            starts.append(k)
        elif t.split()[0].startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")) and k + 1 < len(body):
            starts.append(k + 1)
    starts = sorted(set(starts))
    spans = [(a, b) for a, b in zip(starts, starts[1:] + [len(body)]) if a < b]
    label_block = {}
    for bi, (a, b) in enumerate(spans):
        if body[a][1].endswith(":"):
            label_block[body[a][1][:-1]] = bi
    blocks = []
    for bi, (a, b) in enumerate(spans):
        ins = [t for _, t in body[a:b] if not t.endswith(":")]
        last = ins[-1] if ins else ""
        op = last.split()[0] if last else ""
        succ = []
        if op.startswith(("s_branch", "s_cbranch")):
            tgt = last.split()[-1]
            if tgt in label_block:
                succ.append(label_block[tgt])
            if op.startswith("s_cbranch") and bi + 1 < len(spans):
                succ.append(bi + 1)
        elif op not in ("s_setpc_b64", "s_endpgm") and bi + 1 < len(spans):
            succ.append(bi + 1)
        blocks.append((ins, succ, op))
    return blocks


def _natural_loops(blocks) -> list[set[int]]:
    n = len(blocks)
    if n == 0:
        return []
    preds: list[list[int]] = [[] for _ in range(n)]
    for b, (_, succ, _) in enumerate(blocks):
        for t in succ:
            preds[t].append(b)
    full = set(range(n))
    dom = [full.copy() for _ in range(n)]
    dom[0] = {0}
    changed = True
    while changed:
        changed = False
        for b in range(1, n):
            ps = [dom[p] for p in preds[b]]
            nd = (set.intersection(*ps) if ps else set()) | {b}
            if nd != dom[b]:
                dom[b] = nd
                changed = True
    loops = []
    for u in range(n):
        for h in blocks[u][1]:
            if h in dom[u]:  # back edge u -> h
                # the blocks that reach u without passing h; a self-loop (u == h) is that block alone (walking its
                # predecessors would take in the loop's entry path and everything before it)
                body = {h, u}
                stack = [u] if u != h else []
                while stack:
                    x = stack.pop()
                    for p in preds[x]:
                        if p not in body:
                            body.add(p)
                            stack.append(p)
                loops.append(body)
    return loops


def scan_branch_store_loops(path: str, sub: str = "") -> list[str]:
    """Rule 3: a natural loop (back edge to a dominating block) holding a load in a block entered by a scalar
    conditional branch and a store in the region an s_cbranch_execz skips."""
    found = []

    def has(ins: list[str], kind: str) -> bool:
        return any(_is_vmem(t.split()[0]) and kind in t.split()[0] and "lds" not in t.split()[0] for t in ins)

    for kernel, body in kernels(path).items():
        if sub and sub not in kernel:
            continue
        blocks = _blocks(body)
        for loop in _natural_loops(blocks):
            skipped_load = masked_store = None
            for b in sorted(loop):
                ins, succ, op = blocks[b]
                if op.startswith(("s_cbranch_scc", "s_cbranch_vcc")) and all(t in loop for t in succ):
                    if any(has(blocks[t][0], "load") for t in succ):
                        skipped_load = ins[-1]
                if op == "s_cbranch_execz" and b + 1 in loop and has(blocks[b + 1][0], "store"):
                    masked_store = ins[-1]
            if skipped_load and masked_store:
                found.append(f"{kernel}: loop of {len(loop)} blocks: load behind '{skipped_load}', store behind "
                             f"'{masked_store}'")
    return found


def main() -> None:
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    f1 = scan(path, sub)
    f2, n2 = scan_loads(path, sub)
    f3 = scan_branch_store_loops(path, sub)
    for f in f1 + f2 + f3:
        print(f)
    print(f"{len(f1)} inline-asm VALU -> MFMA hazard(s); {len(f2)} inline-asm load window violation(s) over {n2} "
          f"load(s); {len(f3)} scalar-branch-load + masked-store loop(s)")
    sys.exit(1 if (f1 or f2 or f3) else 0)


if __name__ == "__main__":
    main()
