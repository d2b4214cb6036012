"""Per-tile VALU breakdown of an inference kernel's persistent loop, from a hipcc -save-temps gfx950 .s file.

usage: python tools/valu_breakdown.py <file.s> <kernel-name-substring>

The loop is the natural loop around the block with the most MFMAs (tools/isa_stats.py's blocks); one trip = one
32-query tile of one wave. Every VALU instruction of it is put in one bucket by opcode and context:
  relu_pack   the hidden layers' accumulator -> f16 B operand: compiler-visible v_cvt_pk_f16_f32 and the packed ReLU
              (v_pk_max_f16 / v_pk_max_i16)
  encoder     Composite encoding: everything inside inline-asm blocks (the |x| converts, the OneBlob bin index) and the
              f32 arithmetic of the TriangleWave / OneBlob formulas (fract, fma, mul, sub, med3, max, min, bit ops)
  epilogue    output layer combine and f16 -> f32 result (v_permlane32_swap, v_add_f32, v_cvt_f32_f16)
  address     tile / row indices, 64-bit offsets, compares, queue draw (v_*_u32, v_*_b64, v_cmp*, v_mbcnt*,
              v_readfirstlane, v_cndmask)
  move        v_mov_b32 / v_accvgpr moves
MFMAs are counted apart (SQ_INSTS_VALU of the PMC counts them too: VALU per MFMA there = (valu + mfma) / mfma).
"""
from __future__ import annotations

import json
import re
import sys
from collections import Counter

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import isa_stats  # noqa: E402


def loop_lines(path: str, sub: str, full: bool = False) -> list[tuple[str, bool]]:
    """(opcode, inside inline asm) of the loop blocks, in order (full: the whole instruction text instead)."""
    lines = isa_stats.kernel_lines(path, sub)
    # block boundaries and their instructions, keeping the asm flag
    blocks: dict[str, list[tuple[str, bool]]] = {"entry": []}
    order = ["entry"]
    succ: dict[str, set[str]] = {"entry": set()}
    cur, in_asm = "entry", False
    for ln in lines:
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            prev = cur
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            succ.setdefault(cur, set())
            # fall-through unless the previous block ended in an unconditional branch
            if blocks[prev] and not blocks[prev][-1][0].startswith(("s_branch", "s_endpgm")):
                succ[prev].add(cur)
            continue
        s = ln.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        blocks[cur].append((s if full else op, in_asm))
        t = re.search(r"(\.LBB\S+)", s)
        if op.startswith("s_branch") or op.startswith("s_cbranch"):
            if t:
                succ[cur].add(t.group(1))
    hot = max(order, key=lambda b: sum(1 for op, _ in blocks[b] if op.startswith("v_mfma")))
    # natural loop of the back edge(s) into any block that reaches hot and is reached from it: the blocks from which
    # hot is reachable AND which are reachable from hot
    def reach(src: str) -> set[str]:
        seen, todo = set(), [src]
        while todo:
            b = todo.pop()
            for t in succ.get(b, ()):
                if t not in seen:
                    seen.add(t)
                    todo.append(t)
        return seen

    fwd = reach(hot) | {hot}
    loop = [b for b in order if b in fwd and hot in reach(b) | ({hot} if b == hot else set())]
    return [x for b in loop for x in blocks[b]]


def clamp_registers(ins: list[tuple[str, bool]]) -> set[str]:
    """Third operands of v_med3_f32 shared by >= 16 instructions of the loop: the FP8 activation clamp (ReLU and
    saturation, med3(x, 0, 448.0) with 448.0 held in one register), not encoder arithmetic."""
    c = Counter(t.rsplit(",", 1)[-1].strip() for t, _ in ins if t.startswith("v_med3_f32"))
    regs = {r for r, n in c.items() if n >= 16}
    if sum(1 for t, _ in ins if t.startswith("v_cvt_scalef32_pk_fp8")) >= 16:
        regs.add("relu_e4m3")  # marker: the FP8 loop, whose v_perm / v_bitop3 / shifts by 8 are the byte ReLU
    return regs


def bucket(text: str, in_asm: bool, clamps: frozenset[str] = frozenset()) -> str | None:
    op = text.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if not op.startswith("v_"):
        return None
    if in_asm:
        return "encoder"
    if op.startswith(("v_cvt_pk_f16_f32", "v_pk_max_f16", "v_pk_max_i16", "v_cvt_pk_fp8_f32", "v_cvt_scalef32_pk_fp8")):
        return "relu_pack"
    if op.startswith("v_med3_f32") and text.rsplit(",", 1)[-1].strip() in clamps:
        return "relu_pack"
    if "relu_e4m3" in clamps and (op.startswith(("v_bitop3_b32", "v_perm_b32"))
                                  or (op.startswith("v_lshlrev_b32") and text.split()[2] == "8,")):
        return "relu_pack"  # the FP8 kernel's byte ReLU (relu_e4m3x4: shift, v_perm sign mask, and-not)
    if op.startswith(("v_permlane32_swap", "v_add_f32", "v_cvt_f32_f16")):
        return "epilogue"
    if op.startswith(("v_mov_b32", "v_accvgpr")):
        return "move"
    if op.startswith(("v_fract", "v_fma", "v_mul_f32", "v_sub_f32", "v_med3", "v_max_f32", "v_min_f32", "v_or_b32",
                      "v_and_b32", "v_perm_b32", "v_alignbit", "v_bfi", "v_cvt_flr", "v_lshl_or", "v_pk_mul_f16",
                      "v_pk_fma_f16", "v_cvt_f16", "v_ldexp")):
        return "encoder"
    return "address"


def main() -> None:
    path, sub = sys.argv[1], sys.argv[2]
    ins = loop_lines(path, sub, full=True)
    cl = frozenset(clamp_registers(ins))
    c = Counter(b for t, a in ins if (b := bucket(t, a, cl)))
    ops = Counter(t.split()[0] for t, a in ins if bucket(t, a, cl) == "address")
    valu = sum(v for k, v in c.items() if k != "mfma")
    out = {"kernel": sub, "per_tile": dict(c), "valu_non_mfma": valu, "mfma": c["mfma"],
           "valu_per_mfma_excl": valu / max(c["mfma"], 1),
           "pmc_style_valu_per_mfma": (valu + c["mfma"]) / max(c["mfma"], 1),
           "address_ops": dict(ops.most_common()),
           "opcodes": dict(Counter(t.split()[0] for t, a in ins if t.startswith("v_")).most_common())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
