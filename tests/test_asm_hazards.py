"""ISA hazard rules on the product kernels (tools/asm_hazard_check.py).

Compiles every gfx950 translation unit of libnrc_amd.so to assembly (hipcc cross-compiles without a GPU) and requires:
1. no inline-asm VALU whose result an MFMA reads within 2 wait states (LLVM's hazard recognizer does not see inside
   inline asm; round 2);
2. no inline-asm vector-memory load whose destination VGPRs any instruction reads or writes before the s_waitcnt that
   covers it, and no such window crossing a branch or label (the compiler does not know the load is in flight; the
   round-3 Hash feature-pass ablation faulted the GPU this way — DESIGN.md §10);
3. no loop holding both a load behind a scalar conditional branch and a store behind an s_cbranch_execz (the pair that
   was necessary and sufficient for the round-1 Hash shape's corrupted tiles, cause not isolated — DESIGN.md §10).
Rules 2 and 3 are also checked against small hand-written .s fragments in the shape of the faulting / corrupting
builds, so a checker that silently stops matching fails here."""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "neural-radiance-caching_amd"
sys.path.insert(0, str(ROOT / "tools"))
import asm_hazard_check  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"
# (source, extra flags) as the Makefile builds them for libnrc_amd.so
UNITS = [("nrc_kernels.hip", []), ("nrc_train16.hip", ["-mllvm", "-amdgpu-mfma-vgpr-form"]),
         ("nrc_train_dc.hip", ["-mllvm", "-amdgpu-mfma-vgpr-form"]), ("nrc_frame.hip", []),
         ("nrc_infer16.hip", ["-mllvm", "-amdgpu-mfma-vgpr-form"])]

_ASM: dict[str, Path] = {}


def _compile(tmp_path_factory, src: str, flags: list[str]) -> Path:
    if src not in _ASM:
        out = tmp_path_factory.mktemp("asm") / (src + ".s")
        kflags = [] if src == "nrc_frame.hip" else ["-fno-slp-vectorize"]
        cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *kflags, *flags, f"-I{ROOT / 'include'}",
               f"-I{PKG / 'csrc'}", "--cuda-device-only", "-S", str(PKG / "csrc" / src), "-o", str(out)]
        subprocess.run(cmd, check=True, capture_output=True, timeout=600)
        _ASM[src] = out
    return _ASM[src]


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")
@pytest.mark.parametrize("src,flags", UNITS, ids=[u[0] for u in UNITS])
def test_no_isa_hazards(tmp_path_factory, src, flags):
    s = str(_compile(tmp_path_factory, src, flags))
    found = asm_hazard_check.scan(s)
    assert not found, "\n".join(found)
    loads, checked = asm_hazard_check.scan_loads(s)
    assert not loads, "\n".join(loads)
    if src == "nrc_train16.hip":
        # train16_split_kernel's sample loads (nrc_train16.hip), 8 per instance -- Frequency compact and padded, the
        # gathering Hash instance -- and 16 per Hash feature-workspace instance with 128-sample blocks (compact, padded:
        # + 8 level-feature loads), 8 per 64-sample Hash instance (round 5: compact, padded), 8 per fused-step instance
        # (round 6: train16_fused_kernel, compact and padded): the rule saw them
        assert checked == 88, checked
    loops = asm_hazard_check.scan_branch_store_loops(s)
    assert not loops, "\n".join(loops)


def _write(tmp_path, text: str) -> str:
    p = tmp_path / "k.s"
    p.write_text(text)
    return str(p)


# the faulting ablation build's pattern: an inline-asm load's address pair reused as the next address before the wait
FAULTING = """_Z6kernelv:
\tv_mov_b32 v40, v1
\t;;#ASMSTART
\tglobal_load_dwordx3 v[40:42], v[40:41], off
\t;;#ASMEND
\tv_lshl_add_u64 v[40:41], v[38:39], 0, s[8:9]
\tglobal_load_dword v7, v[40:41], off
\ts_waitcnt vmcnt(0)
\tv_add_f32 v1, v40, v41
\ts_endpgm
.Lfunc_end0:
"""

# train16_split_kernel's pattern: the loads land before anything touches them (vmcnt(2) with 2 younger loads)
CLEAN = """_Z6kernelv:
\t;;#ASMSTART
\tglobal_load_dwordx3 v[2:4], v[6:7], off
\t;;#ASMEND
\tv_lshl_add_u64 v[6:7], v[6:7], 0, 12
\tglobal_load_lds_dwordx4 v[20:21], off
\tglobal_load_lds_dwordx4 v[22:23], off
\ts_waitcnt vmcnt(2)
\tv_mul_f32 v3, v3, v13
\ts_endpgm
.Lfunc_end0:
"""

# the round-1 Hash shape: a loop whose prefetch sits behind s_cbranch_vccnz and whose result store behind execz
ROUND1 = """_Z6kernelv:
\ts_mov_b64 s[2:3], 0
.LBB0_10:
\ts_or_b64 exec, exec, s[4:5]
\ts_cbranch_vccz .LBB0_19
.LBB0_11:
\tbuffer_load_dword v1, v2, s[52:55], 0 offen
\tv_mfma_f32_32x32x16_f16 v[0:15], v[16:19], v[20:23], v[0:15]
\ts_and_b64 vcc, exec, s[2:3]
\ts_cbranch_vccnz .LBB0_16
\tglobal_load_dwordx3 v[68:70], v[72:73], off
.LBB0_16:
\ts_and_saveexec_b64 s[4:5], s[0:1]
\ts_cbranch_execz .LBB0_10
\tglobal_store_dwordx3 v[92:93], v[0:2], off
\ts_branch .LBB0_10
.LBB0_19:
\ts_endpgm
.Lfunc_end0:
"""


def test_load_rule_catches_the_faulting_pattern(tmp_path):
    found, checked = asm_hazard_check.scan_loads(_write(tmp_path, FAULTING))
    assert checked == 1 and len(found) == 2 and "v_lshl_add_u64 v[40:41]" in found[0], found
    found, checked = asm_hazard_check.scan_loads(_write(tmp_path, CLEAN))
    assert checked == 1 and not found, found
    # one wait too early (vmcnt(3) with 2 younger loads does not cover it): the use after it is reported
    found, _ = asm_hazard_check.scan_loads(_write(tmp_path, CLEAN.replace("vmcnt(2)", "vmcnt(3)")))
    assert found and "v_mul_f32 v3" in found[0], found


def test_loop_rule_catches_the_round1_shape(tmp_path):
    found = asm_hazard_check.scan_branch_store_loops(_write(tmp_path, ROUND1))
    assert len(found) == 1, found
    # the branch-free variants (the fixes of DESIGN.md §10's bisect) pass
    no_branch_load = ROUND1.replace("\ts_cbranch_vccnz .LBB0_16\n", "")
    assert not asm_hazard_check.scan_branch_store_loops(_write(tmp_path, no_branch_load))
    no_masked_store = ROUND1.replace("\ts_cbranch_execz .LBB0_10\n", "")
    assert not asm_hazard_check.scan_branch_store_loops(_write(tmp_path, no_masked_store))


# a self-loop of loads only (the grid Adam's slice sum) placed after an exec-masked store region and a scalar-branch
# load: the self-loop is one block, not everything before it (round 5: the checker had walked the self-loop's
# predecessors into the kernel entry and reported a 272-block "loop")
SELF_LOOP = """_Z6kernelv:
\ts_and_b64 vcc, exec, s[2:3]
\ts_cbranch_vccnz .LBB0_2
.LBB0_1:
\tglobal_load_dwordx2 v[6:7], v[4:5], off
.LBB0_2:
\ts_and_saveexec_b64 s[4:5], s[0:1]
\ts_cbranch_execz .LBB0_3
\tglobal_store_dword v1, v1, s[2:3]
.LBB0_3:
\tglobal_load_dwordx2 v[6:7], v[4:5], off sc1
\ts_add_u32 s6, s6, -1
\ts_cmp_lg_u32 s6, 0
\ts_cbranch_scc1 .LBB0_3
\ts_endpgm
.Lfunc_end0:
"""


def test_loop_rule_self_loop_is_one_block(tmp_path):
    path = _write(tmp_path, SELF_LOOP)
    blocks = asm_hazard_check._blocks(next(iter(asm_hazard_check.kernels(path).values())))
    assert [len(l) for l in asm_hazard_check._natural_loops(blocks)] == [1]
    assert not asm_hazard_check.scan_branch_store_loops(path)
