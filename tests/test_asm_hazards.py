"""Inline-asm VALU -> MFMA hazards in the product kernels (tools/asm_hazard_check.py).

LLVM's hazard recognizer does not see inside inline asm; an asm-produced register that an MFMA reads within 2 wait
states gets no s_nop and the MFMA reads a stale value. This compiles every gfx950 translation unit of libnrc_amd.so
to assembly (hipcc cross-compiles without a GPU) and requires that no such pair exists."""
from __future__ import annotations

import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "neural-radiance-caching_amd"
sys.path.insert(0, str(ROOT / "tools"))
import asm_hazard_check  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"
# (source, extra flags) as the Makefile builds them
UNITS = [("nrc_kernels.hip", []), ("nrc_train16.hip", ["-mllvm", "-amdgpu-mfma-vgpr-form"]),
         ("nrc_train_dc.hip", ["-mllvm", "-amdgpu-mfma-vgpr-form"]),
         ("nrc_infer16.hip", ["-mllvm", "-amdgpu-mfma-vgpr-form"])]


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")
@pytest.mark.parametrize("src,flags", UNITS, ids=[u[0] for u in UNITS])
def test_no_inline_asm_mfma_hazards(tmp_path, src, flags):
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", *flags,
           f"-I{ROOT / 'include'}", f"-I{PKG / 'csrc'}", "--cuda-device-only", "-S", str(PKG / "csrc" / src),
           "-o", str(tmp_path / "k.s")]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    found = asm_hazard_check.scan(str(tmp_path / "k.s"))
    assert not found, "\n".join(found)
