"""Every `file:line` citation of a reference source in this repo resolves.

Scans the repo's own sources and docs for citations of files that exist under /root/reference
(`NRCNetwork.cu:41-56`, `Device.cpp:1504`, and bare continuations such as `(:43, :66)` after a cited file
on the same line) and checks that every cited line range lies inside the cited file. A few load-bearing
boundary citations are also checked against the text they must point at. Skipped where /root/reference is
absent (the GPU box): it is a repository-hygiene check, not part of the product.
"""
from __future__ import annotations

import os
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")

pytestmark = pytest.mark.skipif(not REF.is_dir(), reason="reference tree not present")

SCAN_SUFFIXES = {".py", ".h", ".hpp", ".hip", ".cpp", ".c", ".md", ".sh"}
SKIP_DIRS = {".git", "gpurun_out", "__pycache__", ".pytest_cache", "build"}
# the judge's and the surveyor's files are not the builder's citations
SKIP_FILES = {"SURVEY.md", "VERDICT.md", "ADVICE.md", "PROGRESS.jsonl", "test_citations.py"}

CITE = re.compile(r"(?P<file>[\w./-]+\.(?:cu|h|cpp|txt|gitmodules))(?::(?P<a>\d+)(?:-(?P<b>\d+))?)")
BARE = re.compile(r"(?<=[\s(`,]):(?P<a>\d+)(?:-(?P<b>\d+))?\b")


def _ref_index() -> dict[str, list[Path]]:
    idx: dict[str, list[Path]] = {}
    for dirpath, dirnames, filenames in os.walk(REF):
        dirnames[:] = [d for d in dirnames if not d.startswith(".") and d != "imgui"]
        for f in filenames:
            idx.setdefault(f, []).append(Path(dirpath) / f)
    return idx


def _nlines(p: Path) -> int:
    with open(p, "rb") as fh:
        return fh.read().count(b"\n") + 1


def _candidates(idx, cited: str) -> list[Path]:
    base = os.path.basename(cited)
    cands = idx.get(base, [])
    if "/" in cited:
        narrowed = [c for c in cands if str(c).endswith(cited.lstrip("./"))]
        if narrowed:
            return narrowed
    return cands


def _scan():
    idx = _ref_index()
    for dirpath, dirnames, filenames in os.walk(ROOT):
        dirnames[:] = [d for d in dirnames if d not in SKIP_DIRS]
        for f in filenames:
            p = Path(dirpath) / f
            if p.suffix not in SCAN_SUFFIXES or f in SKIP_FILES:
                continue
            for ln_no, line in enumerate(p.read_text(errors="replace").splitlines(), 1):
                last = None
                pos = 0
                while True:
                    m = CITE.search(line, pos)
                    if m is None:
                        break
                    cands = _candidates(idx, m.group("file"))
                    if cands:
                        last = cands
                        if m.group("a"):
                            yield p, ln_no, m.group("file"), int(m.group("a")), int(m.group("b") or m.group("a")), cands
                        # bare continuations up to the next file citation
                        nxt = CITE.search(line, m.end())
                        seg = line[m.end(): nxt.start() if nxt else len(line)]
                        for bm in BARE.finditer(seg):
                            yield p, ln_no, m.group("file"), int(bm.group("a")), int(bm.group("b") or bm.group("a")), last
                    pos = m.end()


def test_every_reference_citation_resolves():
    bad = []
    n = 0
    for p, ln_no, cited, a, b, cands in _scan():
        n += 1
        if a < 1 or b < a or not any(b <= _nlines(c) for c in cands):
            bad.append(f"{p.relative_to(ROOT)}:{ln_no}: {cited}:{a}-{b} (file has {max(_nlines(c) for c in cands)} lines)")
    assert n > 50, f"citation scan found only {n} citations"
    assert not bad, "citations past the end of the cited file:\n" + "\n".join(bad)


# boundary citations that must point at specific code (include/nrc/nrc_c.h)
ANCHORS = [
    ("nrc/src/NRCNetwork.cu", 35, 39, "void Network::destroy()"),
    ("nrc/src/NRCNetwork.cu", 41, 56, "void Network::train("),
    ("nrc/src/NRCNetwork.cu", 43, 43, "if (m_destroyed)"),
    ("nrc/src/NRCNetwork.cu", 51, 52, "BATCH_SIZE"),
    ("nrc/src/NRCNetwork.cu", 53, 53, "training_step"),
    ("nrc/src/NRCNetwork.cu", 54, 55, "trainer->loss"),
    ("nrc/src/NRCNetwork.cu", 64, 77, "void Network::infer("),
    ("nrc/src/NRCNetwork.cu", 72, 72, "BATCH_SIZE_GRANULARITY"),
    ("nrc/src/NRCNetwork.cu", 76, 76, "network->inference"),
    ("nrc/src/NRCNetwork.cu", 85, 88, "void Network::setStream"),
    ("nrc/src/NRCNetwork.cu", 90, 94, "void Network::setHyperParams"),
    ("nrc/src/NRCNetwork.cu", 96, 99, "void Network::setConfig"),
    ("nrc/src/NRCNetwork.cu", 101, 104, "float Network::getLearningRate"),
    ("nrc/src/NRCNetwork.cu", 106, 112, "void Network::init_"),
    ("nrc/src/NRCNetwork.cu", 122, 127, "void Network::printConfig_"),
    ("nrc/inc/NRCNetworkConfigs.h", 129, 131, "Unsupported input encoding"),
    ("nrc/inc/NRCNetworkConfigs.h", 26, 33, "FullyFusedMLP"),
    ("nrc/inc/NRCNetwork.h", 20, 75, "class Network"),
]


@pytest.mark.parametrize("path,a,b,needle", ANCHORS)
def test_boundary_anchor_text(path, a, b, needle):
    lines = (REF / path).read_text(errors="replace").splitlines()
    assert needle in "\n".join(lines[a - 1: b]), f"{path}:{a}-{b} does not contain {needle!r}"
