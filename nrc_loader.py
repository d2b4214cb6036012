"""Loads the package directory ``neural-radiance-caching_amd/`` (not an identifier) as ``nrc_amd``,
and the test-only oracle helpers from ``oracle/``."""
from __future__ import annotations

import importlib.util
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG_DIR = ROOT / "neural-radiance-caching_amd"
ORACLE_DIR = ROOT / "oracle"


def load():
    if "nrc_amd" in sys.modules:
        return sys.modules["nrc_amd"]
    spec = importlib.util.spec_from_file_location("nrc_amd", PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["nrc_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    """Test infrastructure only (tests/, smoke(), bench.py cpu_baseline)."""
    if str(ORACLE_DIR) not in sys.path:
        sys.path.insert(0, str(ORACLE_DIR))
    import orc  # noqa: E402
    return orc
