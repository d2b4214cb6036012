import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

import nrc_loader  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(scope="session")
def nrc():
    return nrc_loader.load()


@pytest.fixture(scope="session")
def orc():
    o = nrc_loader.load_oracle()
    o.lib()
    return o


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    path = ROOT / "tests" / "golden" / "nrc_golden.npz"
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def dev():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    return torch.device("cuda:0")
