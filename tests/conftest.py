import os
import sys
from pathlib import Path

import pytest

# The oracle's torch convs on the GPU (EnvNet-v2 at B = 256 in tests/test_gpu_fullsize.py): MIOpen's
# default find mode benchmarks and compiles solvers for every new shape, minutes of silence on a fresh
# box; FAST takes its immediate-mode choice.  Set before torch loads MIOpen.
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "dl-sound-classification_amd"
for p in (str(REPO), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return dict(np.load(REPO / "tests" / "golden" / "golden.npz", allow_pickle=False))


@pytest.fixture(scope="session")
def golden_aug():
    import numpy as np
    return dict(np.load(REPO / "tests" / "golden" / "golden_aug.npz", allow_pickle=False))


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
