import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a visible ROCm GPU")
    import tspm_amd  # noqa: F401
    tspm_amd._lib.load()
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    path = os.path.join(REPO, "tests", "golden", "avmnist_step_b4.npz")
    return dict(np.load(path, allow_pickle=False))


@pytest.fixture(scope="session")
def lut():
    import numpy as np
    import torch
    with open(os.path.join(REPO, "tests", "golden", "lut_gist_earth_L.bin"), "rb") as f:
        return torch.from_numpy(np.frombuffer(f.read(), dtype=np.uint8).copy())
