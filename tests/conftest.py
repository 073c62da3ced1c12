import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libemrifd.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden_cases():
    import glob
    import numpy as np
    out = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "golden_*.npz"))):
        name = os.path.basename(f)[len("golden_"):-4]
        out[name] = dict(np.load(f))
    return out
