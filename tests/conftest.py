import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


class Golden:
    def __init__(self):
        self.setup = dict(np.load(os.path.join(GOLDEN, "setup.npz")))
        self.integrate = dict(np.load(os.path.join(GOLDEN, "integrate.npz")))
        self.mh = dict(np.load(os.path.join(GOLDEN, "mh.npz")))
        self.mcmc = dict(np.load(os.path.join(GOLDEN, "mcmc.npz")))
        self.replicate = dict(np.load(os.path.join(GOLDEN, "replicate.npz")))
        with open(os.path.join(GOLDEN, "meta.json")) as f:
            self.meta = json.load(f)


@pytest.fixture(scope="session")
def golden():
    return Golden()
