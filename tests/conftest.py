import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X); run with -m gpu")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def unpack_labels(g, key):
    shp = tuple(int(x) for x in g[key + "_shape"])
    return np.unpackbits(g[key])[: int(np.prod(shp))].reshape(shp).astype(np.int64)


@pytest.fixture(scope="session")
def synthetic_sd():
    import clasfv_amd.weights as W
    return W.synthetic_state_dict(W.DEFAULT_SEED)
