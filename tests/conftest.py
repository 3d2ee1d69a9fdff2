import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs via gpurun")
    config.addinivalue_line("markers", "slow: large inputs (1e7+ points)")


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    d = os.path.join(ROOT, "tests", "golden")

    def load(name):
        return np.load(os.path.join(d, name + ".npz"), allow_pickle=False)

    return load


@pytest.fixture(scope="session")
def gpu():
    """The HIP path must be the one that runs: fail (not skip) when the
    library is missing or no device is visible on a GPU run."""
    from nbodyhpc_amd import capi
    n = capi.device_count()
    if n == 0:
        pytest.fail("no HIP device visible but the test is marked gpu")
    return capi
