import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the gfx950 kernels through the C-ABI)")
    # every oracle run of the suite carries the exact sums its doc-order additions approximate ("_exact"):
    # helpers.assert_same compares a floating value with the oracle's or, where the oracle's rounding is the larger
    # error, with the exact one (SURVEY §7 "Float parity")
    import oracle
    oracle.EXACT_DEFAULT = True


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(REPO, "tests", "golden", "kat.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def engine():
    """One device context for the whole GPU session (the box allows few GPU processes; keep it to one)."""
    import elasticsearch_amd as ea
    if ea.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests need an MI355X")
    e = ea.Engine(0)
    yield e
    e.close()
