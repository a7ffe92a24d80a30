import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running")


def load_json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def read_golden(name) -> bytes:
    with open(os.path.join(GOLD, name), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def table():
    return np.fromfile(os.path.join(GOLD, "buzhash32_table.bin"), dtype="<u4")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O  # test infrastructure only
    O.build()
    return O


@pytest.fixture(scope="session")
def gpu():
    """The HIP library, built in-tree; skips only if no GPU is visible."""
    from bs_amd import build, bsgpu
    build.build()
    if bsgpu.device_count() < 1:
        pytest.skip("no HIP device visible")
    return bsgpu
