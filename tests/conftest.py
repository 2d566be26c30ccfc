"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import __graft_entry__ as ge  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def pkg():
    return ge.load_package()


@pytest.fixture(scope="session")
def orc():
    return ge.load_oracle()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_arrays():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "golden_arrays.npz")))


@pytest.fixture
def client(pkg):
    c = pkg.SketchClient(decode_responses=True, device=0)
    yield c
    c.flushall()


@pytest.fixture
def engine(pkg):
    from rtsas_amd.engine import SketchEngine
    return SketchEngine(0)
