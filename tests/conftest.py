import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def load_goldens():
    with open(os.path.join(GOLDEN, "goldens.json")) as f:
        return json.load(f)["graphs"]


def load_known_answers():
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ctx():
    """One HIP solver context shared by the GPU tests (one process on the box)."""
    from ksched_amd import native
    c = native.Context(0)
    yield c
    c.close()
