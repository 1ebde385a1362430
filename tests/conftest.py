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


CELL_ANY = 1 << 16   # ks_opts.cell_nodes above the LDS limit: the cell solver for whatever fits


@pytest.fixture(scope="session")
def ctx():
    """One HIP solver context shared by the GPU tests (one process on the box).
    cell_nodes = CELL_ANY: every graph the cell solver's LDS holds (config-2 size)
    runs in one workgroup (ks_cell.hip), larger ones on the multi-kernel engine (by
    default a lone graph takes the cell solver only up to 4,096 nodes)."""
    from ksched_amd import native
    c = native.Context(0, cell_nodes=CELL_ANY)
    yield c
    c.close()


@pytest.fixture(scope="session")
def ctx_engine():
    """A context pinned to the multi-kernel engine (ks_opts.cell_nodes = -1), so
    small graphs exercise it too."""
    from ksched_amd import native
    c = native.Context(0, cell_nodes=-1)
    yield c
    c.close()


@pytest.fixture(params=["cell", "engine"])
def any_ctx(request, ctx, ctx_engine):
    """Each solver path in turn: the default context (cell solver for small
    graphs) and the engine-pinned one."""
    return ctx if request.param == "cell" else ctx_engine
