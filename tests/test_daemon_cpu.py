"""CPU suite: the flow_scheduler-compatible daemon (ksched_amd/csrc/ks_flow_scheduler.cpp)
parses ksched's DIMACS stream — the full export (dimacs/export.go:11-76) and the
incremental change records (dimacs/*_change.go) — framed by "c EOI"."""
import subprocess

import pytest

from graphs import dimacs_changes, flow_mapping
from ksched_amd import _build, churn
from oracle import ko


@pytest.fixture(scope="module")
def daemon():
    _build.build(verbose=False)
    return _build.build_daemon()


def run(daemon, text, *args):
    return subprocess.run([daemon, "--parse-only", *args], input=text, capture_output=True, text=True, timeout=120)


def test_parses_full_export_and_change_rounds(daemon):
    cell = churn.Cell(300, 30, 3, 5, 7)
    g = cell.graph()
    text = ko.export_dimacs(g)
    _, _, _, fl = ko.cost_scaling(g)
    d1 = cell.step(flow_mapping(g, fl), done=0, arrive=20)
    g1 = cell.graph()
    _, _, _, fl1 = ko.cost_scaling(g1)
    d2 = cell.step(flow_mapping(g1, fl1), done=10, arrive=10)
    text += dimacs_changes(d1) + dimacs_changes(d2)
    p = run(daemon, text)
    assert p.returncode == 0, p.stderr
    lines = p.stdout.splitlines()
    assert lines == [f"iteration full nodes {g.n} arcs {g.m} deltas 0",
                     f"iteration incremental nodes 0 arcs 0 deltas {d1.shape[0]}",
                     f"iteration incremental nodes 0 arcs 0 deltas {d2.shape[0]}"]


def test_daemon_false_stops_after_first_graph(daemon):
    g = churn.Cell(100, 10, 2, 3, 1).graph()
    p = run(daemon, ko.export_dimacs(g) + "r 200\nc EOI\n", "--daemon=false")
    assert p.returncode == 0 and len(p.stdout.splitlines()) == 1


@pytest.mark.parametrize("bad", ["q 1 2\nc EOI\n", "n 1 2\nc EOI\n", "a 1 2 0 1\nc EOI\n", "n 1 0 3\n"])
def test_malformed_input_fails_loudly(daemon, bad):
    p = run(daemon, bad)
    assert p.returncode != 0 and "ks_flow_scheduler" in p.stderr


def test_coalesce_flag_matches_the_c_abi(daemon):
    """--coalesce: each change block goes through ks_coalesce_deltas before it is
    applied (optimizeChanges, graph_change_manager.go:220-229)."""
    import numpy as np
    from ksched_amd import native
    cell = churn.Cell(300, 30, 3, 5, 7)
    g = cell.graph()
    _, _, _, fl = ko.cost_scaling(g)
    d1 = cell.step(flow_mapping(g, fl), done=0, arrive=20)
    g1 = cell.graph()
    _, _, _, fl1 = ko.cost_scaling(g1)
    d2 = cell.step(flow_mapping(g1, fl1), done=30, arrive=10)
    d = np.concatenate([d1, d2])
    p = run(daemon, ko.export_dimacs(g) + dimacs_changes(d), "--coalesce")
    assert p.returncode == 0, p.stderr
    kept = native.coalesce_deltas(d).shape[0]
    assert kept < d.shape[0]
    assert p.stdout.splitlines()[1] == f"iteration incremental nodes 0 arcs 0 deltas {kept}"
