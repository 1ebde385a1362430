"""GPU: the flow_scheduler-compatible daemon end to end — ksched's DIMACS
stream in (full export, then change records), "f"/"s"/"c EOI" blocks out —
checked against the oracle per iteration and read back with the reference's
own flow-line parser (placement/solver.go:134-269, restated in the oracle)."""
import subprocess

import numpy as np
import pytest

from graphs import dimacs_changes
from ksched_amd import _build, churn
from oracle import ko

pytestmark = pytest.mark.gpu


def blocks(out: str):
    cur = []
    for line in out.splitlines():
        cur.append(line)
        if line == "c EOI":
            yield cur
            cur = []
    assert not cur


def test_daemon_full_then_incremental():
    daemon = _build.build_daemon()
    cell = churn.Cell(3_000, 300, 12, 30, 21)
    graphs = [cell.graph()]
    text = ko.export_dimacs(graphs[0])
    mp = None
    for rnd in range(2):
        g = graphs[-1]
        _, _, _, fl = ko.cost_scaling(g)
        from graphs import flow_mapping
        d = cell.step(flow_mapping(g, fl), done=150, arrive=150)
        text += dimacs_changes(d)
        graphs.append(cell.graph())
    p = subprocess.run([daemon, "--graph_has_node_types=true", "--algorithm=successive_shortest_path",
                        "--print_assignments=false", "--debug_output=true"],
                       input=text, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    outs = list(blocks(p.stdout))
    assert len(outs) == 3
    for g, blk in zip(graphs, outs):
        st, cost, flow, _ = ko.cost_scaling(g)
        assert st == 0
        f = [tuple(map(int, l.split()[1:])) for l in blk if l.startswith("f ")]
        assert all(x[2] > 0 for x in f)
        key = {(int(s), int(d)): int(c) for s, d, c in zip(g.src, g.dst, g.cost)}
        assert sum(key[(s, d)] * x for s, d, x in f) == cost
        assert [l for l in blk if l.startswith("s ")] == [f"s {cost}"]
    mp = ko.bfs_mapping_from_text(graphs[0], "\n".join(outs[0]) + "\n")
    assert len(mp) > 0 and all(graphs[0].ntype[p - 1] == 2 for p in mp.values())
