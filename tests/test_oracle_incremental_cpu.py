"""CPU suite: the incremental SSP restatement (oracle/ks_oracle.c
ko_ssp_incremental — Flowlessly's daemon mode, which ksched runs:
placement/solver.go:30-34 Incremental = true, later Solves send only the change
block, :86-89) re-solves each churn round from the previous round's flow and
potentials and must reach the same optimum as a cold solve of the round's full
graph; the change block round-trips through its ExportIncremental text
(dimacs/export.go:31-38, *_change.go GenerateChange)."""
import numpy as np
import pytest

from ksched_amd import churn
from oracle import ko


def test_change_block_text_round_trip():
    cell = churn.Cell(300, 30, 3, 5, 11)
    g = cell.graph()
    st, c, f, flow, _ = ko.ssp(g)
    d = cell.step(ko.bfs_mapping(g, flow), done=20, arrive=20)
    text = ko.IncrementalSSP().export_changes(d)
    assert text.endswith("c EOI\n")
    kinds = {0: "n", 1: "r", 2: "a", 3: "x"}
    lines = text.splitlines()[:-1]
    assert [l[0] for l in lines] == [kinds[int(k)] for k in d["kind"]]
    # field counts as GenerateChange writes them: n 3, r 1, a 6, x 7
    assert all(len(l.split()) - 1 == {"n": 3, "r": 1, "a": 6, "x": 7}[l[0]] for l in lines)
    back = ko.parse_changes(text)
    for name in ("kind", "id", "src", "dst", "low", "cap", "cost"):
        assert (back[name] == d[name]).all(), name
    assert (back["type"][d["kind"] >= 2] == d["type"][d["kind"] >= 2]).all()


@pytest.mark.parametrize("seed", [7, 8])
def test_incremental_ssp_matches_cold_solves_over_rounds(seed):
    cell = churn.Cell(1500, 150, 10, 15, seed)
    g = cell.graph()
    inc = ko.IncrementalSSP()
    st, cost, fv, flow = inc.round(g)
    assert st == 0 and (cost, fv) == ko.ssp(g)[1:3]
    for r in range(5):
        d = cell.step(ko.bfs_mapping(g, flow), done=80, arrive=80)
        g = cell.graph()
        st, cost, fv, flow = inc.round(g, d, cell.last_arrived_ids)
        assert st == 0
        cs = ko.cost_scaling(g)
        assert (cost, fv) == (cs[1], cs[2]) == ko.ssp(g)[1:3], r
        vs = ko.verify(g, flow)
        assert vs[0] == 0 and vs[1] == cost
        assert inc.last["mapped"] >= 0        # the BFS mapping accepts the re-solved flow


def test_incremental_ssp_without_changes_is_a_no_op():
    cell = churn.Cell(500, 50, 5, 5, 3)
    g = cell.graph()
    inc = ko.IncrementalSSP()
    _, cost, _, flow = inc.round(g)
    _, cost2, _, flow2 = inc.round(g)
    assert cost2 == cost and (flow2 == flow).all()
