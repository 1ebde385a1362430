"""CPU suite: the oracle pinned against the committed goldens and the known
answers derived from the reference, the generator twins, and
the DIMACS / "f"-line protocol of placement/solver.go. No GPU needed."""
import numpy as np
import pytest

from conftest import load_goldens, load_known_answers
from graphs import graph_from_lists, random_graphs, random_hub_graphs
from ksched_amd import gen
from oracle import ko


def _graph(e):
    return gen.trivial(*e["params"]) if e["family"] == "trivial" else gen.quincy(*e["params"], e["seed"])


SMALL = [e for e in load_goldens() if e["m"] <= 60000]


@pytest.mark.parametrize("e", SMALL, ids=lambda e: f"{e['family']}-{'x'.join(map(str, e['params']))}-s{e['seed']}")
def test_oracle_ssp_matches_golden(e):
    """Successive shortest path (Flowlessly's configured algorithm, solver.go:32)."""
    g = _graph(e)
    assert (g.n, g.m) == (e["n"], e["m"])
    st, cost, flow, fl, _ = ko.ssp(g)
    assert st == 0
    assert (cost, flow) == (e["cost"], e["flow"])
    vst, vcost, _ = ko.verify(g, fl)
    assert vst == 0 and vcost == cost


@pytest.mark.parametrize("e", SMALL, ids=lambda e: f"{e['family']}-{'x'.join(map(str, e['params']))}-s{e['seed']}")
def test_oracle_cost_scaling_matches_golden(e):
    g = _graph(e)
    st, cost, flow, fl = ko.cost_scaling(g)
    assert st == 0
    assert (cost, flow) == (e["cost"], e["flow"])
    assert ko.verify(g, fl)[0] == 0


def test_known_answer_config1():
    """k8sscheduler -fakeMachines -nm 10, mt 1000, 100 pods in one job: cost 200 flow 100."""
    ka = load_known_answers()["config1"]
    g = gen.trivial(*ka["params"])
    assert (g.n, g.m) == (ka["n"], ka["m"])
    st, cost, flow, fl, _ = ko.ssp(g)
    assert (st, cost, flow) == (0, ka["cost"], ka["flow"])
    mp = ko.bfs_mapping(g, fl, cost)
    assert len(mp) == 100
    assert all(g.ntype[p - 1] == 2 for p in mp.values())


def test_known_answer_multi_schedule_round1():
    r1 = load_known_answers()["multi_schedule_iteration"]["round1_graph"]
    g = graph_from_lists(r1["nodes"], r1["arcs"])
    st, cost, flow, fl, _ = ko.ssp(g)
    assert (st, cost, flow) == (0, r1["cost"], r1["flow"])
    ka = load_known_answers()["multi_schedule_iteration"]
    assert (cost, flow) == (ka["round_costs"][0], ka["round_flows"][0])
    assert len(ko.bfs_mapping(g, fl, cost)) == 2


@pytest.mark.parametrize("params", [(100, 10, 2, 3, 7), (1000, 100, 5, 10, 1), (3000, 300, 12, 30, 10)])
def test_generator_twins_bit_identical(params):
    """numpy generator (product side) == C generator (oracle side), every array."""
    a = gen.quincy(*params)
    b = ko.gen_quincy(*params)
    for k in ("ntype", "supply", "src", "dst", "low", "cap", "cost"):
        assert np.array_equal(np.asarray(getattr(a, k)), np.asarray(getattr(b, k))), k


def test_quincy_sizes_formula():
    for T, M, R, J, _ in gen.CONFIGS.values():
        n, m = gen.quincy_sizes(T, M, R, J)
        assert (n, m) == (T + J + R + 2 * M + 2, 5 * T + R + 3 * M + J)
    assert gen.quincy_sizes(*gen.CONFIGS["config3"][:4]) == (121252, 531250)
    assert gen.quincy_sizes(*gen.CONFIGS["config2"][:4]) == (12127, 53125)


def test_dimacs_export_format():
    """dimacs/export.go:11-76: header, one 'n id excess type' per node, 5-field 'a' lines, 'c EOI'."""
    g = gen.trivial(2, 1, 3)
    txt = ko.export_dimacs(g)
    lines = txt.splitlines()
    assert lines[0] == "c ==========================="
    assert lines[1] == f"p min {g.n} {g.m}"
    assert lines[3] == "c === ALL NODES FOLLOW ==="
    nl = [l for l in lines if l.startswith("n ")]
    al = [l for l in lines if l.startswith("a ")]
    assert len(nl) == g.n and len(al) == g.m
    assert nl[0] == f"n 1 {-3} 3"                 # sink: excess −#tasks, type 3
    assert all(len(l.split()) == 6 for l in al)  # "a src dst low cap cost"
    assert lines[-1] == "c EOI"


def test_bfs_mapping_rejects_non_unit_task():
    """solver.go:223-225 panics when a task would receive != 1 PU."""
    nodes = [(1, -2, 3), (2, 0, 2), (3, 2, 1)]
    arcs = [(2, 1, 0, 2, 0), (3, 2, 0, 2, 1)]
    g = graph_from_lists(nodes, arcs)
    st, cost, _, fl, _ = ko.ssp(g)
    assert st == 0
    with pytest.raises(RuntimeError):
        ko.bfs_mapping(g, fl, cost)


def test_verify_detects_violations():
    g = gen.trivial(2, 1, 3)
    st, cost, _, fl, _ = ko.ssp(g)
    bad = fl.copy()
    i = int(np.argmax(g.cap))
    bad[i] = g.cap[i] + 1
    assert ko.verify(g, bad)[0] != 0
    bad = fl.copy()
    j = int(np.nonzero(fl)[0][0])
    bad[j] -= 1
    assert ko.verify(g, bad)[0] != 0


def test_random_graphs_ssp_equals_cost_scaling():
    """Two independent exact algorithms agree on general digraphs (cycles,
    antiparallel arcs, zero capacities, lower bounds, infeasible cases)."""
    feasible = 0
    for _, g in random_graphs(777, 60):
        st1, c1, f1, fl1, _ = ko.ssp(g)
        st2, c2, f2, fl2 = ko.cost_scaling(g)
        assert (st1 == 0) == (st2 == 0)
        if st1 == 0:
            feasible += 1
            assert (c1, f1) == (c2, f2)
            assert ko.verify(g, fl1)[0] == 0 and ko.verify(g, fl2)[0] == 0
    assert feasible >= 10


def test_hub_graphs_ssp_equals_cost_scaling():
    """The GPU stress graphs (tests/test_gpu_stress.py): the two oracles agree on
    every seed that test uses, and the mix holds feasible and infeasible graphs."""
    feasible = infeasible = 0
    for seed in (2026, 2027):
        for _, g in random_hub_graphs(seed, 16):
            st1, c1, f1, fl1, _ = ko.ssp(g)
            st2, c2, f2, _ = ko.cost_scaling(g)
            assert (st1 == 0) == (st2 == 0)
            if st1 == 0:
                feasible += 1
                assert (c1, f1) == (c2, f2)
                assert ko.verify(g, fl1)[0] == 0
            else:
                infeasible += 1
    assert feasible >= 16 and infeasible >= 2


def test_reference_path_config2():
    """The whole reference CPU path (export → parse → SSP → f lines → BFS) on config 2."""
    T, M, R, J, seed = gen.CONFIGS["config2"]
    g = gen.quincy(T, M, R, J, seed)
    gold = [e for e in load_goldens() if e["params"] == [T, M, R, J] and e["seed"] == seed][0]
    st, cost, flow, mapped, ms = ko.reference_path(g)
    assert (st, cost, flow) == (0, gold["cost"], gold["flow"])
    assert 0 < mapped <= T
