"""CPU suite, config 4: the churn model's delta stream (ksched_amd/churn.py)
encodes exactly the state transitions of the cell — replaying the deltas with
the graph-store semantics of ks_apply_deltas gives the same graph, with the
same optimal cost, as the cell's own full view. Mappings come from the oracle."""
import numpy as np

from graphs import apply_deltas_to_arcs, flow_mapping, graph_from_store
from ksched_amd import churn, gen
from oracle import ko


def store_of(g):
    nodes = {i + 1: [int(g.supply[i]), int(g.ntype[i])] for i in range(g.n)}
    arcs = {(int(s), int(d)): (int(lo), int(c), int(co))
            for s, d, lo, c, co in zip(g.src, g.dst, g.low, g.cap, g.cost)}
    return nodes, arcs


def arcs_of(g):
    return {(int(s), int(d)): (int(lo), int(c), int(co))
            for s, d, lo, c, co in zip(g.src, g.dst, g.low, g.cap, g.cost) if c > 0}


def test_round0_is_the_generator_graph():
    c = churn.Cell(500, 40, 4, 6, 9)
    a, b = c.graph(), gen.quincy(500, 40, 4, 6, 9)
    for k in ("ntype", "supply", "src", "dst", "low", "cap", "cost"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k


def test_delta_stream_replays_to_the_cell_graph():
    cell = churn.Cell(300, 30, 3, 5, 7)
    nodes, arcs = store_of(cell.graph())
    seen_pins = seen_done = 0
    for rnd in range(4):
        g = cell.graph()
        st, cost, flow, fl = ko.cost_scaling(g)
        assert st == 0 and flow == int((g.ntype == 1).sum())
        mp = flow_mapping(g, fl)
        running_before = set(cell.task_ids(cell.RUN).tolist())
        d = cell.step(mp, done=40, arrive=50)
        kinds = np.bincount(d["kind"], minlength=4)
        seen_done += int(kinds[churn.KS_REMOVE_NODE])
        seen_pins += int(((d["kind"] == churn.KS_ADD_ARC) & (d["type"] == churn.RUNNING)).sum())
        assert kinds[churn.KS_ADD_NODE] == 50
        # every removed node was a running task
        assert set(d["id"][d["kind"] == churn.KS_REMOVE_NODE].tolist()) <= running_before | set(
            cell.task_ids(cell.RUN).tolist()) | set(mp)
        apply_deltas_to_arcs(nodes, arcs, d)
        h = graph_from_store(nodes, arcs)
        ref = cell.graph()
        assert arcs_of(h) == arcs_of(ref)
        live = {i for i, (e, t) in nodes.items()}
        assert live == {i + 1 for i in range(ref.n) if ref.ntype[i] != 0 or i + 1 < cell.TASK0}
        s1 = ko.cost_scaling(h)
        s2 = ko.cost_scaling(ref)
        assert (s1[0], s1[1], s1[2]) == (s2[0], s2[1], s2[2]) == (0, s2[1], s2[2])
    assert seen_pins > 0 and seen_done > 0


def test_fifo_id_reuse():
    cell = churn.Cell(100, 10, 2, 3, 1)
    g = cell.graph()
    st, _, _, fl = ko.cost_scaling(g)
    d = cell.step(flow_mapping(g, fl), done=10, arrive=15)
    removed = d["id"][d["kind"] == churn.KS_REMOVE_NODE].tolist()
    added = d["id"][d["kind"] == churn.KS_ADD_NODE].tolist()
    assert added[:10] == removed                         # freed ids first, in order (graph.go:169-182)
    assert added[10:] == list(range(cell.TASK0 + 100, cell.TASK0 + 105))


def test_pinned_task_has_only_its_running_arc():
    cell = churn.Cell(200, 20, 2, 4, 3)
    g = cell.graph()
    _, _, _, fl = ko.cost_scaling(g)
    mp = flow_mapping(g, fl)
    cell.step(mp, done=0, arrive=0, age_cost=0)
    h = cell.graph()
    for t, p in list(mp.items())[:20]:
        out = [(int(d), int(lo), int(c)) for s, d, lo, c in zip(h.src, h.dst, h.low, h.cap) if s == t]
        assert out == [(p, 1, 1)]                        # graph_manager.go:690-735


def test_step_takes_the_mapping_as_arrays():
    """cell.step accepts ks_get_task_mapping's (task ids, PU ids) arrays (what the
    config-4 bench times) and produces the same records as the dict form."""
    import numpy as np
    from ksched_amd import churn
    a = churn.Cell(2_000, 200, 10, 20, 5)
    b = churn.Cell(2_000, 200, 10, 20, 5)
    tasks = a.task_ids(a.WAIT)[:500]
    pus = a.PU0 + (np.arange(tasks.shape[0]) % 200)
    da = a.step(dict(zip(tasks.tolist(), pus.tolist())), done=50, arrive=50)
    db = b.step((tasks.astype(np.uint64), pus.astype(np.uint64)), done=50, arrive=50)
    assert da.shape == db.shape and (da == db).all()
