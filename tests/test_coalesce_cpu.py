"""CPU suite: ks_coalesce_deltas (the change optimisers graph_change_manager.go:220-279,
declared but never implemented in the reference — RemoveDuplicate, MergeToSameArc,
PurgeBeforeNodeRemoval). A coalesced stream must replay, with the graph-store
semantics of ks_apply_deltas, to the same nodes and arcs (type included) as the raw
stream, on hand-written edge cases, random valid streams and multi-round config-4
churn. Host-only: the C-ABI function touches no device."""
import numpy as np
import pytest

from graphs import flow_mapping
from ksched_amd import churn, native
from oracle import ko

ADD_NODE, REMOVE_NODE, ADD_ARC, UPDATE_ARC, SET_EXCESS = 0, 1, 2, 3, 4


def rec(kind, id=0, src=0, dst=0, low=0, cap=0, cost=0, type=0, excess=0, old_cost=0):
    return (kind, type, id, src, dst, low, cap, cost, old_cost, excess)


def arr(rows):
    a = np.zeros(len(rows), native.DELTA_DT)
    for i, r in enumerate(rows):
        a[i] = r
    return a


def replay(nodes: dict, arcs: dict, deltas):
    """ks_apply_deltas semantics (ks_host.cpp, include/ksmcmf.h), arc type kept."""
    nodes, arcs = dict(nodes), dict(arcs)
    for x in deltas:
        k = int(x["kind"])
        if k == ADD_NODE:
            nodes[int(x["id"])] = (int(x["excess"]), int(x["type"]))
        elif k == REMOVE_NODE:
            i = int(x["id"])
            nodes.pop(i)
            for key in [a for a in arcs if i in a]:
                del arcs[key]
        elif k == SET_EXCESS:
            i = int(x["id"])
            nodes[i] = (int(x["excess"]), nodes[i][1])
        else:
            s, d = int(x["src"]), int(x["dst"])
            assert s in nodes and d in nodes
            if k == UPDATE_ARC and int(x["low"]) == 0 and int(x["cap"]) == 0:
                arcs.pop((s, d), None)
            else:
                arcs[(s, d)] = (int(x["low"]), int(x["cap"]), int(x["cost"]), int(x["type"]))
    return nodes, arcs


def check_equivalent(nodes, arcs, d):
    c = native.coalesce_deltas(d)
    assert replay(nodes, arcs, c) == replay(nodes, arcs, d)
    # survivors are a subsequence of the input, in order
    it = iter(d.tobytes()[i:i + d.itemsize] for i in range(0, d.nbytes, d.itemsize))
    for r in c:
        b = r.tobytes()
        assert any(b == x for x in it)
    return c


def test_empty_stream():
    assert native.coalesce_deltas(np.zeros(0, native.DELTA_DT)).shape == (0,)


def test_last_record_per_arc_wins():
    base_n = {1: (0, 3), 2: (1, 1), 3: (0, 2)}
    d = arr([rec(ADD_ARC, src=2, dst=3, cap=1, cost=5),
             rec(UPDATE_ARC, src=2, dst=3, cap=1, cost=7, old_cost=5),
             rec(UPDATE_ARC, src=2, dst=3, cap=1, cost=7, old_cost=5),      # duplicate
             rec(ADD_ARC, src=3, dst=1, cap=4),
             rec(UPDATE_ARC, src=2, dst=3, cap=1, cost=9, type=1, old_cost=7)])
    c = check_equivalent(base_n, {}, d)
    assert c.shape[0] == 2
    assert (int(c[1]["cost"]), int(c[1]["type"])) == (9, 1)


def test_delete_then_readd_and_readd_then_delete():
    base_n = {1: (0, 3), 2: (1, 1)}
    base_a = {(2, 1): (0, 1, 3, 0)}
    d = arr([rec(UPDATE_ARC, src=2, dst=1), rec(ADD_ARC, src=2, dst=1, cap=2, cost=4)])
    assert check_equivalent(base_n, base_a, d).shape[0] == 1
    d = arr([rec(ADD_ARC, src=2, dst=1, cap=2, cost=4), rec(UPDATE_ARC, src=2, dst=1)])
    c = check_equivalent(base_n, base_a, d)
    assert c.shape[0] == 1 and int(c[0]["kind"]) == UPDATE_ARC


def test_purge_before_node_removal_and_id_reuse():
    base_n = {1: (-1, 3), 2: (1, 1), 3: (0, 2), 4: (0, 2)}
    base_a = {(2, 3): (0, 1, 1, 0), (3, 1): (0, 1, 0, 0), (4, 1): (0, 1, 0, 0)}
    d = arr([rec(UPDATE_ARC, src=2, dst=3),                   # purged by "r 2"
             rec(ADD_ARC, src=2, dst=4, low=1, cap=1, type=1),  # purged by "r 2"
             rec(SET_EXCESS, id=2, excess=5),                  # purged by "r 2"
             rec(UPDATE_ARC, src=3, dst=1, cap=2),             # kept (3 survives)
             rec(REMOVE_NODE, id=2),
             rec(ADD_NODE, id=2, excess=1, type=1),            # FIFO id reuse
             rec(ADD_ARC, src=2, dst=3, cap=1, cost=8),        # new incarnation: kept
             rec(SET_EXCESS, id=1, excess=-3),
             rec(SET_EXCESS, id=1, excess=-1)])                # only the last survives
    c = check_equivalent(base_n, base_a, d)
    assert [int(x) for x in c["kind"]] == [UPDATE_ARC, REMOVE_NODE, ADD_NODE, ADD_ARC, SET_EXCESS]


def test_in_place_and_count_query():
    d = arr([rec(ADD_ARC, src=2, dst=3, cap=1), rec(ADD_ARC, src=2, dst=3, cap=2)])
    L = native.load()
    import ctypes as C
    cnt = C.c_size_t()
    assert L.ks_coalesce_deltas(d.ctypes.data, 2, None, 0, C.byref(cnt)) == 0 and cnt.value == 1
    assert L.ks_coalesce_deltas(d.ctypes.data, 2, d.ctypes.data, 2, C.byref(cnt)) == 0 and cnt.value == 1
    assert int(d[0]["cap"]) == 2


def test_invalid_ids_rejected():
    with pytest.raises(native.KsError):
        native.coalesce_deltas(arr([rec(REMOVE_NODE, id=0)]))
    with pytest.raises(native.KsError):
        native.coalesce_deltas(arr([rec(ADD_ARC, src=1 << 31, dst=2, cap=1)]))


def random_stream(rng, n0=12, k=400):
    nodes = {i: (0, int(rng.integers(0, 4))) for i in range(1, n0 + 1)}
    arcs = {}
    for _ in range(3 * n0):
        s, d = (int(v) for v in rng.integers(1, n0 + 1, 2))
        if s != d:
            arcs[(s, d)] = (0, int(rng.integers(1, 4)), int(rng.integers(0, 9)), 0)
    live, free, nxt = set(nodes), [], n0 + 1
    rows = []
    for _ in range(k):
        u = rng.random()
        if u < 0.06 and len(live) > 3:
            v = int(rng.choice(sorted(live)))
            live.discard(v)
            free.append(v)
            rows.append(rec(REMOVE_NODE, id=v))
        elif u < 0.12:
            if free:
                v = free.pop(0)
            else:
                v, nxt = nxt, nxt + 1
            live.add(v)
            rows.append(rec(ADD_NODE, id=v, excess=int(rng.integers(-2, 3)), type=int(rng.integers(0, 4))))
        elif u < 0.18:
            rows.append(rec(SET_EXCESS, id=int(rng.choice(sorted(live))), excess=int(rng.integers(-3, 4))))
        else:
            s, d = (int(v) for v in rng.choice(sorted(live), 2, replace=False))
            kind = ADD_ARC if rng.random() < 0.4 else UPDATE_ARC
            cap = 0 if rng.random() < 0.25 else int(rng.integers(1, 5))
            low = 1 if cap and rng.random() < 0.1 else 0
            rows.append(rec(kind, src=s, dst=d, low=low, cap=cap, cost=int(rng.integers(0, 20)),
                            type=int(rng.integers(0, 2))))
    return nodes, arcs, arr(rows)


def test_random_streams():
    rng = np.random.default_rng(2024)
    shrunk = 0
    for _ in range(40):
        nodes, arcs, d = random_stream(rng)
        c = check_equivalent(nodes, arcs, d)
        shrunk += d.shape[0] - c.shape[0]
    assert shrunk > 0


def test_churn_rounds_concatenated():
    """Config-4 churn (ksched_amd/churn.py), three rounds batched into one stream
    (a daemon that falls behind a round): pins of tasks completed in the same
    batch and repeated ageing of one arc collapse."""
    cell = churn.Cell(300, 30, 3, 5, 11)
    g = cell.graph()
    nodes = {i + 1: (int(g.supply[i]), int(g.ntype[i])) for i in range(g.n)}
    arcs = {(int(s), int(t)): (int(lo), int(c), int(co), int(ty))
            for s, t, lo, c, co, ty in zip(g.src, g.dst, g.low, g.cap, g.cost, g.atype)}
    parts = []
    for _ in range(3):
        gg = cell.graph()
        st, _, _, fl = ko.cost_scaling(gg)
        assert st == 0
        parts.append(cell.step(flow_mapping(gg, fl), done=40, arrive=50))
    d = np.concatenate(parts)
    c = check_equivalent(nodes, arcs, d)
    assert c.shape[0] < d.shape[0]
