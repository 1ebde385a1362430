"""Differential stress: medium general graphs with hubs (tests/graphs.py
random_hub_graphs: 300–6,000 nodes, one to four nodes joined to a quarter to all
of the others, antiparallel and zero-capacity arcs, large capacities, lower
bounds out of sources, several sources and sinks) through both solver paths,
against the oracle's successive shortest path (the reference's algorithm,
placement/solver.go:32). Bit-exact cost and flow value, the oracle's verifier
on the downloaded flows, no certificate repair; an infeasible graph must fail
with KS_E_INFEASIBLE."""
import numpy as np
import pytest

from graphs import random_hub_graphs
from ksched_amd import native
from oracle import ko
from test_gpu_parity import solve_and_check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [2026, 2027])
def test_random_hub_graphs_vs_oracle(any_ctx, seed, request):
    ctx = any_ctx
    feasible = infeasible = on_cell = 0
    for trial, g in random_hub_graphs(seed, 16):
        st, cost, fv, _, _ = ko.ssp(g)
        if st == 0:
            r = solve_and_check(ctx, g, cost, fv)
            feasible += 1
            on_cell += r.raw["solver"] == 1
        else:
            ctx.load_graph(g)
            with pytest.raises(native.KsError) as ei:
                ctx.solve()
            assert ei.value.code == native.KS_E_INFEASIBLE, f"trial {trial}"
            infeasible += 1
    assert feasible >= 8 and infeasible >= 1
    # the cell path really ran the cell solver (one workgroup per graph), the engine path never
    assert on_cell == (feasible if request.node.callspec.params["any_ctx"] == "cell" else 0)


def test_resolve_is_repeatable(ctx_engine):
    """The same hub graph solved five times in a row on one context: every solve
    starts from the loaded state, so every result is the oracle's (a race in the
    hub paths would show as a different cost or a verifier failure)."""
    for trial, g in random_hub_graphs(99, 6, n_lo=4000, n_hi=6000):
        st, cost, fv, _, _ = ko.ssp(g)
        if st != 0:
            continue
        ctx_engine.load_graph(g)
        for _ in range(5):
            r = ctx_engine.solve()
            assert (r.cost, r.flow) == (cost, fv)
            assert r.raw["recoveries"] == 0


def _random_stream(rng, nodes, arcs, nrec):
    """A random ks_delta stream over the store state (nodes {id: [excess, type]},
    arcs {(s, d): (low, cap, cost)}), applied to that state as it is made: node
    removals (zero-supply nodes; their arcs go with them) and re-additions of the
    freed ids with new arcs, arc upserts, in-place edits, deletions (UPDATE 0/0),
    an arc deleted and re-created inside one stream (the store keeps the LAST
    record for a key), and a few units moved between two sources (SET_EXCESS
    pairs). The generator's expensive feasibility arcs are left alone, so most
    rounds stay feasible."""
    from graphs import apply_deltas_to_arcs
    recs = []
    free_ids = []
    alive = sorted(nodes)
    keep = {x for (s, d), (_, _, c) in arcs.items() if c >= 50_000 for x in (s, d)}   # feasibility arcs' ends

    def emit(**x):
        r = np.zeros(1, native.DELTA_DT)
        for k, v in x.items():
            r[0][k] = v
        apply_deltas_to_arcs(nodes, arcs, r)
        recs.append(r[0])

    keys = list(arcs)
    while len(recs) < nrec:
        op = rng.random()
        if op < 0.05:
            i = int(rng.choice(alive))
            if nodes.get(i, [1])[0] == 0 and i not in keep:
                emit(kind=native.KS_REMOVE_NODE, id=i)
                free_ids.append(i)
                alive = sorted(nodes)
        elif op < 0.10 and free_ids:
            i = free_ids.pop(0)   # FIFO id reuse (graph.go:169-182)
            emit(kind=native.KS_ADD_NODE, id=i, excess=0, type=0)
            alive = sorted(nodes)
            for j in rng.choice(alive, 3, replace=False).tolist():
                if j != i:
                    s, d = (i, j) if rng.random() < 0.5 else (j, i)
                    emit(kind=native.KS_ADD_ARC, src=s, dst=d, low=0, cap=int(rng.integers(1, 30)),
                         cost=int(rng.integers(0, 1000)))
        elif op < 0.40:
            s, d = (int(x) for x in rng.choice(alive, 2, replace=False))
            emit(kind=native.KS_ADD_ARC, src=s, dst=d, low=0, cap=int(rng.integers(0, 30)),
                 cost=int(rng.integers(0, 1000)))
        elif op < 0.90 and keys:
            s, d = keys[int(rng.integers(0, len(keys)))]
            if (s, d) not in arcs or arcs[(s, d)][2] >= 50_000:   # (the generator's feasibility arcs stay)
                continue
            low, cap, cost = arcs[(s, d)]
            r = rng.random()
            if r < 0.3:     # delete (UPDATE to 0/0), sometimes re-created later in this stream
                emit(kind=native.KS_UPDATE_ARC, src=s, dst=d, low=0, cap=0, cost=cost, old_cost=cost)
                if rng.random() < 0.3:
                    emit(kind=native.KS_ADD_ARC, src=s, dst=d, low=0, cap=int(rng.integers(1, 30)),
                         cost=int(rng.integers(0, 1000)))
            else:           # new capacity and cost in place (the flow is clamped)
                emit(kind=native.KS_UPDATE_ARC, src=s, dst=d, low=low, cap=max(low, int(rng.integers(0, 60))),
                     cost=int(rng.integers(0, 1000)), old_cost=cost)
        elif op < 0.92:    # a few units moved from one source to another
            src = [i for i in alive if nodes[i][0] > 3]
            if len(src) < 2:
                continue
            a, b = (int(x) for x in rng.choice(src, 2, replace=False))
            k = int(rng.integers(1, 4))
            emit(kind=native.KS_SET_EXCESS, id=a, excess=nodes[a][0] + k)
            emit(kind=native.KS_SET_EXCESS, id=b, excess=nodes[b][0] - k)
    return np.array(recs, native.DELTA_DT)


@pytest.mark.parametrize("seed,nrec", [(5, 2000), (6, 2000), (7, 20000)])
def test_random_delta_streams_match_full_graph(any_ctx, seed, nrec):
    """Random delta streams (four rounds of 2,000 or of 20,000 records) on a hub
    graph: after ks_apply_deltas the device solve equals the oracle on the full
    graph the test-side restatement of the store builds
    (graphs.apply_deltas_to_arcs), or both are infeasible."""
    from graphs import graph_from_store
    ctx = any_ctx
    rng = np.random.default_rng(seed)
    g = next(g for _, g in random_hub_graphs(seed, 20, n_lo=1500, n_hi=4000) if ko.ssp(g)[0] == 0)
    nodes = {i + 1: [int(g.supply[i]), int(g.ntype[i])] for i in range(g.n)}
    arcs = {(int(s), int(d)): (int(lo), int(c), int(k))
            for s, d, lo, c, k in zip(g.src, g.dst, g.low, g.cap, g.cost)}
    ctx.load_graph(g)
    ctx.solve()
    solved = 0
    for rnd in range(4):
        ctx.apply_deltas(_random_stream(rng, nodes, arcs, nrec))
        h = graph_from_store(nodes, arcs)
        st, cost, fv, _, _ = ko.ssp(h)
        if st == 0:
            r = ctx.solve()
            assert (r.cost, r.flow) == (cost, fv), f"round {rnd}"
            assert r.raw["recoveries"] == 0
            solved += 1
        else:
            with pytest.raises(native.KsError) as ei:
                ctx.solve()
            assert ei.value.code == native.KS_E_INFEASIBLE, f"round {rnd}"
    assert solved >= 2


@pytest.mark.parametrize("bad", ["missing_endpoint", "self_loop", "remove_missing", "add_present"])
def test_large_stream_error_rolls_back(ctx_engine, bad):
    """A 20,000-record stream with one bad record near its end: the call fails,
    nothing of the stream is applied (host or device: all or nothing, ks_host.cpp),
    and the valid stream alone then solves as the oracle says."""
    from graphs import graph_from_store
    rng = np.random.default_rng(11)
    g = next(g for _, g in random_hub_graphs(11, 20, n_lo=3000, n_hi=5000) if ko.ssp(g)[0] == 0)
    nodes = {i + 1: [int(g.supply[i]), int(g.ntype[i])] for i in range(g.n)}
    arcs = {(int(s), int(d)): (int(lo), int(c), int(k))
            for s, d, lo, c, k in zip(g.src, g.dst, g.low, g.cap, g.cost)}
    ctx_engine.load_graph(g)
    ctx_engine.solve()
    before = (dict((k, list(v)) for k, v in nodes.items()), dict(arcs))
    good = _random_stream(rng, nodes, arcs, 20000)
    alive = sorted(nodes)
    row = np.zeros(1, native.DELTA_DT)
    if bad == "missing_endpoint":   # (an id past every node ever present)
        row[0]["kind"], row[0]["src"], row[0]["dst"], row[0]["cap"] = native.KS_ADD_ARC, max(nodes) + 10, alive[0], 1
    elif bad == "self_loop":
        row[0]["kind"], row[0]["src"], row[0]["dst"], row[0]["cap"] = native.KS_ADD_ARC, alive[0], alive[0], 1
    elif bad == "remove_missing":
        row[0]["kind"], row[0]["id"] = native.KS_REMOVE_NODE, max(nodes) + 10
    else:
        row[0]["kind"], row[0]["id"] = native.KS_ADD_NODE, alive[1]
    stream = np.concatenate([good[:19000], row, good[19000:]])
    with pytest.raises(native.KsError) as ei:
        ctx_engine.apply_deltas(stream)
    assert ei.value.code in (native.KS_E_INVALID, native.KS_E_RANGE)
    # nothing applied: the original graph still solves as before
    nodes, arcs = before
    h = graph_from_store(nodes, arcs)
    st, cost, fv, _, _ = ko.ssp(h)
    r = ctx_engine.solve()
    assert (r.cost, r.flow) == (cost, fv)
    # and the valid stream alone applies and solves as the restatement says
    ctx_engine.apply_deltas(good)
    from graphs import apply_deltas_to_arcs
    apply_deltas_to_arcs(nodes, arcs, good)
    h = graph_from_store(nodes, arcs)
    st, cost, fv, _, _ = ko.ssp(h)
    if st == 0:
        r = ctx_engine.solve()
        assert (r.cost, r.flow) == (cost, fv)
