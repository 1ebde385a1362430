"""GPU parity: the HIP solver (through the C-ABI) against the CPU oracle and the
committed goldens. Bit-exact total cost and flow value; flows verified for
capacity and conservation; task mappings validated (SURVEY §7 hard part 5)."""
import numpy as np
import pytest

from conftest import CELL_ANY, load_goldens, load_known_answers
from graphs import graph_from_lists, random_graphs
from ksched_amd import gen, native
from oracle import ko

pytestmark = pytest.mark.gpu


def flows_by_arc(ctx, g):
    """Per-input-arc flow vector from the f lines."""
    f = ctx.flows()
    idx = {(int(s), int(d)): i for i, (s, d) in enumerate(zip(g.src.tolist(), g.dst.tolist()))}
    out = np.zeros(g.m, np.int64)
    for s, d, x in zip(f["src"].tolist(), f["dst"].tolist(), f["flow"].tolist()):
        out[idx[(s, d)]] = x
    return out


def check_mapping(g, mapping):
    pu_cap = {}
    for s, d, c in zip(g.src.tolist(), g.dst.tolist(), g.cap.tolist()):
        if g.ntype[s - 1] == 2 and g.ntype[d - 1] == 3:
            pu_cap[s] = c
    load = {}
    for t, p in mapping.items():
        assert g.ntype[t - 1] == 1, "mapped node is not a task"
        assert g.ntype[p - 1] == 2, "task mapped to a non-PU node"   # graph_manager.go:259-262
        load[p] = load.get(p, 0) + 1
    for p, k in load.items():
        assert k <= pu_cap.get(p, k), "PU over capacity"


def solve_and_check(ctx, g, cost, flow, check_flows=True):
    ctx.load_graph(g)
    r = ctx.solve()
    assert r.cost == cost
    assert r.flow == flow
    # a certificate repair must not hide an ε-optimality bug — no
    # recovery may run unless a test injects the fault
    if not ctx.opts.fault_inject:
        assert r.raw["recoveries"] == 0, "the optimality certificate needed a repair"
    if check_flows:
        fl = flows_by_arc(ctx, g)
        st, c2, _ = ko.verify(g, fl)
        assert st == 0, "oracle verifier rejected the GPU flow"
        assert c2 == cost
    return r


def test_config1_known_answer(any_ctx):
    ctx = any_ctx
    ka = load_known_answers()["config1"]
    g = gen.trivial(*ka["params"])
    assert (g.n, g.m) == (ka["n"], ka["m"])
    solve_and_check(ctx, g, ka["cost"], ka["flow"])
    mp = ctx.task_mapping()
    assert len(mp) == 100          # every pod placed through the cluster EC (cost 2 < 5)
    check_mapping(g, mp)


def test_multi_schedule_round1(ctx):
    r1 = load_known_answers()["multi_schedule_iteration"]["round1_graph"]
    g = graph_from_lists(r1["nodes"], r1["arcs"])
    solve_and_check(ctx, g, r1["cost"], r1["flow"])
    mp = ctx.task_mapping()
    assert len(mp) == 2
    check_mapping(g, mp)


@pytest.mark.parametrize("e", [e for e in load_goldens() if e["m"] <= 60000 and not 1004 <= e["seed"] < 1064],
                         ids=lambda e: f"{e['family']}-{'x'.join(map(str, e['params']))}-s{e['seed']}")
def test_goldens(any_ctx, e):
    ctx = any_ctx
    g = gen.trivial(*e["params"]) if e["family"] == "trivial" else gen.quincy(*e["params"], e["seed"])
    r = solve_and_check(ctx, g, e["cost"], e["flow"])
    # which path ran: the cell solver holds every golden up to config-2 size
    assert r.raw["solver"] == (0 if ctx.opts.cell_nodes < 0 else 1)
    check_mapping(g, ctx.task_mapping())


def test_reference_bfs_accepts_gpu_flow(ctx):
    """The reference's own decomposition (solver.go:183-269) over the GPU f lines."""
    g = gen.quincy(3000, 300, 12, 30, 10)
    ctx.load_graph(g)
    r = ctx.solve()
    fl = flows_by_arc(ctx, g)
    ref_map = ko.bfs_mapping(g, fl, r.cost)
    mp = ctx.task_mapping()
    assert len(ref_map) == len(mp)
    check_mapping(g, ref_map)


def test_config3_full_size(ctx):
    T, M, R, J, seed = gen.CONFIGS["config3"]
    g = gen.quincy(T, M, R, J, seed)
    gold = [e for e in load_goldens() if e["params"] == [T, M, R, J] and e["seed"] == seed]
    if gold:
        cost = gold[0]["cost"]
    else:
        st, cost, fv, _ = ko.cost_scaling(g)
        assert st == 0
    solve_and_check(ctx, g, cost, T)
    check_mapping(g, ctx.task_mapping())


# ----------------------------------------------------------------- edge cases ---
def test_empty_graph(any_ctx):
    ctx = any_ctx
    ctx.load_arrays(np.zeros(0, native.NODE_DT), np.zeros(0, native.ARC_DT))
    r = ctx.solve()
    assert (r.cost, r.flow) == (0, 0)


def test_isolated_nodes_no_arcs(any_ctx):
    ctx = any_ctx
    nodes = [(1, 0, 3), (2, 0, 0), (5, 0, 1)]
    g = graph_from_lists(nodes, np.zeros((0, 5), np.int64))
    ctx.load_graph(g)
    r = ctx.solve()
    assert (r.cost, r.flow) == (0, 0)


def test_infeasible_reports_error(any_ctx):
    ctx = any_ctx
    # 3 tasks, one PU slot, no unscheduled escape → supply cannot reach the sink
    nodes = [(1, -3, 3), (2, 0, 2), (3, 1, 1), (4, 1, 1), (5, 1, 1)]
    arcs = [(2, 1, 0, 1, 0), (3, 2, 0, 1, 1), (4, 2, 0, 1, 1), (5, 2, 0, 1, 1)]
    g = graph_from_lists(nodes, arcs)
    ctx.load_graph(g)
    with pytest.raises(native.KsError) as ei:
        ctx.solve()
    assert ei.value.code == native.KS_E_INFEASIBLE


def test_lower_bound_running_arc(any_ctx):
    ctx = any_ctx
    # pinned task: running arc low=1 cap=1 to a PU (graph_manager.go:675-720)
    nodes = [(1, -2, 3), (2, 0, 2), (3, 0, 2), (4, 1, 1), (5, 1, 1), (6, 0, 0)]
    arcs = [(2, 1, 0, 5, 0), (3, 1, 0, 5, 0), (4, 3, 1, 1, 7), (5, 2, 0, 1, 3), (5, 6, 0, 1, 5), (6, 1, 0, 2, 0)]
    g = graph_from_lists(nodes, arcs)
    st, c, fv, _, _ = ko.ssp(g)
    assert st == 0
    solve_and_check(ctx, g, c, fv)
    assert ctx.task_mapping() == {4: 3, 5: 2}


def test_random_graphs_vs_oracle(any_ctx):
    ctx = any_ctx
    for trial, g in random_graphs(12345, 40):
        st, c, fv, _, _ = ko.ssp(g)
        ctx.load_graph(g)
        if st == 0:
            solve_and_check(ctx, g, c, fv)
        else:
            with pytest.raises(native.KsError) as ei:
                ctx.solve()
            assert ei.value.code == native.KS_E_INFEASIBLE


def test_deltas_match_full_reload(ctx):
    """Incremental protocol (ExportIncremental: n / r / a / x lines) vs a full export."""
    g = gen.quincy(1000, 100, 5, 10, 4)
    ctx.load_graph(g)
    r0 = ctx.solve()
    # complete the first 50 tasks ("r id"), add 30 new tasks with 5 arcs each,
    # raise the unscheduled cost of 100 waiting tasks ("x" lines)
    R, M = 5, 100
    TASK0 = 3 + R + 2 * M + 10
    U0 = 3 + R + 2 * M
    d = []
    removed = list(range(TASK0, TASK0 + 50))
    for t in removed:
        d.append(dict(kind=native.KS_REMOVE_NODE, id=t))
    new_ids = removed[:30]     # FIFO id reuse (graph.go:169-182)
    rng = np.random.default_rng(7)
    new_arcs = []
    for t in new_ids:
        d.append(dict(kind=native.KS_ADD_NODE, id=t, excess=1, type=1))
        j = int(rng.integers(0, 10))
        m1, m2 = (int(x) for x in rng.choice(M, 2, replace=False))
        for dst, cost in ((U0 + j, 500), (2, 250), (3 + int(rng.integers(0, R)), 100),
                          (3 + R + m1, 10), (3 + R + m2, 20)):
            d.append(dict(kind=native.KS_ADD_ARC, src=t, dst=dst, low=0, cap=1, cost=cost))
            new_arcs.append((t, dst, 0, 1, cost))
    upd = {}
    src, dst, cost = g.src.tolist(), g.dst.tolist(), g.cost.tolist()
    for i in range(5 * 60, 5 * 160, 5):     # task→U arcs of 100 surviving tasks
        d.append(dict(kind=native.KS_UPDATE_ARC, src=src[i], dst=dst[i], low=0, cap=1, cost=cost[i] + 10,
                      old_cost=cost[i]))
        upd[(src[i], dst[i])] = cost[i] + 10
    arr = np.zeros(len(d), native.DELTA_DT)
    for i, x in enumerate(d):
        for k, v in x.items():
            arr[i][k] = v
    ctx.apply_deltas(arr)
    r1 = ctx.solve()
    # equivalent full graph
    keep = [i for i in range(g.m) if src[i] not in removed and dst[i] not in removed]
    arcs = [(src[i], dst[i], int(g.low[i]), int(g.cap[i]), upd.get((src[i], dst[i]), cost[i])) for i in keep]
    arcs += new_arcs
    sup = g.supply.copy()
    for t in removed[30:]:
        sup[t - 1] = 0
    sup[0] = -int(sup[1:].sum())          # auto-sink: the sink absorbs every other supply
    nodes = [(i + 1, int(sup[i]), int(g.ntype[i])) for i in range(g.n)]
    h = graph_from_lists(nodes, arcs)
    st, c, fv, _, _ = ko.ssp(h)
    assert st == 0
    assert (r1.cost, r1.flow) == (c, fv)
    assert r0.flow == 1000 and r1.flow == 980


def test_device_decomposition_matches_pu_flows(ctx):
    """The device path decomposition hands out exactly the units each PU sends
    to the sink: per PU, mapped tasks == flow on PU→sink (every unit through a
    PU comes from a task in the Quincy shape)."""
    g = gen.quincy(5000, 500, 20, 50, 31)
    ctx.load_graph(g)
    ctx.solve()
    fl = flows_by_arc(ctx, g)
    mp = ctx.task_mapping()
    per_pu = {}
    for p in mp.values():
        per_pu[p] = per_pu.get(p, 0) + 1
    for i in range(g.m):
        s, d = int(g.src[i]), int(g.dst[i])
        if g.ntype[s - 1] == 2 and g.ntype[d - 1] == 3:
            assert per_pu.get(s, 0) == int(fl[i])
    # and the tasks left unmapped are exactly those whose unit ends unscheduled (→ U_j → sink)
    sched = sum(int(fl[i]) for i in range(g.m) if g.ntype[int(g.src[i]) - 1] == 2)
    assert len(mp) == sched


def test_out_of_range_update_is_rejected_without_side_effects(ctx):
    """An "x" record whose id does not fit the store's key space is rejected
    (KS_E_RANGE) instead of aliasing another arc: x 0 2^32+5 0 0 would otherwise
    hash like arc 1→5 and delete it."""
    nodes = [(1, 1, 1), (2, 0, 2), (3, -1, 3), (5, 0, 0)]
    arcs = [(1, 5, 0, 1, 4), (5, 3, 0, 1, 0), (1, 2, 0, 1, 9), (2, 3, 0, 1, 0)]
    g = graph_from_lists(nodes, arcs)
    ctx.load_graph(g)
    bad = np.zeros(1, native.DELTA_DT)
    bad[0]["kind"], bad[0]["src"], bad[0]["dst"] = native.KS_UPDATE_ARC, 0, (1 << 32) + 5
    with pytest.raises(native.KsError) as ei:
        ctx.apply_deltas(bad)
    assert ei.value.code == native.KS_E_RANGE
    r = ctx.solve()
    assert (r.cost, r.flow) == (4, 1)      # 1→5→3 still there


def test_mapping_with_flow_cycles_terminates_and_respects_pus(ctx):
    """Task → PU decomposition on graphs whose optimal flow may run round
    zero-cost cycles between intermediate nodes (ksched's own graphs are DAGs;
    DESIGN §8 item 1): it must terminate, map only tasks to PUs, and keep every
    PU within its PU → sink capacity."""
    rng = np.random.default_rng(2024)
    for trial in range(6):
        T, K, P = 40, 12, 8                       # tasks, intermediate nodes, PUs
        sink = 1
        inter = list(range(2, 2 + K))
        pus = list(range(2 + K, 2 + K + P))
        tasks = list(range(2 + K + P, 2 + K + P + T))
        nodes = [(sink, -T, 3)] + [(v, 0, 0) for v in inter] + [(p, 0, 2) for p in pus] + [(t, 1, 1) for t in tasks]
        arcs = {}
        for t in tasks:                            # each task: two intermediates and the sink (unscheduled)
            for v in rng.choice(inter, 2, replace=False).tolist():
                arcs[(t, v)] = (0, 1, int(rng.integers(1, 20)))
            arcs[(t, sink)] = (0, 1, 200)
        for _ in range(3 * K):                     # zero-cost arcs among intermediates (cycles)
            a, b = rng.choice(inter, 2, replace=False).tolist()
            arcs[(a, b)] = (0, int(rng.integers(1, 6)), 0)
        for v in inter:
            for p in rng.choice(pus, 2, replace=False).tolist():
                arcs[(v, p)] = (0, int(rng.integers(1, 8)), int(rng.integers(0, 5)))
        for p in pus:
            arcs[(p, sink)] = (0, 4, 0)
        g = graph_from_lists(nodes, [(s, d, lo, c, w) for (s, d), (lo, c, w) in arcs.items()])
        st, cost, fv, _, _ = ko.ssp(g)
        assert st == 0
        ctx.load_graph(g)
        r = ctx.solve()
        assert (r.cost, r.flow) == (cost, fv), trial
        check_mapping(g, ctx.task_mapping())


@pytest.mark.parametrize("opts", [{"walk_slack": -1}, {"walk_slack": 1}, {"walk_slack": 4, "tail_sweeps": 2}])
def test_tail_walks_do_not_change_the_optimum(opts):
    """The phase-tail walks (k_augment / k_aug_hub) off, at slack 1
    (ε-optimality kept) and at the default slack with the fewest tail sweeps —
    set through ks_opts, not the environment: the same optimal cost and flow, the
    flow re-verified by the oracle — on a config-2-sized Quincy cell (hub excess
    in every phase's tail) and on random graphs with several deficits, lower
    bounds and parallel paths."""
    with native.Context(0, cell_nodes=-1, **opts) as c2:   # the engine's tail (the cell solver has none)
        g = gen.quincy(10_000, 1_000, 25, 100, 2)
        st, c, fv, _, _ = ko.ssp(g)
        assert st == 0
        solve_and_check(c2, g, c, fv)
        for trial, g in random_graphs(777, 15):
            st, c, fv, _, _ = ko.ssp(g)
            if st == 0:
                solve_and_check(c2, g, c, fv)


@pytest.mark.parametrize("opts", [{"fwd_nodes": -1}, {"fwd_nodes": 64}, {"fwd_nodes": 4096, "tail_nodes": 4096},
                                  {"bf_bound": -1}, {"fwd_nodes": 16, "price_refine": 0}])
def test_tail_updates_do_not_change_the_optimum(opts):
    """The tail's update kinds: the forward update (a search from the
    excess nodes to the nearest deficit, pushes along its shortest paths) off,
    from 64 excess nodes, from any count (every cycle once a phase is in its
    tail), and down to ε = 1 without price refinement; the bounded global update
    off. Same optimum as the oracle, flow re-verified, on a config-2-sized cell
    and random graphs (several deficits, lower bounds, parallel paths)."""
    # α 8: a config-2 solve at its default α (32 on the engine below 32,768 nodes)
    # has no coarse phase with a tail
    with native.Context(0, cell_nodes=-1, alpha=8, **opts) as c2:   # the engine's tail updates
        g = gen.quincy(10_000, 1_000, 25, 100, 2)
        st, c, fv, _, _ = ko.ssp(g)
        assert st == 0
        fwd = solve_and_check(c2, g, c, fv).raw["fwd_updates"]
        for trial, g in random_graphs(4242, 15):
            st, c, fv, _, _ = ko.ssp(g)
            if st == 0:
                fwd += solve_and_check(c2, g, c, fv).raw["fwd_updates"]
        # the forward update really ran where it is on
        if opts.get("fwd_nodes", 64) in (64, 4096) and opts.get("bf_bound", 1) >= 0:
            assert fwd > 0, "no forward tail update ran"


@pytest.mark.parametrize("fault,path", [(1, "engine"), (2, "engine"), (2, "cell")])
def test_failed_certificate_is_recovered(fault, path):
    """A failed final optimality certificate is repaired, not fatal
    (replaces the panic of placement/solver.go:223-225 on a bad solve):
    fault 1 — with price refinement off the ladder runs down to ε = 1 and the
    last phase's walks use the coarse slack (the flow may end 4-optimal only);
    fault 2 — an optimal flow whose prices are perturbed before verification.
    Either way the solve returns the oracle's cost, the flow re-verified, and
    fault 2 always needs (and counts) a recovery — on the engine and inside the
    cell solver's workgroups (its recovery mode: refinement, else one ε = 1 phase)."""
    opts = {"fault_inject": fault, "cell_nodes": -1 if path == "engine" else CELL_ANY}
    if fault == 1:
        opts["price_refine"] = 0
    with native.Context(0, **opts) as c2:
        for g in (gen.quincy(10_000, 1_000, 25, 100, 2), gen.quincy(3_000, 300, 12, 30, 10)):
            st, c, fv, _, _ = ko.ssp(g)
            r = solve_and_check(c2, g, c, fv)
            assert r.raw["solver"] == (1 if path == "cell" else 0)
            if fault == 2:
                assert r.raw["recoveries"] >= 1
            assert r.raw["recoveries"] <= 2


def test_failed_load_leaves_the_context_usable(ctx):
    """a load rejected for a bad arc changes nothing (host table and
    device store); a later apply + solve works on the previous graph."""
    g = gen.quincy(1_000, 100, 5, 10, 1)
    st, c, fv, _, _ = ko.ssp(g)
    ctx.load_graph(g)
    r = ctx.solve()
    assert (r.cost, r.flow) == (c, fv)
    nodes, arcs = native.graph_arrays(gen.quincy(500, 50, 5, 10, 9))
    arcs[3]["dst"] = 10 ** 6                      # an endpoint that does not exist
    with pytest.raises(native.KsError) as e:
        ctx.load_arrays(nodes, arcs)
    assert e.value.code == native.KS_E_INVALID
    d = np.zeros(1, native.DELTA_DT)              # a no-op upsert of an existing arc
    d[0]["kind"] = native.KS_ADD_ARC
    d[0]["src"], d[0]["dst"], d[0]["cap"], d[0]["cost"] = g.src[0], g.dst[0], g.cap[0], g.cost[0]
    ctx.apply_deltas(d)
    r = ctx.solve()
    assert (r.cost, r.flow) == (c, fv)
    check_mapping(g, ctx.task_mapping())


@pytest.mark.parametrize("path", ["engine", "cell"])
def test_verifier_checks_conservation_from_the_flows(path):
    """The verifier balances every node from the arc flows the caller downloads
    (plus its supply), not from the solver's excess words: fault_inject bit 6
    moves one unit on an arc after the solve without touching any excess, and the
    solve must fail with KS_E_VERIFY (conservation) instead of returning a flow
    that breaks it (north star: conservation verified on every solve)."""
    g = gen.quincy(2_000, 200, 5, 20, 4)
    with native.Context(0, cell_nodes=20_000 if path == "cell" else -1, fault_inject=64) as c:
        c.load_graph(g)
        with pytest.raises(native.KsError) as e:
            c.solve()
        assert e.value.code == native.KS_E_VERIFY
        assert "conservation" in str(e.value)


def test_cell_range_fallback_on_a_warm_start():
    """a warm solve whose new costs no longer fit the cell solver's
    compact record (scaled cost · (n+1) beyond int32) falls back to the engine; the
    warm start's price shift is applied once, and the result equals the oracle's,
    then and on the next warm solve."""
    g = gen.quincy(1_000, 100, 5, 10, 31)          # 1,217 nodes: the cell solver by default
    with native.Context(0, warm_start=1) as ctx:
        ctx.load_graph(g)
        r0 = ctx.solve()
        assert r0.raw["solver"] == 1
        assert (r0.cost, r0.flow) == ko.cost_scaling(g)[1:3]
        src, dst, cost = g.src.tolist(), g.dst.tolist(), g.cost.tolist()
        big = 3_000_000                            # × 1,218 > 2^31
        d = np.zeros(50, native.DELTA_DT)
        upd = {}
        for k, i in enumerate(range(0, 5 * 50, 5)):   # task → U arcs (ageing)
            d[k]["kind"], d[k]["src"], d[k]["dst"], d[k]["cap"] = native.KS_UPDATE_ARC, src[i], dst[i], 1
            d[k]["cost"], d[k]["old_cost"] = cost[i] + big, cost[i]
            upd[i] = cost[i] + big
        ctx.apply_deltas(d)
        h = gen.Graph(g.ntype, g.supply, g.src, g.dst, g.low, g.cap,
                      np.asarray([upd.get(i, c) for i, c in enumerate(cost)], np.int64))
        want = ko.cost_scaling(h)[1:3]
        r1 = ctx.solve()
        assert r1.raw["solver"] == 0 and r1.raw["warm_started"] == 1
        assert (r1.cost, r1.flow) == want
        r2 = ctx.solve()
        assert (r2.cost, r2.flow) == want


@pytest.mark.parametrize("path,opts", [("engine", {}), ("engine", {"price_refine": 2}),
                                       ("engine", {"fault_inject": 32}), ("engine", {"compact_pos": -1}),
                                       ("cell", {}), ("cell", {"price_refine": 2}), ("cell", {"fault_inject": 32})])
def test_cycle_cancelling_finish(path, opts):
    """The cycle-cancelling finish (ks_opts.price_refine 1): the
    last coarse phase drains, then price refinement cancels the negative cycles of
    its parent graph until it certifies the flow. Against the plain final phase
    (price_refine 2), the finish giving up early (fault_inject bit 5: the final
    phase follows), and the engine's 32-B records: the same optimum as the oracle
    on config-2-sized graphs (on the engine and in the cell solver) and random
    graphs, every flow re-verified."""
    cc = 0
    cell = path == "cell"
    with native.Context(0, cell_nodes=20_000 if cell else -1, **opts) as c2:
        for seed in (2, 7, 11):
            g = gen.quincy(10_000, 1_000, 25, 100, seed)
            st, c, fv, _ = ko.cost_scaling(g)
            assert st == 0
            r = solve_and_check(c2, g, c, fv)
            assert r.raw["solver"] == (1 if cell else 0)
            cc += r.raw["cycles_cancelled"]
            assert r.raw["recoveries"] == 0
        for trial, g in random_graphs(9191, 12):
            st, c, fv, _, _ = ko.ssp(g)
            if st == 0:
                solve_and_check(c2, g, c, fv)
    if opts.get("price_refine", 1) == 2:
        assert cc == 0
    elif not opts.get("fault_inject"):
        assert cc > 0, "no negative cycle was cancelled on three config-2 cells"


def _search_graphs(with_config3):
    """Three config-2 cells (seeds 2, 7, 11) and, on the engine, config 3 — with the
    oracle's (cost, flow) from the committed goldens or the cost-scaling oracle."""
    out = []
    seeds = [("config2", 2), ("config2", 7), ("config2", 11)] + ([("config3", 3)] if with_config3 else [])
    gold = {(tuple(e["params"]), e["seed"]): e for e in load_goldens() if e["family"] == "quincy"}
    for name, seed in seeds:
        T, M, R, J, _ = gen.CONFIGS[name]
        g = gen.quincy(T, M, R, J, seed)
        e = gold.get(((T, M, R, J), seed))
        if e is not None:
            want = (e["cost"], e["flow"])
        else:
            st, c, fv, _ = ko.cost_scaling(g)
            assert st == 0
            want = (c, fv)
        out.append((g, want))
    return out


@pytest.mark.parametrize("path", ["engine", "cell"])
def test_cycle_search_rejects_chains(path):
    """the finish's union-of-cycles test on its rejection path.
    fault_inject bit 7 shortens every parent-graph search to a 32-node window, far
    shorter than the refinement's parent chains, so chain nodes get marked and run
    into cycles' groups (the case that once pushed along a chain and returned
    3,257,657 with KS_OK). The test must reject them (cycles_rejected > 0) and the
    cycles it keeps must still be cancelled: every solve returns the oracle's cost
    with no recovery and no KS_E_VERIFY — on three config-2 cells and config 3 on
    the engine (k_cyc_check), and on the config-2 cells in the cell solver (whose
    leader walk must close on itself). Config 3 is beyond the cell solver's size."""
    cell = path == "cell"
    cc = rej = 0
    with native.Context(0, cell_nodes=20_000 if cell else -1, fault_inject=128) as c2:
        for g, (cost, flow) in _search_graphs(with_config3=not cell):
            r = solve_and_check(c2, g, cost, flow)
            assert r.raw["solver"] == (1 if cell else 0)
            assert r.raw["recoveries"] == 0
            cc += r.raw["cycles_cancelled"]
            rej += r.raw["cycles_rejected"]
    assert cc > 0, "no cycle was cancelled through the short window"
    assert rej > 0, "the short window never produced a group the test had to reject"


def test_cycle_search_without_the_check_fails_loudly():
    """The same short window with the engine's union-of-cycles test only counting
    (fault_inject bit 8): groups joined by a chain are then pushed along, which
    breaks conservation. The verifier (conservation from the downloaded flows) must
    turn that into KS_E_VERIFY on at least one graph — and no solve may return a
    cost other than the oracle's."""
    failed = 0
    with native.Context(0, cell_nodes=-1, fault_inject=128 | 256) as c2:
        for g, (cost, flow) in _search_graphs(with_config3=True):
            c2.load_graph(g)
            try:
                r = c2.solve()
            except native.KsError as e:
                assert e.code == native.KS_E_VERIFY, str(e)
                failed += 1
                continue
            assert (r.cost, r.flow) == (cost, flow)
    assert failed > 0, "no chain was pushed along: the unchecked search never met the bad case"


def test_kind_timing_and_counters():
    """The per-kind device times the bench's roofline divides by (ks_result ABI 3/5):
    the Bellman-Ford rounds by HIP events less the finish's searches (device
    clock), the sweeps by the device clock — each positive and together within the
    solve's own time; and both hops of a Bellman-Ford round counted (the second,
    a task's or PU's own in-arcs in the same launch: gu_leaf_scans)."""
    g = gen.quincy(10_000, 1_000, 25, 100, 2)
    with native.Context(0, cell_nodes=-1) as c:
        c.load_graph(g)
        for _ in range(2):
            r = c.solve()
            raw = r.raw
            assert raw["ms_gu_kernels"] > 0 and raw["ms_sweep_kernels"] > 0
            assert raw["ms_gu_kernels"] + raw["ms_sweep_kernels"] < raw["ms"]["total"]
            assert raw["gu_arc_scans"] > 0 and raw["gu_leaf_scans"] > 0
            assert raw["gu_launches"] >= raw["gu_iterations"] > 0
