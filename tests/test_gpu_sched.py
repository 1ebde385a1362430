"""GPU: the scheduler-side sweeps of a round on the device-resident graph (SURVEY
§8 row f) against CPU restatements of the reference (oracle/sched_ref.py) and
against the reference's own harness replayed (tests/golden/multi_schedule_iteration.json):
scheduling deltas (graph_manager.go:253-339), ComputeTopologyStatistics
(:480-511) and UpdateAllCostsToUnscheduledAggs (:462-475)."""
import numpy as np
import pytest

from graphs import graph_from_lists, load_multi_schedule, parse_dimacs, same_graph
from ksched_amd import churn, gen, native
from oracle import ko, sched_ref

pytestmark = pytest.mark.gpu


def as_list(d):
    return [(int(x["type"]), int(x["task"]), int(x["pu"])) for x in d]


def test_multi_schedule_deltas_and_statistics():
    """Each round of TestMultiScheduleIteration: the device's topology statistics
    equal the reference's at the round's start, and its scheduling deltas equal
    the restatement of NodeBindingToSchedulingDelta on the device's own mapping
    (2 PLACEs in rounds 1 and 4, nothing in rounds 2, 3 and 5, as in the reference)."""
    rounds = load_multi_schedule()
    bindings = {}
    with native.Context(0) as ctx:
        for r in rounds:
            nodes, arcs, d = parse_dimacs(r["dimacs"])
            if r["kind"] == "full":
                ctx.load_graph(graph_from_lists(nodes, arcs))
            else:
                ctx.apply_deltas(d)
                gone = set(int(x) for x in d["id"][d["kind"] == native.KS_REMOVE_NODE])
                bindings = {t: p for t, p in bindings.items() if t not in gone}   # HandleTaskCompletion
            # ComputeTopologyStatistics with the reference's CurrentRunningTasks lengths
            ts = r["topology_stats"]
            sl, rn = ctx.topology_stats(1, {int(k): v for k, v in ts["pu_running"].items()})
            for nid, (slots, running) in ts["slots_running"].items():
                assert (int(sl[int(nid) - 1]), int(rn[int(nid) - 1])) == (slots, running), (r["round"], nid)
            res = ctx.solve()
            mp = ctx.task_mapping()
            want = sched_ref.scheduling_deltas(bindings, mp, list(mp) + list(bindings))
            got = as_list(ctx.scheduling_deltas(commit=False))
            assert got == want, r["round"]
            assert [k for k, _, _ in got] == [sched_ref.PLACE if k == "PLACE" else k for k, _, _ in r["deltas"]]
            # keep the device's bindings in step with the stream's pins (the fixture's placements)
            old = bindings
            bindings = {int(t): int(p) for t, p in r["mapping"].items()}
            ctx.set_bindings({t: 0 for t in old if t not in bindings} | bindings)
            assert res.cost == r["cost"]


def test_scheduling_deltas_commit_over_churn_rounds():
    """Config-4 churn at config-2 size: the device deltas (committed on device)
    equal the restatement every round; completions unbind tasks on device."""
    cell = churn.Cell(10_000, 1_000, 25, 100, 12)
    bindings = {}
    with native.Context(0) as ctx:
        ctx.load_graph(cell.graph())
        ctx.solve()
        mp = ctx.task_mapping()
        got = as_list(ctx.scheduling_deltas(commit=True))
        assert got == sched_ref.scheduling_deltas(bindings, mp, mp.keys())
        bindings = sched_ref.apply_deltas(bindings, got)
        for _ in range(3):
            d = cell.step(mp, done=500, arrive=500)
            gone = set(int(x) for x in d["id"][d["kind"] == native.KS_REMOVE_NODE])
            bindings = {t: p for t, p in bindings.items() if t not in gone}
            ctx.apply_deltas(d)
            ctx.solve()
            mp = ctx.task_mapping()
            live = cell.task_ids(cell.RUN).tolist() + cell.task_ids(cell.WAIT).tolist()
            want = sched_ref.scheduling_deltas(bindings, mp, live)
            got = as_list(ctx.scheduling_deltas(commit=True))
            assert got == want
            assert all(k == sched_ref.PLACE for k, _, _ in got)   # pinned tasks never move (low = 1)
            bindings = sched_ref.apply_deltas(bindings, got)


def test_topology_statistics_config3_size():
    """ComputeTopologyStatistics on the config-3 cell (X → racks → machines → PUs
    → sink; X plays the coordinator): device BFS vs the FIFO restatement."""
    T, M, R, J, seed = gen.CONFIGS["config3"]
    g = gen.quincy(T, M, R, J, seed)
    rng = np.random.default_rng(5)
    pus = (np.nonzero(g.ntype == 2)[0] + 1).tolist()
    running = {p: int(x) for p, x in zip(pus, rng.integers(0, 4, len(pus)))}
    # resources: PUs, machines, the racks and X (type 0 here, like ksched's coordinator)
    resource = set((np.nonzero(np.isin(g.ntype, [2, 4, 5]))[0] + 1).tolist()) | set(range(2, 3 + R))
    want = sched_ref.topology_stats(g, resource, running, 10)
    with native.Context(0) as ctx:
        ctx.load_graph(g)
        sl, rn = ctx.topology_stats(10, running)
    got = {v: (int(sl[v - 1]), int(rn[v - 1])) for v in resource}
    assert got == want
    assert got[2] == (10 * M, sum(running.values()))


def test_unscheduled_cost_ageing_on_device_matches_the_stream():
    """UpdateAllCostsToUnscheduledAggs on device (ADD 10 per round to every waiting
    task's arc into its unscheduled aggregator, before the round's stream) gives
    the same graph — and the same optimum — as the stream's own ageing records."""
    cell_a = churn.Cell(10_000, 1_000, 25, 100, 9)
    cell_b = churn.Cell(10_000, 1_000, 25, 100, 9)
    with native.Context(0) as a, native.Context(0) as b:
        for c, cell in ((a, cell_a), (b, cell_b)):
            c.load_graph(cell.graph())
            c.solve()
        mp = a.task_mapping()
        for _ in range(3):
            waiting = int((cell_b.state[:cell_b.n_slots] == cell_b.WAIT).sum())
            da = cell_a.step(mp, done=500, arrive=500)                       # ageing in the stream
            changed = b.update_unsched_costs(10, native.KS_COST_ADD)        # ageing on device ...
            db = cell_b.step(mp, done=500, arrive=500, age_cost=0)          # ... and not in the stream
            assert changed == waiting                # every task waiting before the round
            a.apply_deltas(da)
            b.apply_deltas(db)
            same_graph(b, cell_a.graph())
            ra, rb = a.solve(), b.solve()
            st, cost, flow, _ = ko.cost_scaling(cell_a.graph())
            assert st == 0 and ra.cost == cost and rb.cost == cost
            mp = a.task_mapping()


def test_trivial_model_unscheduled_refresh_changes_nothing():
    """With the trivial model every task→U arc already costs 5
    (trivial_cost_modeler.go:41-43): the refresh emits no change, as
    ChangeArcCost does not when the cost is equal (graph_change_manager.go:171-182)."""
    g = gen.trivial(10, 1000, 100)
    with native.Context(0) as ctx:
        ctx.load_graph(g)
        assert ctx.update_unsched_costs(5, native.KS_COST_SET) == 0
        r = ctx.solve()
        assert (r.cost, r.flow) == (200, 100)
        assert ctx.update_unsched_costs(7, native.KS_COST_SET) == 100
        assert ctx.solve().cost == 200       # still cheaper through the EC (2 < 7)
