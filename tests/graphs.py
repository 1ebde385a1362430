"""Test graph builders shared by the CPU and GPU suites."""
from __future__ import annotations

import numpy as np

from ksched_amd import gen


def graph_from_lists(nodes, arcs):
    """nodes: [(id, excess, dimacs_type)], arcs: [(src, dst, low, cap, cost)] (1-based ids)."""
    n = max(i for i, _, _ in nodes) if len(nodes) else 0
    ntype = np.zeros(n, np.int32)
    supply = np.zeros(n, np.int64)
    for i, e, t in nodes:
        ntype[i - 1] = t
        supply[i - 1] = e
    a = np.asarray(arcs, np.int64).reshape(-1, 5)
    return gen.Graph(ntype, supply, a[:, 0].copy(), a[:, 1].copy(), a[:, 2].copy(), a[:, 3].copy(),
                     a[:, 4].copy())


def flow_mapping(g, flow) -> dict[int, int]:
    """task → last PU on its unit's path, following positive-flow arcs (the
    scheduling network is a DAG); the test-side twin of ks_get_task_mapping."""
    out = {}
    pos = np.nonzero(np.asarray(flow) > 0)[0]
    nxt: dict[int, list] = {}
    for i in pos.tolist():
        nxt.setdefault(int(g.src[i]), []).append([int(g.dst[i]), int(flow[i])])
    for t in (np.nonzero(g.ntype == 1)[0] + 1).tolist():
        v, last = t, None
        for _ in range(g.n + 1):
            if g.ntype[v - 1] == 2:
                last = v
            lst = nxt.get(v)
            while lst and lst[0][1] == 0:
                lst.pop(0)
            if not lst:
                break
            lst[0][1] -= 1
            v = lst[0][0]
        if last is not None:
            out[t] = last
    return out


def apply_deltas_to_arcs(nodes: dict, arcs: dict, deltas) -> None:
    """Test-side restatement of the graph-store semantics of ks_apply_deltas
    (include/ksmcmf.h): nodes {id: [excess, type]}, arcs {(s, d): (low, cap, cost)}."""
    for x in deltas:
        k = int(x["kind"])
        if k == 0:
            assert int(x["id"]) not in nodes
            nodes[int(x["id"])] = [int(x["excess"]), int(x["type"])]
        elif k == 1:
            i = int(x["id"])
            del nodes[i]
            for key in [a for a in arcs if i in a]:
                del arcs[key]
        elif k == 2:
            s, d = int(x["src"]), int(x["dst"])
            assert s in nodes and d in nodes
            arcs[(s, d)] = (int(x["low"]), int(x["cap"]), int(x["cost"]))
        elif k == 3:
            s, d = int(x["src"]), int(x["dst"])
            if int(x["low"]) == 0 and int(x["cap"]) == 0:
                arcs.pop((s, d), None)
            else:
                arcs[(s, d)] = (int(x["low"]), int(x["cap"]), int(x["cost"]))
        else:
            nodes[int(x["id"])][0] = int(x["excess"])


def dimacs_changes(deltas) -> str:
    """ks_delta records as the incremental DIMACS text of dimacs/*_change.go
    (GenerateChange), terminated by "c EOI" (dimacs/export.go:31-38)."""
    out = []
    for x in deltas:
        k = int(x["kind"])
        if k == 0:
            out.append(f"n {int(x['id'])} {int(x['excess'])} {int(x['type'])}")
        elif k == 1:
            out.append(f"r {int(x['id'])}")
        elif k == 2:
            out.append(f"a {int(x['src'])} {int(x['dst'])} {int(x['low'])} {int(x['cap'])} {int(x['cost'])} "
                       f"{int(x['type'])}")
        elif k == 3:
            out.append(f"x {int(x['src'])} {int(x['dst'])} {int(x['low'])} {int(x['cap'])} {int(x['cost'])} "
                       f"{int(x['type'])} {int(x['old_cost'])}")
        else:
            raise ValueError("SET_EXCESS has no DIMACS record")
    out.append("c EOI")
    return "\n".join(out) + "\n"


def graph_from_store(nodes: dict, arcs: dict):
    n = max(nodes) if nodes else 0
    ntype = np.zeros(n, np.int32)
    supply = np.zeros(n, np.int64)
    for i, (e, t) in nodes.items():
        ntype[i - 1] = t
        supply[i - 1] = e
    sink = np.nonzero(ntype == 3)[0]
    if sink.shape[0] == 1:                  # auto_sink: the sink absorbs every other supply
        supply[sink[0]] = 0
        supply[sink[0]] = -int(supply.sum())
    keys = sorted(arcs)
    a = np.asarray([(s, d, *arcs[(s, d)]) for s, d in keys], np.int64).reshape(-1, 5)
    return gen.Graph(ntype, supply, a[:, 0].copy(), a[:, 1].copy(), a[:, 2].copy(), a[:, 3].copy(),
                     a[:, 4].copy())


def random_graphs(seed: int, count: int, max_n: int = 60, cost_lo: int = 0, cost_hi: int = 100):
    """General digraphs (cycles, antiparallel arcs, zero capacities, some lower
    bounds) with a few random balanced supply/demand pairs; may be infeasible."""
    rng = np.random.default_rng(seed)
    for trial in range(count):
        n = int(rng.integers(4, max_n))
        m = min(int(rng.integers(n, 6 * n)), n * (n - 1) // 2)
        pairs = set()
        arcs = []
        while len(arcs) < m:
            s, d = (int(x) for x in rng.integers(1, n + 1, 2))
            if s == d or (s, d) in pairs:
                continue
            pairs.add((s, d))
            lo = int(rng.integers(0, 2)) if rng.random() < 0.1 else 0
            cap = lo + int(rng.integers(0, 20))
            arcs.append((s, d, lo, cap, int(rng.integers(cost_lo, cost_hi))))
        supply = np.zeros(n, np.int64)
        for _ in range(int(rng.integers(1, 6))):
            a, b = (int(x) for x in rng.integers(0, n, 2))
            k = int(rng.integers(1, 10))
            supply[a] += k
            supply[b] -= k
        nodes = [(i + 1, int(supply[i]), 0) for i in range(n)]
        yield trial, graph_from_lists(nodes, arcs)


def parse_dimacs(text: str):
    """ksched's solver wire text (dimacs/export.go:11-76 for a full graph,
    dimacs/*_change.go GenerateChange for an incremental block) →
    (nodes [(id, excess, type)], arcs [(src, dst, low, cap, cost)], deltas DELTA_DT).
    A full export yields nodes/arcs, a change block yields delta records."""
    from ksched_amd import native
    nodes, arcs, recs = [], [], []
    for line in text.splitlines():
        f = line.split()
        if not f or f[0] in ("c", "p"):
            continue
        v = [int(x) for x in f[1:]]
        if f[0] == "n":
            nodes.append(tuple(v))
            recs.append(dict(kind=native.KS_ADD_NODE, id=v[0], excess=v[1], type=v[2]))
        elif f[0] == "a":
            arcs.append(tuple(v[:5]))
            recs.append(dict(kind=native.KS_ADD_ARC, src=v[0], dst=v[1], low=v[2], cap=v[3], cost=v[4],
                             type=v[5] if len(v) > 5 else 0))
        elif f[0] == "x":
            recs.append(dict(kind=native.KS_UPDATE_ARC, src=v[0], dst=v[1], low=v[2], cap=v[3], cost=v[4],
                             type=v[5], old_cost=v[6] if len(v) > 6 else 0))
        elif f[0] == "r":
            recs.append(dict(kind=native.KS_REMOVE_NODE, id=v[0]))
        else:
            raise ValueError(f"unknown DIMACS record {line!r}")
    d = np.zeros(len(recs), native.DELTA_DT)
    for i, x in enumerate(recs):
        for k, val in x.items():
            d[i][k] = val
    return nodes, arcs, d


def load_multi_schedule():
    """tests/golden/multi_schedule_iteration.json (gen_multi_schedule.py)."""
    import json
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "multi_schedule_iteration.json")
    with open(p) as f:
        return json.load(f)["rounds"]


def same_graph(ctx, g):
    """The device-resident graph (ks_get_graph) equals g up to arcs of capacity 0
    (an "x … 0 0" record removes them from the store)."""
    nodes, arcs = ctx.graph()
    dev = sorted(zip(arcs["src"].tolist(), arcs["dst"].tolist(), arcs["low"].tolist(), arcs["cap"].tolist(),
                     arcs["cost"].tolist()))
    want = sorted(a for a in zip(g.src.tolist(), g.dst.tolist(), g.low.tolist(), g.cap.tolist(), g.cost.tolist())
                  if a[3] > 0)
    assert dev == want
    live = np.nonzero(g.ntype != 0)[0] + 1
    assert set(live.tolist()) <= set(nodes["id"].tolist())


def random_hub_graphs(seed: int, count: int, n_lo: int = 300, n_hi: int = 6000, cost_hi: int = 1000):
    """Medium general graphs for differential testing against the oracle: random
    arcs plus one to four hubs (a node joined to a quarter to all of the others,
    in both directions), a few large capacities, antiparallel
    and zero-capacity arcs, several sources and sinks. Hubs exercise the engine's
    hub chunks and inboxes and the cell solver's workgroup-wide items. Lower
    bounds of 1 sit on some arcs out of sources. Costs are
    non-negative, as in ksched's cost models (the reference's SSP assumes no
    negative cycle). Four in five graphs get expensive source → hub → sink arcs
    that make them feasible; the rest may be infeasible (then the solver must
    say so)."""
    rng = np.random.default_rng(seed)
    for trial in range(count):
        n = int(rng.integers(n_lo, n_hi))
        mb = int(rng.integers(2 * n, 6 * n))
        k = int(rng.integers(2, 40))
        ends = rng.choice(n, 2 * k, replace=False) + 1
        units = rng.integers(1, 200, k)
        hubs = rng.choice(n, int(rng.integers(1, 5)), replace=False) + 1
        src, dst = [], []
        if rng.random() < 0.8:   # feasibility arcs first: they win the de-duplication below
            src += [ends[:k], np.full(k, hubs[0])]
            dst += [np.full(k, hubs[0]), ends[k:]]
        nf = sum(x.shape[0] for x in src)
        src.append(rng.integers(1, n + 1, mb))
        dst.append(rng.integers(1, n + 1, mb))
        for h in hubs:
            deg = int(rng.integers(n // 4, n))
            other = rng.choice(n, deg, replace=False) + 1
            into = rng.random(deg) < 0.5
            src.append(np.where(into, other, h))
            dst.append(np.where(into, h, other))
        src = np.concatenate(src).astype(np.int64)
        dst = np.concatenate(dst).astype(np.int64)
        keep = src != dst
        src, dst = src[keep], dst[keep]
        _, first = np.unique(src * (n + 1) + dst, return_index=True)
        first.sort()
        src, dst = src[first], dst[first]
        m = src.shape[0]
        feas = first < nf   # (first is sorted: kept feasibility arcs come first)
        cap = rng.integers(0, 40, m)
        big = rng.random(m) < 0.03
        cap[big] = rng.integers(1000, 200000, int(big.sum()))
        # lower bounds only on arcs out of sources (as ksched's running arcs out of a
        # pinned task): anywhere else they mostly make a random graph infeasible
        low = np.zeros(m, np.int64)
        lb = np.isin(src, ends[:k]) & (cap > 0) & (rng.random(m) < 0.3)
        low[lb] = 1
        cost = rng.integers(0, cost_hi, m)
        cap[feas] = 200
        low[feas] = 0
        cost[feas] = 50 * cost_hi
        supply = np.zeros(n, np.int64)
        supply[ends[:k] - 1] += units
        supply[ends[k:] - 1] -= units
        ntype = np.zeros(n, np.int32)
        yield trial, gen.Graph(ntype, supply, src, dst, low, cap.astype(np.int64), cost.astype(np.int64))
