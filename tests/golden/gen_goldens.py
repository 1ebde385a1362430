"""Generate the committed golden fixtures (run in the build container only).

    python tests/golden/gen_goldens.py [--big]

Each golden is ``(family, params, seed) → (n, m, cost, flow)`` where cost/flow
come from ``networkx.network_simplex`` (exact on integer data; networkx 3.4.2
in the build container). networkx never travels to the GPU box: there the
graphs are regenerated from (params, seed) and checked against these numbers.

``--big`` also solves the config-3 graph (100k tasks × 10k machines, ≈15 min).
``--batch64`` adds all 64 config-5 cells (config-2 graphs, seeds 1000..1063),
solved in parallel worker processes (≈9 s each).
"""
from __future__ import annotations

import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

import networkx as nx

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from ksched_amd import gen  # noqa: E402

OUT = os.path.join(os.path.dirname(__file__), "goldens.json")


def nx_solve(g):
    G = nx.DiGraph()
    for v in range(g.n):
        G.add_node(v + 1, demand=int(-g.supply[v]))
    const = 0
    for s, d, lo, ca, co in zip(g.src.tolist(), g.dst.tolist(), g.low.tolist(), g.cap.tolist(),
                                g.cost.tolist()):
        if lo:  # lower-bound transform
            G.nodes[s]["demand"] += lo
            G.nodes[d]["demand"] -= lo
            const += lo * co
        G.add_edge(s, d, capacity=ca - lo, weight=co)
    cost, _ = nx.network_simplex(G)
    flow = int(sum(max(int(x), 0) for x in g.supply.tolist()))
    return int(cost) + const, flow


def solve_case(case):
    fam, params, seed = case
    g = gen.trivial(*params) if fam == "trivial" else gen.quincy(*params, seed)
    t0 = time.time()
    cost, flow = nx_solve(g)
    dt = time.time() - t0
    print(f"{fam} {params} seed={seed}: n={g.n} m={g.m} cost={cost} flow={flow} ({dt:.1f}s)", flush=True)
    return {"family": fam, "params": list(params), "seed": seed, "n": g.n, "m": g.m,
            "cost": cost, "flow": flow, "solver": f"networkx {nx.__version__} network_simplex"}


def main():
    big = "--big" in sys.argv
    cases = []
    # config 1 (ksched trivial topology)
    cases.append(("trivial", (10, 1000, 100), 0))
    cases.append(("trivial", (2, 1, 3), 0))
    cases.append(("trivial", (3, 2, 10), 0))     # overloaded: 6 slots for 10 pods
    # small Quincy graphs: normal, overloaded, underloaded
    for seed in range(1, 6):
        cases.append(("quincy", (1000, 100, 5, 10), seed))
    cases.append(("quincy", (100, 10, 2, 3), 7))
    cases.append(("quincy", (2000, 100, 5, 20), 8))    # ~200 % load
    cases.append(("quincy", (500, 100, 10, 7), 9))     # ~50 % load
    cases.append(("quincy", (3000, 300, 12, 30), 10))
    # config 2 and a slice of config 5's seeds
    cases.append(("quincy", gen.CONFIGS["config2"][:4], gen.CONFIGS["config2"][4]))
    for seed in range(1000, 1004):
        cases.append(("quincy", gen.CONFIGS["config2"][:4], seed))
    if big:
        cases.append(("quincy", gen.CONFIGS["config3"][:4], gen.CONFIGS["config3"][4]))
    if "--batch64" in sys.argv:      # config 5: 64 config-2 cells, seeds 1000..1063
        for seed in range(1004, 1064):
            cases.append(("quincy", gen.CONFIGS["config2"][:4], seed))

    old = {}
    if os.path.exists(OUT):
        for e in json.load(open(OUT))["graphs"]:
            old[(e["family"], tuple(e["params"]), e["seed"])] = e
    todo = [c for c in cases if (c[0], tuple(c[1]), c[2]) not in old]
    workers = int(os.environ.get("GOLDEN_WORKERS", "6"))
    with ProcessPoolExecutor(max(1, workers)) as ex:
        fresh = dict(zip(todo, ex.map(solve_case, todo)))
    res = []
    for fam, params, seed in cases:
        key = (fam, tuple(params), seed)
        res.append(old[key] if key in old else fresh[(fam, params, seed)])
    for k, e in old.items():
        if all((r["family"], tuple(r["params"]), r["seed"]) != k for r in res):
            res.append(e)
    json.dump({"generator": "ksched_amd.gen (splitmix64 counter stream, SURVEY §8d)", "graphs": res},
              open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
