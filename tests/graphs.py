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
