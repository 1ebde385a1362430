"""Synthetic scheduling flow graphs (numpy, vectorised).

Two families, both emitted as ksched-shaped node/arc arrays with 1-based NodeIDs
(flowgraph/graph.go:169-182 allocates ids densely from 1):

* ``quincy(T, M, R, J, seed)`` — the Quincy-shaped cell graph of SURVEY §8(d):
  tasks → {unscheduled aggregator U_j, cluster aggregator X, one rack, two
  machines}; X → racks → machines → PUs → sink; U_j → sink. Costs are drawn from
  a splitmix64 counter stream x_i = mix(seed + (i+1)·0x9E3779B97F4A7C15) so the
  C oracle (oracle/ks_oracle.c: ko_gen_quincy) produces bit-identical arrays.
* ``trivial(machines, mt, pods)`` — ksched's own topology for config 1
  (cmd/k8sscheduler/scheduler.go:191-202, 332-350 fake machines with one PU
  each; arc families of flowmanager/graph_manager.go:1116-1305 and the trivial
  cost model, costmodel/trivial_cost_modeler.go:41-110).

Arrays: ``ntype`` (DIMACS type codes, dimacs/export.go:56-68), ``supply``
(node excess), ``src``/``dst``/``low``/``cap``/``cost`` per arc.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# SURVEY §8(d) configurations (T, M, R, J, seed)
CONFIGS = {
    "config2": (10_000, 1_000, 25, 100, 2),
    "config3": (100_000, 10_000, 250, 1_000, 3),
}


@dataclass
class Graph:
    ntype: np.ndarray   # int32 [n]
    supply: np.ndarray  # int64 [n]
    src: np.ndarray     # int64 [m] 1-based
    dst: np.ndarray     # int64 [m]
    low: np.ndarray     # int64 [m]
    cap: np.ndarray     # int64 [m]
    cost: np.ndarray    # int64 [m]
    atype: np.ndarray | None = None  # int32 [m] flowgraph.ArcType (0 other, 1 running)

    @property
    def n(self) -> int:
        return int(self.ntype.shape[0])

    @property
    def m(self) -> int:
        return int(self.src.shape[0])

    def arc_types(self) -> np.ndarray:
        return self.atype if self.atype is not None else np.zeros(self.m, np.int32)


def _mix(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def stream(seed: int, start: int, count: int) -> np.ndarray:
    """x_i for i in [start, start+count)."""
    i = np.arange(start, start + count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i + np.uint64(1)) * _GAMMA
    return _mix(z)


def _u(a: int, b: int, x: np.ndarray) -> np.ndarray:
    return (np.int64(a) + (x % np.uint64(b - a + 1)).astype(np.int64))


def quincy_sizes(T: int, M: int, R: int, J: int) -> tuple[int, int]:
    return T + J + R + 2 * M + 2, 5 * T + R + 3 * M + J


def quincy(T: int, M: int, R: int, J: int, seed: int) -> Graph:
    if T < 1 or M < 2 or R < 1 or J < 1 or R > M:
        raise ValueError("quincy: need T>=1, M>=2, 1<=R<=M, J>=1")
    SINK, X, RACK0 = 1, 2, 3
    MACH0 = RACK0 + R
    PU0 = MACH0 + M
    U0 = PU0 + M
    TASK0 = U0 + J
    n, m = quincy_sizes(T, M, R, J)

    ntype = np.zeros(n, np.int32)
    supply = np.zeros(n, np.int64)
    ntype[SINK - 1] = 3
    ntype[MACH0 - 1:MACH0 - 1 + M] = 4
    ntype[PU0 - 1:PU0 - 1 + M] = 2
    ntype[TASK0 - 1:TASK0 - 1 + T] = 1
    supply[TASK0 - 1:TASK0 - 1 + T] = 1
    supply[SINK - 1] = -T

    slots = _u(8, 12, stream(seed, 0, M))
    k = np.arange(M, dtype=np.int64)
    rackslots = np.bincount(k % R, weights=slots, minlength=R).astype(np.int64)

    x = stream(seed, M, 9 * T).reshape(T, 9)
    j = (x[:, 0] % np.uint64(J)).astype(np.int64)
    cU = _u(200, 1000, x[:, 1])
    cX = _u(100, 400, x[:, 2])
    rk = (x[:, 3] % np.uint64(R)).astype(np.int64)
    cR = _u(20, 200, x[:, 4])
    m1 = (x[:, 5] % np.uint64(M)).astype(np.int64)
    m2 = (m1 + 1 + (x[:, 6] % np.uint64(M - 1)).astype(np.int64)) % M
    c1 = _u(0, 100, x[:, 7])
    c2 = _u(0, 100, x[:, 8])
    jobtasks = np.bincount(j, minlength=J).astype(np.int64)

    tid = TASK0 + np.arange(T, dtype=np.int64)
    t_src = np.repeat(tid, 5)
    t_dst = np.stack([U0 + j, np.full(T, X, np.int64), RACK0 + rk, MACH0 + m1, MACH0 + m2], 1).reshape(-1)
    t_cost = np.stack([cU, cX, cR, c1, c2], 1).reshape(-1)

    r = np.arange(R, dtype=np.int64)
    jj = np.arange(J, dtype=np.int64)
    src = np.concatenate([t_src, np.full(R, X, np.int64), RACK0 + (k % R), MACH0 + k, PU0 + k, U0 + jj])
    dst = np.concatenate([t_dst, RACK0 + r, MACH0 + k, PU0 + k, np.full(M, SINK, np.int64),
                          np.full(J, SINK, np.int64)])
    cap = np.concatenate([np.ones(5 * T, np.int64), rackslots, slots, slots, slots, jobtasks])
    cost = np.concatenate([t_cost, np.zeros(R + 3 * M + J, np.int64)])
    low = np.zeros(m, np.int64)
    assert src.shape[0] == m
    return Graph(ntype, supply, src, dst, low, cap, cost)


def trivial_sizes(machines: int, pods: int) -> tuple[int, int]:
    return 2 + 2 * machines + 2 + pods, 4 * machines + 2 * pods + 1


def trivial(machines: int = 10, mt: int = 1000, pods: int = 100) -> Graph:
    """ksched config 1: ``k8sscheduler -fakeMachines -nm machines -mt mt`` + pods in one job."""
    n, m = trivial_sizes(machines, pods)
    SINK, COORD = 1, 2
    U = 3 + 2 * machines
    EC = U + 1
    TASK0 = EC + 1
    ntype = np.zeros(n, np.int32)
    supply = np.zeros(n, np.int64)
    ntype[SINK - 1] = 3
    supply[SINK - 1] = -pods
    src, dst, cap, cost = [], [], [], []

    def arc(s, d, c, co):
        src.append(s); dst.append(d); cap.append(c); cost.append(co)

    for k in range(machines):
        mach, pu = 3 + 2 * k, 4 + 2 * k
        ntype[mach - 1] = 4
        ntype[pu - 1] = 2
        arc(pu, SINK, mt, 0)          # graph_manager.go:1116-1129
        arc(mach, pu, mt, 0)          # :624
        arc(COORD, mach, 0, 0)        # :624 (NumSlotsBelow 0 at creation)
    arc(U, SINK, pods, 0)             # :1291-1305
    for t in range(pods):
        tid = TASK0 + t
        ntype[tid - 1] = 1
        supply[tid - 1] = 1
        arc(tid, U, 1, 5)             # trivial_cost_modeler.go:41-43
        arc(tid, EC, 1, 2)            # :69-74
    for k in range(machines):
        arc(EC, 3 + 2 * k, mt, 0)     # :76-83 (free slots)
    a = lambda v: np.asarray(v, np.int64)
    g = Graph(ntype, supply, a(src), a(dst), np.zeros(m, np.int64), a(cap), a(cost))
    assert g.m == m
    return g
