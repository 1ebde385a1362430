"""Config 4: a Quincy cell under churn, emitted as ksched's incremental change stream.

``Cell`` holds the scheduling state of one Quincy-shaped cell (``gen.quincy``)
and turns each scheduling round into the delta records that the reference's
graph manager would log between two ``Solve`` calls
(flowmanager/graph_change_manager.go:93-206 → dimacs.ExportIncremental,
placement/solver.go:118-123), in mutation order:

1. **Pin** every task the last solve placed (graph_manager.go:690-735
   ``pinTaskToNode``): each of its out-arcs is deleted (``DeleteArc`` emits
   ``x src dst 0 0 cost type cost``, graph_change_manager.go:184-193), a
   running arc task→PU with low=1, cap=1, cost 0 is added, and the job's
   unscheduled aggregator loses one unit of capacity
   (``updateUnscheduledAggNode(-1)``).
2. **Complete** up to ``done`` running tasks (``r id``; the reference emits
   only the node removal, graph_change_manager.go:129-139).
3. **Arrive** ``arrive`` new tasks, reusing freed node ids first-in first-out
   (graph.go:169-182): ``n id 1 1`` plus the five preference arcs of the
   Quincy shape, and +1 on the job's U_j→sink arc.
4. **Age** every task that was already waiting: +``age_cost`` on its →U_j arc
   (``UpdateAllCostsToUnscheduledAggs``, graph_manager.go:462-475, is called
   inside ``Solve`` before the incremental export, solver.go:86).
5. **Capacities** of the resource arcs (X→rack, rack→machine, machine→PU:
   free slots = slots − running, ``capacityFromResNodeToParent``
   graph_manager.go:487-492 with Preemption=false) and of U_j→sink, one
   ``x`` record per changed arc.

The sink's demand is left to the solver (``ks_opts.auto_sink``), exactly the
drift of graph_manager.go:640, 808. Random draws come from the same splitmix64
counter stream as the generator (seed = 4 + round in SURVEY §8d).
"""
from __future__ import annotations

from collections import deque

import numpy as np

from . import gen

KS_ADD_NODE, KS_REMOVE_NODE, KS_ADD_ARC, KS_UPDATE_ARC = 0, 1, 2, 3
RUNNING = 1

DELTA_DT = np.dtype({"names": ["kind", "type", "id", "src", "dst", "low", "cap", "cost", "old_cost", "excess"],
                     "formats": ["<i4", "<i4", "<u8", "<u8", "<u8", "<u8", "<u8", "<i8", "<i8", "<i8"],
                     "offsets": [0, 4, 8, 16, 24, 32, 40, 48, 56, 64], "itemsize": 72})


class Cell:
    """Scheduling state of one Quincy cell; ``graph()`` is the equivalent full graph."""

    WAIT, RUN, DEAD = 0, 1, 2

    def __init__(self, T: int, M: int, R: int, J: int, seed: int):
        self.T0, self.M, self.R, self.J = T, M, R, J
        self.SINK, self.X, self.RACK0 = 1, 2, 3
        self.MACH0 = self.RACK0 + R
        self.PU0 = self.MACH0 + M
        self.U0 = self.PU0 + M
        self.TASK0 = self.U0 + J
        g = gen.quincy(T, M, R, J, seed)
        self.slots = g.cap[5 * T + R:5 * T + R + M].copy()          # rack→machine caps at creation
        k = np.arange(M, dtype=np.int64)
        self.rack_of = k % R
        cap = T + 1
        self.state = np.full(cap, self.DEAD, np.int8)                # index = task slot (id − TASK0)
        self.state[:T] = self.WAIT
        self.job = np.zeros(cap, np.int64)
        self.adst = np.zeros((cap, 5), np.int64)                     # preference arcs of a waiting task
        self.acost = np.zeros((cap, 5), np.int64)
        self.pu = np.zeros(cap, np.int64)                            # PU node id of a running task
        self.job[:T] = g.dst[0:5 * T:5] - self.U0
        self.adst[:T] = g.dst[:5 * T].reshape(T, 5)
        self.acost[:T] = g.cost[:5 * T].reshape(T, 5)
        self.running_on = np.zeros(M, np.int64)
        self.free_ids: deque[int] = deque()
        self.n_slots = T
        self.round = 0
        self.initial = g
        self.last_arrived_ids: list[int] = []   # task ids (re)created by the last step

    # ----------------------------------------------------------------- views
    def _grow(self, need: int):
        cap = self.state.shape[0]
        if need <= cap:
            return
        new = max(need, 2 * cap)
        for name in ("state", "job", "pu"):
            a = getattr(self, name)
            b = np.zeros(new, a.dtype) if name != "state" else np.full(new, self.DEAD, np.int8)
            b[:cap] = a
            setattr(self, name, b)
        for name in ("adst", "acost"):
            a = getattr(self, name)
            b = np.zeros((new, 5), np.int64)
            b[:cap] = a
            setattr(self, name, b)

    def waiting_per_job(self) -> np.ndarray:
        s = self.state[:self.n_slots]
        return np.bincount(self.job[:self.n_slots][s == self.WAIT], minlength=self.J).astype(np.int64)

    def resource_caps(self):
        run = self.running_on
        rack_free = np.bincount(self.rack_of, weights=self.slots - run, minlength=self.R).astype(np.int64)
        return rack_free, self.slots - run, self.slots - run           # X→rack, rack→machine, machine→PU

    def graph(self) -> gen.Graph:
        """The full graph equivalent to the initial graph plus every delta so far."""
        M, R, J = self.M, self.R, self.J
        ns = self.n_slots
        n = self.TASK0 - 1 + ns
        ntype = np.zeros(n, np.int32)
        supply = np.zeros(n, np.int64)
        ntype[self.SINK - 1] = 3
        ntype[self.MACH0 - 1:self.MACH0 - 1 + M] = 4
        ntype[self.PU0 - 1:self.PU0 - 1 + M] = 2
        st = self.state[:ns]
        tid = self.TASK0 + np.arange(ns, dtype=np.int64)
        alive = st != self.DEAD
        ntype[tid[alive] - 1] = 1
        supply[tid[alive] - 1] = 1
        supply[self.SINK - 1] = -int(alive.sum())
        w = st == self.WAIT
        r = st == self.RUN
        tw = tid[w]
        k = np.arange(M, dtype=np.int64)
        jj = np.arange(J, dtype=np.int64)
        rack_free, rm, mp = self.resource_caps()
        src = np.concatenate([np.repeat(tw, 5), tid[r], np.full(R, self.X, np.int64), self.RACK0 + self.rack_of,
                              self.MACH0 + k, self.PU0 + k, self.U0 + jj])
        dst = np.concatenate([self.adst[:ns][w].reshape(-1), self.pu[:ns][r], self.RACK0 + np.arange(R),
                              self.MACH0 + k, self.PU0 + k, np.full(M, self.SINK, np.int64),
                              np.full(J, self.SINK, np.int64)])
        nr = int(r.sum())
        low = np.concatenate([np.zeros(5 * tw.shape[0], np.int64), np.ones(nr, np.int64),
                              np.zeros(R + 3 * M + J, np.int64)])
        cap = np.concatenate([np.ones(5 * tw.shape[0] + nr, np.int64), rack_free, rm, mp, self.slots,
                              self.waiting_per_job()])
        cost = np.concatenate([self.acost[:ns][w].reshape(-1), np.zeros(nr + R + 3 * M + J, np.int64)])
        atype = np.zeros(src.shape[0], np.int32)
        atype[5 * tw.shape[0]:5 * tw.shape[0] + nr] = RUNNING
        return gen.Graph(ntype, supply, src, dst, low, cap, cost, atype)

    def task_ids(self, which: int) -> np.ndarray:
        return self.TASK0 + np.nonzero(self.state[:self.n_slots] == which)[0].astype(np.int64)

    # ---------------------------------------------------------------- rounds
    def step(self, mapping, done: int, arrive: int, age_cost: int = 10,
             seed: int | None = None) -> np.ndarray:
        """Advance one scheduling round given the last solve's task→PU mapping (a
        dict, or the (task ids, PU ids) arrays of ks_get_task_mapping);
        returns the delta records (``DELTA_DT``) in mutation order."""
        self.round += 1
        seed = 4 + self.round if seed is None else seed
        out = []
        M = self.M
        waiting_before = self.state[:self.n_slots] == self.WAIT
        old_rm = self.resource_caps()
        old_u = self.waiting_per_job()

        # 1. pin the tasks the solver placed
        if isinstance(mapping, tuple):   # (task ids, PU ids) arrays, as the C-ABI returns them
            mapping = (np.asarray(mapping[0], np.int64), np.asarray(mapping[1], np.int64))
        if isinstance(mapping, tuple) and mapping[0].shape[0]:
            t, p = mapping
        elif isinstance(mapping, dict) and mapping:
            t = np.fromiter(mapping.keys(), np.int64, len(mapping))
            p = np.fromiter(mapping.values(), np.int64, len(mapping))
        else:
            t = None
        if t is not None:
            order = np.argsort(t, kind="stable")
            t, p = t[order], p[order]
            sl = t - self.TASK0
            keep = (sl >= 0) & (sl < self.n_slots)
            t, p, sl = t[keep], p[keep], sl[keep]
            keep = self.state[sl] == self.WAIT
            t, p, sl = t[keep], p[keep], sl[keep]
            if np.any((p < self.PU0) | (p >= self.PU0 + M)):
                raise ValueError("mapping names a non-PU node")
            for ti, pi, si in zip(t.tolist(), p.tolist(), sl.tolist()):
                for d, c in zip(self.adst[si].tolist(), self.acost[si].tolist()):
                    out.append((KS_UPDATE_ARC, 0, 0, ti, d, 0, 0, c, c, 0))
                out.append((KS_ADD_ARC, RUNNING, 0, ti, pi, 1, 1, 0, 0, 0))
            self.state[sl] = self.RUN
            self.pu[sl] = p
            np.add.at(self.running_on, p - self.PU0, 1)

        # 2. completions (running tasks, drawn by the round's stream)
        run = self.task_ids(self.RUN)
        k = min(done, run.shape[0])
        if k:
            pick = run[np.argsort(gen.stream(seed, 0, run.shape[0]), kind="stable")[:k]]
            pick.sort()
            for ti in pick.tolist():
                out.append((KS_REMOVE_NODE, 0, ti, 0, 0, 0, 0, 0, 0, 0))
                self.free_ids.append(ti)
            sl = pick - self.TASK0
            np.add.at(self.running_on, self.pu[sl] - self.PU0, -1)
            self.state[sl] = self.DEAD

        # 3. arrivals (FIFO id reuse, then fresh ids)
        arrived = []
        self.last_arrived_ids = []
        if arrive:
            x = gen.stream(seed, 1 << 32, 9 * arrive).reshape(arrive, 9)
            J, R = self.J, self.R
            j = (x[:, 0] % np.uint64(J)).astype(np.int64)
            cU = gen._u(200, 1000, x[:, 1])
            cX = gen._u(100, 400, x[:, 2])
            rk = (x[:, 3] % np.uint64(R)).astype(np.int64)
            cR = gen._u(20, 200, x[:, 4])
            m1 = (x[:, 5] % np.uint64(M)).astype(np.int64)
            m2 = (m1 + 1 + (x[:, 6] % np.uint64(M - 1)).astype(np.int64)) % M
            c1 = gen._u(0, 100, x[:, 7])
            c2 = gen._u(0, 100, x[:, 8])
            dsts = np.stack([self.U0 + j, np.full(arrive, self.X, np.int64), self.RACK0 + rk, self.MACH0 + m1,
                             self.MACH0 + m2], 1)
            costs = np.stack([cU, cX, cR, c1, c2], 1)
            for a in range(arrive):
                if self.free_ids:
                    ti = self.free_ids.popleft()
                else:
                    ti = self.TASK0 + self.n_slots
                    self._grow(self.n_slots + 1)
                    self.n_slots += 1
                si = ti - self.TASK0
                arrived.append(si)
                self.state[si] = self.WAIT
                self.job[si] = j[a]
                self.adst[si] = dsts[a]
                self.acost[si] = costs[a]
                self.last_arrived_ids.append(ti)
                out.append((KS_ADD_NODE, 1, ti, 0, 0, 0, 0, 0, 0, 1))
                for d, c in zip(dsts[a].tolist(), costs[a].tolist()):
                    out.append((KS_ADD_ARC, 0, 0, ti, d, 0, 1, c, 0, 0))

        # 4. ageing of the tasks that were already waiting (not an arrival that took
        #    over the id of a task that completed this round)
        if age_cost:
            ns0 = waiting_before.shape[0]
            still = waiting_before & (self.state[:ns0] == self.WAIT)
            fresh = np.asarray([a for a in arrived if a < ns0], np.int64)
            still[fresh] = False
            aged = np.nonzero(still)[0]
            for si in aged.tolist():
                c = int(self.acost[si, 0])
                ti = self.TASK0 + si
                out.append((KS_UPDATE_ARC, 0, 0, ti, int(self.adst[si, 0]), 0, 1, c + age_cost, c, 0))
            self.acost[aged, 0] += age_cost

        # 5. capacity refresh of resource and unscheduled-aggregator arcs
        new_rm = self.resource_caps()
        k = np.arange(M, dtype=np.int64)
        fams = ((np.full(self.R, self.X, np.int64), self.RACK0 + np.arange(self.R)),
                (self.RACK0 + self.rack_of, self.MACH0 + k), (self.MACH0 + k, self.PU0 + k))
        for (s, d), old, new in zip(fams, old_rm, new_rm):
            for i in np.nonzero(old != new)[0].tolist():
                out.append((KS_UPDATE_ARC, 0, 0, int(s[i]), int(d[i]), 0, int(new[i]), 0, 0, 0))
        new_u = self.waiting_per_job()
        for i in np.nonzero(old_u != new_u)[0].tolist():
            out.append((KS_UPDATE_ARC, 0, 0, self.U0 + i, self.SINK, 0, int(new_u[i]), 0, 0, 0))

        arr = np.zeros(len(out), DELTA_DT)
        if out:
            cols = list(zip(*out))
            for name, col in zip(DELTA_DT.names, cols):
                arr[name] = np.asarray(col, dtype=DELTA_DT[name])
        return arr
