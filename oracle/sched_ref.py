"""CPU restatements of the scheduler-side sweeps that libksmcmf runs on device
(ksched_amd/csrc/ks_sched.hip). TEST INFRASTRUCTURE ONLY — the checker, never
imported by the product. Paths relative to the ksched tree.
"""
from __future__ import annotations

from collections import deque

import numpy as np

PLACE, PREEMPT, MIGRATE = 0, 1, 2     # pb.SchedulingDelta_ChangeType (proto/scheduling_delta.proto:11-16)


def scheduling_deltas(bindings: dict[int, int], mapping: dict[int, int], live_tasks) -> list[tuple[int, int, int]]:
    """SchedulingDeltasForPreemptedTasks (flowmanager/graph_manager.go:297-339):
    a bound, still-live task absent from the mapping is preempted; then
    NodeBindingToSchedulingDelta (:253-295) per mapping entry: unbound → PLACE,
    bound elsewhere → MIGRATE, bound here → nothing. The reference iterates Go
    maps; this restatement (and the device) orders each group by task id."""
    live = set(int(t) for t in live_tasks)
    out = [(PREEMPT, t, p) for t, p in sorted(bindings.items()) if p and t in live and t not in mapping]
    for t, p in sorted(mapping.items()):
        b = bindings.get(t, 0)
        if not b:
            out.append((PLACE, t, p))
        elif b != p:
            out.append((MIGRATE, t, p))
    return out


def apply_deltas(bindings: dict[int, int], deltas) -> dict[int, int]:
    """applySchedulingDeltas (flowscheduler/scheduler.go:377-412) on the bindings."""
    b = dict(bindings)
    for kind, t, p in deltas:
        if kind == PREEMPT:
            b.pop(t, None)
        else:
            b[t] = p
    return b


def topology_stats(g, resource: set[int], pu_running: dict[int, int], mtpp: int):
    """ComputeTopologyStatistics (flowmanager/graph_manager.go:480-511) with the
    trivial model's PrepareStats / GatherStats (costmodel/trivial_cost_modeler.go:147-176):
    FIFO BFS from the sink over in-arcs. Returns {resource id: (slots, running)}."""
    inc: dict[int, list[int]] = {}
    for s, d in zip(g.src.tolist(), g.dst.tolist()):
        inc.setdefault(int(d), []).append(int(s))
    sink = int(np.nonzero(g.ntype == 3)[0][0]) + 1
    slots = {v: 0 for v in resource}
    run = {v: 0 for v in resource}
    seen = {sink}
    q = deque([sink])
    while q:
        cur = q.popleft()
        for src in inc.get(cur, []):
            if src not in seen:
                seen.add(src)
                if src in resource:
                    slots[src] = run[src] = 0          # PrepareStats
                q.append(src)
            if src not in resource:                    # GatherStats: accumulator must be a resource
                continue
            if cur not in resource:
                if g.ntype[cur - 1] == 3:              # from the sink: a PU's own counts
                    run[src] = pu_running.get(src, 0)
                    slots[src] = mtpp
                continue
            run[src] += run[cur]
            slots[src] += slots[cur]
    return {v: (slots[v], run[v]) for v in resource}
