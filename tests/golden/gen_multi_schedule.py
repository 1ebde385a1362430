"""Fixture generator: the five rounds of ksched's TestMultiScheduleIteration as
the exact DIMACS wire stream the reference sends to its solver.

    python tests/golden/gen_multi_schedule.py      # writes multi_schedule_iteration.json

TEST INFRASTRUCTURE (build container only). The reference cannot run here (Go,
no toolchain; its solver Flowlessly is not vendored), so this script restates
the parts of the reference that produce the solver's input for this one test,
line by line in behaviour (paths relative to the ksched tree):

* the test's event sequence  scheduling/flow/flowscheduler/schedule_iteration_test.go:16-91
  (2 machines × 1 core × 1 PU, maxTasksPerPu 1; jobs of 1, 1, 1 tasks; round 2
  adds a job of 2 tasks; before round 3 the 2 running tasks complete)
* scheduler rounds           flowscheduler/scheduler.go:309-375 (ScheduleAllJobs,
                             runSchedulingIteration), :377-412 (applySchedulingDeltas),
                             :106-132 (HandleTaskCompletion), :414-416, :421-437, :493-529
* graph manager              flowmanager/graph_manager.go:161-208 (AddOrUpdateJobNodes),
                             :297-339 (SchedulingDeltasForPreemptedTasks), :253-295,
                             :389-405 (TaskCompleted), :454-475, :480-511
                             (ComputeTopologyStatistics), :557-648, :662-720 (pinning),
                             :803-813, :895-1305 (updateFlowGraph and helpers)
* change log                 flowmanager/graph_change_manager.go:93-206
* graph store / ids          flowgraph/graph.go:60-182 (FIFO id reuse)
* trivial cost model         costmodel/trivial_cost_modeler.go:41-176
* wire format                dimacs/export.go:11-76, dimacs/*_change.go GenerateChange
* solver protocol            placement/solver.go:60-123 (first Solve: full export;
                             later: UpdateAllCostsToUnscheduledAggs + incremental)

Go map iteration order is random in the reference; this restatement iterates in
insertion order, which is one of the orders the reference can take. The solve
of each round uses the C oracle's successive shortest path and the reference's
own BFS decomposition (oracle/ko.bfs_mapping, a restatement of solver.go:183-269)
to pick the placements that drive the next round's pins; the fixture records
those placements so a replay is deterministic.
"""
from __future__ import annotations

import json
import os
import sys
from collections import OrderedDict, deque

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
from ksched_amd import gen  # noqa: E402
from oracle import ko  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "multi_schedule_iteration.json")

# flowgraph.NodeType (node.go:25-41)
ROOT_TASK, SCHED_TASK, UNSCHED_TASK, JOB_AGG, SINK, EQUIV, COORD, MACHINE, NUMA, SOCKET, CACHE, CORE, PU = range(13)
ARC_OTHER, ARC_RUNNING = 0, 1
CLUSTER_AGG_EC = 0x7A  # any fixed id: the trivial model has one EC (ClusterAggregatorEC)
# TaskDescriptor states used here
CREATED, RUNNABLE, RUNNING, COMPLETED = "Created", "Runnable", "Running", "Completed"


def dimacs_type(t):  # dimacs/add_node_change.go:64-78
    return {PU: 2, MACHINE: 4, SINK: 3, NUMA: 5, SOCKET: 5, CACHE: 5, CORE: 5,
            UNSCHED_TASK: 1, SCHED_TASK: 1, ROOT_TASK: 1}.get(t, 0)


class Node:
    def __init__(self, nid):
        self.id, self.type, self.excess = nid, None, 0
        self.out: OrderedDict[int, Arc] = OrderedDict()
        self.inc: OrderedDict[int, Arc] = OrderedDict()
        self.task = self.job = self.rd = self.ec = None
        self.visited = 0


class Arc:
    def __init__(self, s, d):
        self.src, self.dst = s, d
        self.low = self.cap = self.cost = 0
        self.type = ARC_OTHER


class Graph:                                    # flowgraph/graph.go
    def __init__(self):
        self.nodes: OrderedDict[int, Node] = OrderedDict()
        self.arcs: OrderedDict[tuple, Arc] = OrderedDict()
        self.next_id, self.unused = 1, deque()

    def add_node(self):
        nid = self.unused.popleft() if self.unused else self.next_id
        if nid == self.next_id:
            self.next_id += 1
        n = Node(nid)
        self.nodes[nid] = n
        return n

    def add_arc(self, s: Node, d: Node):
        a = Arc(s, d)
        assert d.id not in s.out and s.id not in d.inc
        s.out[d.id] = a
        d.inc[s.id] = a
        self.arcs[(s.id, d.id)] = a
        return a

    def delete_arc(self, a: Arc):
        a.src.out.pop(a.dst.id, None)
        a.dst.inc.pop(a.src.id, None)
        self.arcs.pop((a.src.id, a.dst.id), None)

    def delete_node(self, n: Node):
        self.unused.append(n.id)
        for a in list(n.out.values()):
            self.delete_arc(a)
        for a in list(n.inc.values()):
            self.delete_arc(a)
        del self.nodes[n.id]


class ChangeManager:                           # flowmanager/graph_change_manager.go:93-206
    def __init__(self):
        self.g = Graph()
        self.changes: list[str] = []

    def add_arc(self, s, d, low, cap, cost, typ):
        a = self.g.add_arc(s, d)
        a.low, a.cap, a.cost, a.type = low, cap, cost, typ
        self.changes.append(f"a {s.id} {d.id} {low} {cap} {cost} {typ}")
        return a

    def add_node(self, typ, excess):
        n = self.g.add_node()
        n.type, n.excess = typ, excess
        self.changes.append(f"n {n.id} {excess} {dimacs_type(typ)}")
        return n

    def delete_node(self, n):
        self.changes.append(f"r {n.id}")
        self.g.delete_node(n)

    def change_arc(self, a, low, cap, cost):
        old = a.cost
        if (a.low, a.cap, old) == (low, cap, cost):
            return
        a.low, a.cap, a.cost = low, cap, cost
        self.changes.append(f"x {a.src.id} {a.dst.id} {low} {cap} {cost} {a.type} {old}")

    def change_arc_capacity(self, a, cap):
        if a.cap == cap:
            return
        a.cap = cap
        self.changes.append(f"x {a.src.id} {a.dst.id} {a.low} {cap} {a.cost} {a.type} {a.cost}")

    def change_arc_cost(self, a, cost):
        old = a.cost
        if old == cost:
            return
        a.cost = cost
        self.changes.append(f"x {a.src.id} {a.dst.id} {a.low} {a.cap} {cost} {a.type} {old}")

    def delete_arc(self, a):
        a.cap = a.low = 0
        self.changes.append(f"x {a.src.id} {a.dst.id} 0 0 {a.cost} {a.type} {a.cost}")
        self.g.delete_arc(a)


class RD:                                       # pb.ResourceDescriptor (fields used)
    def __init__(self, uuid, typ, children=()):
        self.uuid, self.type, self.children = uuid, typ, list(children)
        self.parent = None
        self.slots = self.running = 0
        self.current_running: list[int] = []
        for c in self.children:
            c.parent = self


class Task:
    def __init__(self, uid, job):
        self.uid, self.job, self.state = uid, job, CREATED
        self.spawned: list[Task] = []


class GraphManager:                             # flowmanager/graph_manager.go
    def __init__(self, max_tasks_per_pu):
        self.cm = ChangeManager()
        self.sink = self.cm.add_node(SINK, 0)
        self.mtpp = max_tasks_per_pu
        self.res_node: dict[int, Node] = {}
        self.task_node: dict[int, Node] = {}
        self.ec_node: dict[int, Node] = {}
        self.job_unsched: dict[int, Node] = {}
        self.running_arc: dict[int, Arc] = {}
        self.parent: dict[int, Node] = {}
        self.leaf_ids: dict[int, None] = {}
        self.machines: OrderedDict[int, RD] = OrderedDict()   # trivial model machineToResTopo
        self.counter = 0

    # -- resources (:238-251, :557-630, :1116-1129)
    def add_resource_topology(self, rd: RD):
        self._add_dfs(rd)
        if rd.parent is not None:
            self._stats_up(self.res_node[rd.parent.uuid], rd.slots - rd.running, rd.slots, rd.running)

    def _add_dfs(self, rd: RD):
        node = self.res_node.get(rd.uuid)
        added = node is None
        if added:
            node = self.cm.add_node(rd.type, 0)
            node.rd = rd
            self.res_node[rd.uuid] = node
            if node.type == PU:
                self.leaf_ids[node.id] = None
                self._res_to_sink(node)
                if rd.slots == 0:
                    rd.slots = self.mtpp
                    if rd.running == 0:
                        rd.running = len(rd.current_running)
            else:
                if node.type == MACHINE:
                    self.machines.setdefault(rd.uuid, rd)
                rd.slots = rd.running = 0
        else:
            rd.slots = rd.running = 0
        for c in rd.children:
            self._add_dfs(c)
            rd.slots += c.slots
            rd.running += c.running
        if rd.parent is None:
            assert rd.type == COORD
            return
        if added:
            p = self.res_node[rd.parent.uuid]
            self.parent[node.id] = p
            self.cm.add_arc(p, node, 0, rd.slots - rd.running, 0, ARC_OTHER)

    def _stats_up(self, cur: Node, cap_d, slots_d, run_d):
        while True:
            p = self.parent.get(cur.id)
            if p is None:
                return
            a = p.out[cur.id]
            self.cm.change_arc_capacity(a, a.cap + cap_d)
            p.rd.slots += slots_d
            p.rd.running += run_d
            cur = p

    def _res_to_sink(self, node):
        a = node.out.get(self.sink.id)
        if a is None:
            self.cm.add_arc(node, self.sink, 0, self.mtpp, 0, ARC_OTHER)
        else:
            self.cm.change_arc_cost(a, 0)

    # -- statistics (:480-511 with trivial PrepareStats/GatherStats :147-176)
    def compute_topology_statistics(self):
        self.counter += 1
        q = deque([self.sink])
        self.sink.visited = self.counter
        while q:
            cur = q.popleft()
            for a in list(cur.inc.values()):
                src = a.src
                if src.visited != self.counter:
                    if src.rd is not None:
                        src.rd.slots = src.rd.running = 0
                    q.append(src)
                    src.visited = self.counter
                if src.rd is None:
                    continue
                if cur.rd is None:
                    if cur.type == SINK:
                        src.rd.running = len(src.rd.current_running)
                        src.rd.slots = self.mtpp
                    continue
                src.rd.running += cur.rd.running
                src.rd.slots += cur.rd.slots

    # -- jobs and tasks (:161-208, :632-660, :895-929, :1183-1305)
    def add_or_update_job_nodes(self, jobs):
        queue, marked = deque(), set()
        for job in jobs:
            u = self.job_unsched.get(job["id"])
            if u is None:
                u = self._add_unsched(job["id"])
            root = job["root"]
            tn = self.task_node.get(root.uid)
            if tn is not None:
                queue.append((tn, root))
                marked.add(tn.id)
                continue
            if root.state in (RUNNABLE, RUNNING):
                tn = self._add_task(job["id"], root)
                self._update_unsched(u, 1)
                queue.append((tn, root))
                marked.add(tn.id)
            else:
                queue.append((None, root))
        self._update_flow_graph(queue, marked)

    def _add_unsched(self, jid):
        u = self.cm.add_node(JOB_AGG, 0)
        u.job = jid
        self.job_unsched[jid] = u
        return u

    def _add_task(self, jid, td):
        n = self.cm.add_node(UNSCHED_TASK, 1)
        n.task, n.job = td, jid
        self.sink.excess -= 1
        self.task_node[td.uid] = n
        return n

    def _update_unsched(self, u, d):
        a = u.out.get(self.sink.id)
        if a is not None:
            self.cm.change_arc(a, a.low, a.cap + d, 0)
            return
        assert d >= 1
        self.cm.add_arc(u, self.sink, 0, d, 0, ARC_OTHER)

    def _update_flow_graph(self, queue, marked):
        while queue:
            node, td = queue.popleft()
            if node is None:
                self._update_children(td, queue, marked)
            elif node.task is not None:
                self._update_task_node(node, queue, marked)
                self._update_children(td, queue, marked)
            elif node.type == EQUIV:
                self._update_ec(node, queue, marked)
            elif node.rd is not None:
                for a in list(node.out.values()):
                    if a.dst.rd is None:
                        self._res_to_sink(node)
                        continue
                    self.cm.change_arc_cost(a, 0)
                    if a.dst.id not in marked:
                        marked.add(a.dst.id)
                        queue.append((a.dst, None))
            else:
                raise AssertionError("unexpected node type")

    def _update_children(self, td, queue, marked):
        for c in td.spawned:
            cn = self.task_node.get(c.uid)
            if cn is not None:
                if cn.id not in marked:
                    queue.append((cn, c))
                    marked.add(cn.id)
                continue
            if c.state not in (RUNNABLE, RUNNING):
                queue.append((None, c))
                continue
            cn = self._add_task(c.job, c)
            self._update_unsched(self.job_unsched[c.job], 1)
            queue.append((cn, c))
            marked.add(cn.id)

    def _update_task_node(self, tn, queue, marked):
        if tn.task.state == RUNNING:                    # updateRunningTaskNode, Preemption off
            self.cm.change_arc_cost(self.running_arc[tn.task.uid], 0)
            return
        self._task_to_unsched(tn)
        # updateTaskToEquivArcs: the trivial model's only EC is the cluster aggregator
        ecn = self.ec_node.get(CLUSTER_AGG_EC)
        if ecn is None:
            ecn = self.cm.add_node(EQUIV, 0)
            ecn.ec = CLUSTER_AGG_EC
            self.ec_node[CLUSTER_AGG_EC] = ecn
        a = tn.out.get(ecn.id)
        if a is None:
            self.cm.add_arc(tn, ecn, 0, 1, 2, ARC_OTHER)
        else:
            self.cm.change_arc(a, a.low, a.cap, 2)
        if ecn.id not in marked:
            marked.add(ecn.id)
            queue.append((ecn, None))
        # updateTaskToResArcs: no preferences → drop arcs to resources
        for a in [a for a in tn.out.values() if a.dst.rd is not None]:
            self.cm.delete_arc(a)

    def _task_to_unsched(self, tn):
        u = self.job_unsched.get(tn.job) or self._add_unsched(tn.job)
        a = tn.out.get(u.id)
        if a is None:
            self.cm.add_arc(tn, u, 0, 1, 5, ARC_OTHER)
        else:
            self.cm.change_arc_cost(a, 5)

    def _update_ec(self, ecn, queue, marked):
        # updateEquivToEquivArcs: no EC→EC preferences; nothing to remove
        for muuid, mrd in self.machines.items():       # updateEquivToResArcs
            mn = self.res_node[muuid]
            cap = mrd.slots - mrd.running
            a = ecn.out.get(mn.id)
            if a is None:
                self.cm.add_arc(ecn, mn, 0, cap, 0, ARC_OTHER)
            else:
                self.cm.change_arc(a, a.low, cap, 0)
            if mn.id not in marked:
                marked.add(mn.id)
                queue.append((mn, None))

    # -- scheduling results (:253-339, :389-405, :454-475, :675-720)
    def update_all_costs_to_unscheduled_aggs(self):
        for u in list(self.job_unsched.values()):
            for a in list(u.inc.values()):
                if a.src.task.state == RUNNING:
                    self.cm.change_arc_cost(self.running_arc[a.src.task.uid], 0)
                else:
                    self._task_to_unsched(a.src)

    def task_scheduled(self, td, pu_node):
        tn = self.task_node[td.uid]
        tn.type = SCHED_TASK
        added = False
        for did, a in list(tn.out.items()):
            if did != pu_node.id:
                self.cm.delete_arc(a)
                continue
            added = True
            a.type = ARC_RUNNING
            self.cm.change_arc(a, 1, 1, 0)
            self.running_arc[td.uid] = a
        self._update_unsched(self.job_unsched[tn.job], -1)
        if not added:
            self.running_arc[td.uid] = self.cm.add_arc(tn, pu_node, 1, 1, 0, ARC_RUNNING)

    def task_completed(self, td):
        tn = self.task_node[td.uid]
        self.running_arc.pop(td.uid, None)
        tn.excess = 0
        self.sink.excess += 1
        del self.task_node[td.uid]
        self.cm.delete_node(tn)


class Scheduler:                                 # flowscheduler/scheduler.go
    def __init__(self, mtpp):
        self.gm = GraphManager(mtpp)
        self.root = RD(9000, COORD)
        self.gm.add_resource_topology(self.root)
        self.jobs: OrderedDict[int, dict] = OrderedDict()
        self.runnable: dict[int, set] = {}
        self.bindings: OrderedDict[int, RD] = OrderedDict()
        self.rds: dict[int, RD] = {}
        self.uid = 100

    def _next(self):
        self.uid += 1
        return self.uid

    def add_machine(self):                        # schedule_iteration_test.go:257-314
        pu = RD(self._next(), PU)
        core = RD(self._next(), CORE, [pu])
        m = RD(self._next(), MACHINE, [core])
        m.parent = self.root
        self.root.children.append(m)
        for rd in (m, core, pu):
            self.rds[rd.uuid] = rd
        self.gm.add_resource_topology(m)

    def add_job(self, ntasks):                    # schedule_iteration_test.go:152-162, 212-253
        jid = self._next()
        tasks = [Task(self._next(), jid) for _ in range(ntasks)]
        for t in tasks[1:]:
            tasks[0].spawned.append(t)
        self.jobs[jid] = {"id": jid, "root": tasks[0], "tasks": tasks}

    def _runnable_for(self, job):                 # :493-529
        q = deque()
        if job["root"].state in (CREATED, RUNNING, RUNNABLE, COMPLETED):
            q.append(job["root"])
        while q:
            t = q.popleft()
            q.extend(t.spawned)
            if t.state == CREATED:
                t.state = RUNNABLE
                self.runnable.setdefault(job["id"], set()).add(t.uid)
        return self.runnable.setdefault(job["id"], set())

    def schedule_all_jobs(self, solve):           # :309-375
        jds = [j for j in self.jobs.values() if self._runnable_for(j)]
        if not jds:
            return 0, None
        self.gm.compute_topology_statistics()
        self.stats = {"pu_running": {str(n.id): len(n.rd.current_running) for n in self.gm.res_node.values()
                                     if n.type == PU},
                      "slots_running": {str(n.id): [n.rd.slots, n.rd.running] for n in self.gm.res_node.values()}}
        self.gm.add_or_update_job_nodes(jds)
        mapping, info = solve(self.gm)
        # SchedulingDeltasForPreemptedTasks (:297-339): no task is preempted here; clear lists
        deltas = []
        for rd in self.rds.values():
            for tid in rd.current_running:
                tn = self.gm.task_node.get(tid)
                if tn is not None and tn.id not in mapping:
                    deltas.append(("PREEMPT", tid, rd))
            rd.current_running = []
        by_node = {n.id: n for n in self.gm.cm.g.nodes.values()}
        for tnid, pid in mapping.items():        # NodeBindingToSchedulingDelta (:253-295)
            tn, pn = by_node[tnid], by_node[pid]
            assert tn.task is not None and pn.type == PU
            bound = self.bindings.get(tn.task.uid)
            if bound is None:
                deltas.append(("PLACE", tn.task.uid, pn.rd))
            elif bound is not pn.rd:
                deltas.append(("MIGRATE", tn.task.uid, pn.rd))
            else:
                pn.rd.current_running.append(tn.task.uid)
        placed = 0
        for kind, tid, rd in deltas:              # applySchedulingDeltas (:377-412)
            assert kind == "PLACE", kind
            td = next(t for j in self.jobs.values() for t in j["tasks"] if t.uid == tid)
            self.gm.task_scheduled(td, self.gm.res_node[rd.uuid])
            rd.current_running.append(tid)        # bindTaskToResource (:421-437)
            self.bindings[tid] = rd
            self.runnable[td.job].discard(tid)
            td.state = RUNNING
            placed += 1
        info["placed"] = placed
        info["topology_stats"] = self.stats      # ComputeTopologyStatistics at the round's start
        info["deltas"] = [[kind, self._node_of_task(tid), self.gm.res_node[rd.uuid].id] for kind, tid, rd in deltas]
        return placed, info

    def _node_of_task(self, tid):
        n = self.gm.task_node.get(tid)
        return n.id if n is not None else 0

    def complete(self, td):                      # HandleTaskCompletion (:106-132)
        del self.bindings[td.uid]
        td.state = COMPLETED
        self.gm.task_completed(td)


def graph_arrays(gm: GraphManager):
    g = gm.cm.g
    n = max(g.nodes)
    ntype = np.zeros(n, np.int32)
    supply = np.zeros(n, np.int64)
    for v in g.nodes.values():
        ntype[v.id - 1] = dimacs_type(v.type)
        supply[v.id - 1] = v.excess
    arcs = list(g.arcs.values())
    a = lambda f: np.asarray([f(x) for x in arcs], np.int64)
    return gen.Graph(ntype, supply, a(lambda x: x.src.id), a(lambda x: x.dst.id), a(lambda x: x.low),
                     a(lambda x: x.cap), a(lambda x: x.cost))


def full_export(gm: GraphManager) -> str:        # dimacs/export.go:11-76
    g = gm.cm.g
    out = ["c ===========================", f"p min {len(g.nodes)} {len(g.arcs)}",
           "c ===========================", "c === ALL NODES FOLLOW ==="]
    out += [f"n {v.id} {v.excess} {dimacs_type(v.type)}" for v in g.nodes.values()]
    out.append("c === ALL ARCS FOLLOW ===")
    out += [f"a {a.src.id} {a.dst.id} {a.low} {a.cap} {a.cost}" for a in g.arcs.values()]
    out.append("c EOI")
    return "\n".join(out) + "\n"


def main():
    s = Scheduler(1)
    for _ in range(2):
        s.add_machine()
    for _ in range(3):
        s.add_job(1)
    rounds = []
    state = {"started": False}

    def solve(gm):                                # placement/solver.go:60-90
        if not state["started"]:
            state["started"] = True
            text = full_export(gm)
            kind = "full"
        else:
            gm.update_all_costs_to_unscheduled_aggs()
            text = "\n".join(gm.cm.changes) + ("\n" if gm.cm.changes else "") + "c EOI\n"
            kind = "incremental"
        gm.cm.changes = []
        g = graph_arrays(gm)
        sink = int(np.nonzero(g.ntype == 3)[0][0])
        assert g.supply[sink] == -int(g.supply[g.supply > 0].sum())   # the sink's drift is exact here
        st, cost, flow, fl, _ = ko.ssp(g)
        assert st == 0
        mapping = ko.bfs_mapping(g, fl, cost)
        rec = {"round": len(rounds) + 1, "kind": kind, "dimacs": text, "cost": int(cost), "flow": int(flow),
               "n": g.n, "m": g.m, "m_cap": int((g.cap > 0).sum()), "mapping": {str(k): int(v) for k, v in sorted(mapping.items())}}
        rounds.append(rec)
        return mapping, rec

    s.schedule_all_jobs(solve)                    # round 1
    s.add_job(2)
    s.schedule_all_jobs(solve)                    # round 2
    running = [t for j in s.jobs.values() for t in j["tasks"] if t.state == RUNNING][:2]
    for t in running:
        s.complete(t)
    s.schedule_all_jobs(solve)                    # rounds 3-5
    s.schedule_all_jobs(solve)
    s.schedule_all_jobs(solve)
    for r in rounds:
        print(f"round {r['round']}: {r['kind']:11s} n={r['n']} m={r['m']} cost={r['cost']} flow={r['flow']} "
              f"placed={r['placed']}")
    out = {"source": "scheduling/flow/flowscheduler/schedule_iteration_test.go:16-91, replayed through a "
                     "restatement of the reference graph manager (tests/golden/gen_multi_schedule.py)",
           "solver_args": "--graph_has_node_types=true --algorithm=successive_shortest_path "
                          "--print_assignments=false --debug_output=true (placement/solver.go:272-285)",
           "rounds": rounds}
    json.dump(out, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
