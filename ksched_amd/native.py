"""ctypes binding of libksmcmf.so (include/ksmcmf.h).

The product path: every call goes to the in-tree HIP library. There is no CPU
fallback — if the library or a HIP device is missing, construction raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _build

KS_OK, KS_E_INVALID, KS_E_INFEASIBLE, KS_E_DEVICE, KS_E_VERIFY, KS_E_RANGE = 0, -1, -2, -3, -4, -5
KS_ADD_NODE, KS_REMOVE_NODE, KS_ADD_ARC, KS_UPDATE_ARC, KS_SET_EXCESS = 0, 1, 2, 3, 4

EXPORTED_SYMBOLS = (
    "ks_abi_version", "ks_default_opts", "ks_create", "ks_destroy", "ks_last_error", "ks_load_graph",
    "ks_apply_deltas", "ks_solve", "ks_get_flows", "ks_get_task_mapping", "ks_get_task_pu_device", "ks_solve_many",
    "ks_coalesce_deltas", "ks_get_store_stats", "ks_set_bindings", "ks_scheduling_deltas",
    "ks_update_unsched_costs", "ks_topology_stats", "ks_get_graph",
    "ks_batch_create", "ks_batch_create_rank", "ks_batch_unique_id", "ks_batch_destroy", "ks_batch_last_error",
    "ks_batch_load", "ks_batch_solve", "ks_batch_gather",
    "ks_batch_slots", "ks_batch_owner", "ks_batch_block_len", "ks_batch_unpack",
)
ABI_VERSION = 5
KS_DELTA_PLACE, KS_DELTA_PREEMPT, KS_DELTA_MIGRATE, KS_DELTA_NOOP = 0, 1, 2, 3
KS_COST_SET, KS_COST_ADD = 0, 1

NODE_DT = np.dtype({"names": ["id", "excess", "type", "_pad"],
                    "formats": ["<u8", "<i8", "<i4", "<i4"], "offsets": [0, 8, 16, 20], "itemsize": 24})
ARC_DT = np.dtype({"names": ["src", "dst", "low", "cap", "cost", "type", "_pad"],
                   "formats": ["<u8", "<u8", "<u8", "<u8", "<i8", "<i4", "<i4"],
                   "offsets": [0, 8, 16, 24, 32, 40, 44], "itemsize": 48})
DELTA_DT = np.dtype({"names": ["kind", "type", "id", "src", "dst", "low", "cap", "cost", "old_cost", "excess"],
                     "formats": ["<i4", "<i4", "<u8", "<u8", "<u8", "<u8", "<u8", "<i8", "<i8", "<i8"],
                     "offsets": [0, 4, 8, 16, 24, 32, 40, 48, 56, 64], "itemsize": 72})
SCHED_DELTA_DT = np.dtype({"names": ["type", "_pad", "task", "pu"], "formats": ["<i4", "<i4", "<u8", "<u8"],
                           "offsets": [0, 4, 8, 16], "itemsize": 24})
FLOW_DT = np.dtype({"names": ["src", "dst", "flow"], "formats": ["<u8", "<u8", "<i8"],
                    "offsets": [0, 8, 16], "itemsize": 24})


class KsOpts(C.Structure):
    """ks_opts (include/ksmcmf.h): 0 in a tuning field selects the library default."""
    _fields_ = [("alpha", C.c_int32), ("verify", C.c_int32), ("auto_sink", C.c_int32),
                ("price_refine", C.c_int32), ("gu_interval", C.c_int32), ("warm_start", C.c_int32),
                ("walk_slack", C.c_int32), ("final_div", C.c_int32), ("pr_rounds", C.c_int32),
                ("phase_exit", C.c_int32), ("phase_frac", C.c_int32), ("tail_sweeps", C.c_int32),
                ("bf_margin", C.c_int32), ("two_hop", C.c_int32), ("log_cycles", C.c_int32),
                ("fault_inject", C.c_int32), ("walk_passes", C.c_int32), ("tail_nodes", C.c_int32),
                ("bf_bound", C.c_int32), ("fwd_nodes", C.c_int32), ("cell_nodes", C.c_int32),
                ("warm_shift", C.c_int32),
                ("warm_canon", C.c_int32),
                ("compact_pos", C.c_int32)]


class KsResult(C.Structure):
    _fields_ = [("total_cost", C.c_int64), ("flow_value", C.c_int64), ("status", C.c_int32),
                ("phases", C.c_int32), ("sweeps", C.c_uint64), ("arc_scans", C.c_uint64),
                ("node_visits", C.c_uint64), ("pushes", C.c_uint64), ("relabels", C.c_uint64),
                ("global_updates", C.c_uint64), ("gu_iterations", C.c_uint64), ("gu_arc_scans", C.c_uint64),
                ("ms_phase", C.c_double * 6), ("n_nodes", C.c_int64), ("n_arcs", C.c_int64),
                ("sweep_launches", C.c_uint64), ("ms_sweep_kernels", C.c_double),
                ("gu_launches", C.c_uint64), ("ms_gu_kernels", C.c_double), ("warm_started", C.c_int32),
                ("rebuilt", C.c_int32), ("recoveries", C.c_int32), ("solver", C.c_int32),
                ("fs_launches", C.c_uint64), ("ms_fs_kernels", C.c_double), ("fwd_updates", C.c_uint64),
                ("cells", C.c_int32), ("compact", C.c_int32), ("ms_cell_kernel", C.c_double),
                ("cell_ticks_max", C.c_uint64), ("cell_ticks_sum", C.c_uint64), ("fs_arc_scans", C.c_uint64),
                ("cell_fallbacks", C.c_uint64), ("cycles_cancelled", C.c_uint64), ("fb_resets", C.c_uint64),
                ("cycles_rejected", C.c_uint64), ("gu_leaf_scans", C.c_uint64), ("reserved3", C.c_uint64 * 2)]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("ms_phase", "reserved3")}
        names = ("build", "saturate", "cycles", "price_refine", "verify", "total")
        d["ms"] = dict(zip(names, list(self.ms_phase)))
        return d


class KsStoreStats(C.Structure):
    _fields_ = [("live_arcs", C.c_int64), ("inserted", C.c_int64), ("updated", C.c_int64),
                ("killed", C.c_int64), ("superseded", C.c_int64), ("rebuilds", C.c_int64),
                ("residual_slots", C.c_int64), ("reserved", C.c_int64 * 4)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


class KsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ksmcmf error {code}: {msg}")
        self.code = code


_LIB = None


def lib_path() -> str:
    """The in-tree library; KS_LIB_VARIANT=<tag> selects libksmcmf_<tag>.so built
    by _build.build_variant (compile-time tuning experiments)."""
    tag = os.environ.get("KS_LIB_VARIANT")
    return _build.variant_path(tag) if tag else _build.LIB


_VARIANTS: dict = {}


def load(build_if_missing: bool = True, variant: str | None = None):
    """Load the in-tree library (building it with hipcc if absent and allowed).
    variant: an in-tree build of it, ksched_amd/libksmcmf_<variant>.so (tests use
    the fake-communicator build "fakecomm", _build.build_fake_comm)."""
    global _LIB
    if variant is not None:
        if variant not in _VARIANTS:
            path = _build.variant_path(variant)
            if not os.path.exists(path):
                raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
            _VARIANTS[variant] = _bind(path)
        return _VARIANTS[variant]
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        if not build_if_missing:
            raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
        _build.build()
    _LIB = _bind(path)
    return _LIB


def _bind(path: str):
    if os.environ.get("KS_PRELOAD_TORCH", "1") != "0":
        # One HIP runtime per process: torch ships its own libamdhip64 (SONAME
        # libamdhip64.so.7) and links it by file name, so if the library loaded
        # /opt/rocm's copy first, a later torch.cuda init would bring up a second
        # HIP/HSA runtime and fail ("No HIP GPUs are available"). Importing torch
        # first makes libksmcmf bind to the runtime already loaded (same SONAME),
        # so the RCCL gather and the solver share device pointers and streams.
        import torch  # noqa: F401
    L = C.CDLL(path)
    P, V = C.POINTER, C.c_void_p
    L.ks_abi_version.restype = C.c_int
    L.ks_default_opts.argtypes = [P(KsOpts)]
    L.ks_create.argtypes = [C.c_int, P(KsOpts)]
    L.ks_create.restype = V
    L.ks_destroy.argtypes = [V]
    L.ks_last_error.argtypes = [V]
    L.ks_last_error.restype = C.c_char_p
    L.ks_load_graph.argtypes = [V, V, C.c_size_t, V, C.c_size_t]
    L.ks_apply_deltas.argtypes = [V, V, C.c_size_t]
    L.ks_solve.argtypes = [V, P(KsResult)]
    L.ks_get_flows.argtypes = [V, V, C.c_size_t, P(C.c_size_t)]
    L.ks_get_task_mapping.argtypes = [V, V, V, C.c_size_t, P(C.c_size_t)]
    L.ks_get_task_pu_device.argtypes = [V, V, C.c_size_t, P(C.c_size_t)]
    L.ks_solve_many.argtypes = [P(V), C.c_size_t, C.c_int, P(KsResult)]
    L.ks_coalesce_deltas.argtypes = [V, C.c_size_t, V, C.c_size_t, P(C.c_size_t)]
    L.ks_get_store_stats.argtypes = [V, P(KsStoreStats)]
    L.ks_get_graph.argtypes = [V, V, C.c_size_t, P(C.c_size_t), V, C.c_size_t, P(C.c_size_t)]
    L.ks_batch_create.argtypes = [P(C.c_int), C.c_int, P(KsOpts)]
    L.ks_batch_create.restype = V
    L.ks_batch_create_rank.argtypes = [C.c_int, C.c_int, C.c_int, V, P(KsOpts)]
    L.ks_batch_create_rank.restype = V
    L.ks_batch_unique_id.argtypes = [V]
    L.ks_batch_destroy.argtypes = [V]
    L.ks_batch_last_error.argtypes = [V]
    L.ks_batch_last_error.restype = C.c_char_p
    L.ks_batch_load.argtypes = [V, C.c_size_t, P(V), P(C.c_size_t), P(V), P(C.c_size_t)]
    L.ks_batch_solve.argtypes = [V, P(KsResult)]
    L.ks_batch_gather.argtypes = [V, C.c_size_t, V, V, V]
    L.ks_batch_slots.argtypes = [C.c_size_t, C.c_int]
    L.ks_batch_slots.restype = C.c_size_t
    L.ks_batch_owner.argtypes = [C.c_size_t, C.c_int, P(C.c_int), P(C.c_size_t)]
    L.ks_batch_block_len.argtypes = [C.c_size_t, C.c_int, C.c_size_t]
    L.ks_batch_block_len.restype = C.c_size_t
    L.ks_batch_unpack.argtypes = [V, C.c_size_t, C.c_int, C.c_size_t, V, V, V]
    L.ks_set_bindings.argtypes = [V, V, V, C.c_size_t]
    L.ks_scheduling_deltas.argtypes = [V, C.c_int, V, C.c_size_t, P(C.c_size_t)]
    L.ks_update_unsched_costs.argtypes = [V, V, C.c_size_t, C.c_int32, C.c_int64, C.c_int64, P(C.c_size_t)]
    L.ks_topology_stats.argtypes = [V, C.c_uint64, V, V, C.c_size_t, V, V, C.c_size_t, P(C.c_size_t)]
    return L


def default_opts(**kw) -> KsOpts:
    o = KsOpts()
    load().ks_default_opts(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


@dataclass
class SolveResult:
    cost: int
    flow: int
    raw: dict


class Context:
    """One solver context on one HIP device (ks_create … ks_destroy)."""

    def __init__(self, device: int = 0, **opts):
        self._L = load()
        self.opts = default_opts(**opts)
        h = self._L.ks_create(device, C.byref(self.opts))
        if not h:
            raise KsError(KS_E_DEVICE, f"ks_create failed: no usable HIP device {device}")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.ks_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int):
        if rc != KS_OK:
            raise KsError(rc, self._L.ks_last_error(self._h).decode(errors="replace"))

    # -- graph upload -------------------------------------------------------
    def load_arrays(self, nodes: np.ndarray, arcs: np.ndarray):
        nodes = np.ascontiguousarray(nodes, NODE_DT)
        arcs = np.ascontiguousarray(arcs, ARC_DT)
        self._check(self._L.ks_load_graph(self._h, nodes.ctypes.data, nodes.shape[0],
                                          arcs.ctypes.data, arcs.shape[0]))

    def load_graph(self, g):
        """Upload a ksched_amd.gen.Graph (1-based ids, all nodes alive)."""
        nodes = np.zeros(g.n, NODE_DT)
        nodes["id"] = np.arange(1, g.n + 1, dtype=np.uint64)
        nodes["excess"] = g.supply
        nodes["type"] = g.ntype
        arcs = np.zeros(g.m, ARC_DT)
        arcs["src"], arcs["dst"] = g.src, g.dst
        arcs["low"], arcs["cap"], arcs["cost"] = g.low, g.cap, g.cost
        arcs["type"] = g.arc_types()
        self.load_arrays(nodes, arcs)

    def apply_deltas(self, deltas: np.ndarray):
        deltas = np.ascontiguousarray(deltas, DELTA_DT)
        self._check(self._L.ks_apply_deltas(self._h, deltas.ctypes.data, deltas.shape[0]))

    # -- solve & results ----------------------------------------------------
    def solve(self) -> SolveResult:
        r = KsResult()
        rc = self._L.ks_solve(self._h, C.byref(r))
        self._check(rc)
        return SolveResult(r.total_cost, r.flow_value, r.as_dict())

    def flows(self) -> np.ndarray:
        cnt = C.c_size_t()
        self._check(self._L.ks_get_flows(self._h, None, 0, C.byref(cnt)))
        out = np.zeros(cnt.value, FLOW_DT)
        self._check(self._L.ks_get_flows(self._h, out.ctypes.data, cnt.value, C.byref(cnt)))
        return out

    def task_mapping_arrays(self) -> tuple[np.ndarray, np.ndarray]:
        """ks_get_task_mapping as the C-ABI returns it: parallel (task id, PU id) arrays."""
        cnt = C.c_size_t()
        self._check(self._L.ks_get_task_mapping(self._h, None, None, 0, C.byref(cnt)))
        t = np.zeros(cnt.value, np.uint64)
        p = np.zeros(cnt.value, np.uint64)
        self._check(self._L.ks_get_task_mapping(self._h, t.ctypes.data, p.ctypes.data, cnt.value, C.byref(cnt)))
        return t[:cnt.value], p[:cnt.value]

    def task_mapping(self) -> dict[int, int]:
        t, p = self.task_mapping_arrays()
        return dict(zip(t.tolist(), p.tolist()))

    def store_stats(self) -> dict:
        st = KsStoreStats()
        self._check(self._L.ks_get_store_stats(self._h, C.byref(st)))
        return st.as_dict()

    def graph(self):
        """The device-resident graph: (nodes NODE_DT, arcs ARC_DT)."""
        n, m = C.c_size_t(), C.c_size_t()
        self._check(self._L.ks_get_graph(self._h, None, 0, C.byref(n), None, 0, C.byref(m)))
        nodes = np.zeros(n.value, NODE_DT)
        arcs = np.zeros(m.value, ARC_DT)
        self._check(self._L.ks_get_graph(self._h, nodes.ctypes.data, n.value, C.byref(n), arcs.ctypes.data, m.value,
                                         C.byref(m)))
        return nodes, arcs

    # -- scheduler-side sweeps on device (ks_sched.hip) ----------------------
    def set_bindings(self, bindings: dict[int, int]):
        t = np.fromiter(bindings.keys(), np.uint64, len(bindings))
        p = np.fromiter(bindings.values(), np.uint64, len(bindings))
        self._check(self._L.ks_set_bindings(self._h, t.ctypes.data, p.ctypes.data, t.shape[0]))

    def scheduling_deltas(self, commit: bool = True) -> np.ndarray:
        """PREEMPT / PLACE / MIGRATE records (SCHED_DELTA_DT) of the last solve."""
        cnt = C.c_size_t()
        self._check(self._L.ks_scheduling_deltas(self._h, 0, None, 0, C.byref(cnt)))
        out = np.zeros(cnt.value, SCHED_DELTA_DT)
        self._check(self._L.ks_scheduling_deltas(self._h, int(commit), out.ctypes.data, cnt.value, C.byref(cnt)))
        return out[:cnt.value]

    def update_unsched_costs(self, cost: int, mode: int = KS_COST_SET, continuation: int = 0,
                             unsched_ids=None) -> int:
        ch = C.c_size_t()
        ids = None if unsched_ids is None else np.ascontiguousarray(unsched_ids, np.uint64)
        self._check(self._L.ks_update_unsched_costs(self._h, None if ids is None else ids.ctypes.data,
                                                    0 if ids is None else ids.shape[0], mode, cost, continuation,
                                                    C.byref(ch)))
        return ch.value

    def topology_stats(self, max_tasks_per_pu: int, pu_running: dict[int, int] | None = None):
        """(slots_below, running_below) per node id − 1."""
        cnt = C.c_size_t()
        self._check(self._L.ks_topology_stats(self._h, max_tasks_per_pu, None, None, 0, None, None, 0,
                                              C.byref(cnt)))
        sl = np.zeros(cnt.value, np.uint64)
        rn = np.zeros(cnt.value, np.uint64)
        ids = vals = None
        k = 0
        if pu_running is not None:
            ids = np.fromiter(pu_running.keys(), np.uint64, len(pu_running))
            vals = np.fromiter(pu_running.values(), np.uint64, len(pu_running))
            k = ids.shape[0]
        self._check(self._L.ks_topology_stats(self._h, max_tasks_per_pu, None if ids is None else ids.ctypes.data,
                                              None if vals is None else vals.ctypes.data, k, sl.ctypes.data,
                                              rn.ctypes.data, cnt.value, C.byref(cnt)))
        return sl, rn

    def task_pu_device(self, dev_ptr: int, cap: int) -> int:
        cnt = C.c_size_t()
        self._check(self._L.ks_get_task_pu_device(self._h, C.c_void_p(dev_ptr), cap, C.byref(cnt)))
        return cnt.value


def graph_arrays(g):
    """gen.Graph → (NODE_DT, ARC_DT) arrays with 1-based ids."""
    nodes = np.zeros(g.n, NODE_DT)
    nodes["id"] = np.arange(1, g.n + 1, dtype=np.uint64)
    nodes["excess"] = g.supply
    nodes["type"] = g.ntype
    arcs = np.zeros(g.m, ARC_DT)
    arcs["src"], arcs["dst"] = g.src, g.dst
    arcs["low"], arcs["cap"], arcs["cost"] = g.low, g.cap, g.cost
    arcs["type"] = g.arc_types()
    return nodes, arcs


class Batch:
    """Config 5 through the C-ABI (ks_batch_*): independent graphs, graph g on
    global rank g mod world, each device solving the union of its graphs; the
    per-graph rows gathered to rank 0 over RCCL inside libksmcmf.

    Batch(devices=[0, 1, ...]) drives several devices from one process;
    Batch(device=d, world=W, rank=r, uid=bytes) is one rank of a
    process-per-GPU job (uid from Batch.unique_id() on rank 0)."""

    def __init__(self, devices=None, device: int = 0, world: int = 1, rank: int = 0, uid: bytes | None = None,
                 variant: str | None = None, **opts):
        self._L = load(variant=variant)   # variant: an in-tree test build (tests: "fakecomm")
        self.opts = default_opts(**opts)
        if uid is None:
            devs = list(devices if devices is not None else [device])
            arr = (C.c_int * len(devs))(*devs)
            h = self._L.ks_batch_create(arr, len(devs), C.byref(self.opts))
            self.local = len(devs)
        else:
            buf = C.create_string_buffer(bytes(uid), 128)
            h = self._L.ks_batch_create_rank(device, world, rank, buf, C.byref(self.opts))
            self.local = 1
        if not h:
            raise KsError(KS_E_DEVICE, "ks_batch_create failed (device or RCCL unavailable)")
        self._h = h
        self.ngraphs = 0

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        rc = load().ks_batch_unique_id(buf)
        if rc != KS_OK:
            raise KsError(rc, "ks_batch_unique_id failed")
        return buf.raw

    def _check(self, rc):
        if rc != KS_OK:
            raise KsError(rc, self._L.ks_batch_last_error(self._h).decode(errors="replace"))

    def close(self):
        if getattr(self, "_h", None):
            self._L.ks_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load(self, graphs):
        arrs = [graph_arrays(g) for g in graphs]
        k = len(arrs)
        self._keep = arrs
        npt = (C.c_void_p * max(1, k))(*[a[0].ctypes.data for a in arrs])
        apt = (C.c_void_p * max(1, k))(*[a[1].ctypes.data for a in arrs])
        ns = (C.c_size_t * max(1, k))(*[a[0].shape[0] for a in arrs])
        ms = (C.c_size_t * max(1, k))(*[a[1].shape[0] for a in arrs])
        self._check(self._L.ks_batch_load(self._h, k, npt, ns, apt, ms))
        self.ngraphs = k

    def solve(self) -> list[SolveResult]:
        rs = (KsResult * self.local)()
        self._check(self._L.ks_batch_solve(self._h, rs))
        return [SolveResult(r.total_cost, r.flow_value, r.as_dict()) for r in rs]

    def gather(self, max_tasks: int, root: bool = True):
        """→ (pu [ngraphs, max_tasks] uint64, cost [ngraphs], flow [ngraphs]) on rank 0."""
        pu = np.zeros((self.ngraphs, max_tasks), np.uint64) if root else None
        cost = np.zeros(self.ngraphs, np.int64) if root else None
        flow = np.zeros(self.ngraphs, np.int64) if root else None
        p = lambda a: None if a is None else a.ctypes.data
        self._check(self._L.ks_batch_gather(self._h, max_tasks, p(pu), p(cost), p(flow)))
        return pu, cost, flow


def batch_owner(g: int, world: int) -> tuple[int, int]:
    """ks_batch_owner: (global rank, slot on that rank) of graph g."""
    r, sl = C.c_int(), C.c_size_t()
    if load().ks_batch_owner(g, world, C.byref(r), C.byref(sl)) != KS_OK:
        raise KsError(KS_E_INVALID, "ks_batch_owner")
    return r.value, sl.value


def batch_block_len(ngraphs: int, world: int, max_tasks: int) -> int:
    return int(load().ks_batch_block_len(ngraphs, world, max_tasks))


def batch_unpack(gathered: np.ndarray, ngraphs: int, world: int, max_tasks: int):
    """ks_batch_unpack over the world blocks rank 0 received → (pu, cost, flow) in graph order."""
    gathered = np.ascontiguousarray(gathered, np.int64)
    pu = np.zeros((ngraphs, max_tasks), np.uint64)
    cost = np.zeros(ngraphs, np.int64)
    flow = np.zeros(ngraphs, np.int64)
    rc = load().ks_batch_unpack(gathered.ctypes.data, ngraphs, world, max_tasks, pu.ctypes.data, cost.ctypes.data,
                                flow.ctypes.data)
    if rc != KS_OK:
        raise KsError(rc, "ks_batch_unpack: a rank reported a failure")
    return pu, cost, flow


def solve_many(ctxs: list[Context], workers: int = 0) -> list[SolveResult]:
    """ks_solve_many: solve independent contexts concurrently (native worker
    threads, one stream per context). Raises KsError on the first failure."""
    L = load()
    k = len(ctxs)
    hs = (C.c_void_p * max(1, k))(*[c._h for c in ctxs])
    rs = (KsResult * max(1, k))()
    rc = L.ks_solve_many(hs, k, workers, rs)
    if rc != KS_OK:
        bad = next((c for c, r in zip(ctxs, rs) if r.status != KS_OK), None)
        if bad is None:   # rejected before any solve ran (e.g. a null context)
            raise KsError(rc, "ks_solve_many failed")
        bad._check(rc)
    return [SolveResult(r.total_cost, r.flow_value, r.as_dict()) for r in rs[:k]]


def coalesce_deltas(deltas: np.ndarray) -> np.ndarray:
    """ks_coalesce_deltas: the change optimisers of graph_change_manager.go:220-279
    (merge per arc, drop duplicates, purge before node removal). Host-only."""
    d = np.ascontiguousarray(deltas, DELTA_DT)
    out = np.zeros(d.shape[0], DELTA_DT)
    cnt = C.c_size_t()
    rc = load().ks_coalesce_deltas(d.ctypes.data, d.shape[0], out.ctypes.data, d.shape[0], C.byref(cnt))
    if rc != KS_OK:
        raise KsError(rc, "ks_coalesce_deltas: invalid node id in delta stream")
    return out[:cnt.value]
