"""ctypes binding of the CPU oracle (oracle/libksoracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg — never by the ksched_amd product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class KoGraph(C.Structure):
    _fields_ = [("n", C.c_int64), ("m", C.c_int64),
                ("ntype", C.POINTER(C.c_int32)), ("supply", C.POINTER(C.c_int64)),
                ("src", C.POINTER(C.c_int64)), ("dst", C.POINTER(C.c_int64)),
                ("low", C.POINTER(C.c_int64)), ("cap", C.POINTER(C.c_int64)),
                ("cost", C.POINTER(C.c_int64))]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "libksoracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libksoracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        P = C.POINTER
        L.ko_ssp.argtypes = [P(KoGraph), P(C.c_int64), P(C.c_int64), P(C.c_int64), P(C.c_int64)]
        L.ko_cost_scaling.argtypes = [P(KoGraph), C.c_int, P(C.c_int64), P(C.c_int64), P(C.c_int64)]
        L.ko_verify.argtypes = [P(KoGraph), P(C.c_int64), P(C.c_int64), P(C.c_int64)]
        L.ko_gen_quincy.argtypes = [C.c_int64] * 4 + [C.c_uint64, P(KoGraph)]
        L.ko_gen_trivial.argtypes = [C.c_int64] * 3 + [P(KoGraph)]
        L.ko_quincy_sizes.argtypes = [C.c_int64] * 4 + [P(C.c_int64), P(C.c_int64)]
        L.ko_trivial_sizes.argtypes = [C.c_int64] * 2 + [P(C.c_int64), P(C.c_int64)]
        L.ko_reference_path.argtypes = [P(KoGraph), P(C.c_int64), P(C.c_int64), P(C.c_int64), P(C.c_double)]
        L.ko_export_dimacs.argtypes = [P(KoGraph), C.c_char_p, C.c_int64]
        L.ko_export_dimacs.restype = C.c_int64
        L.ko_flow_lines.argtypes = [P(KoGraph), P(C.c_int64), C.c_int64, C.c_char_p, C.c_int64]
        L.ko_flow_lines.restype = C.c_int64
        L.ko_bfs_mapping_from_lines.argtypes = [P(KoGraph), C.c_char_p, C.c_int64, P(C.c_int64), P(C.c_int64)]
        L.ko_bfs_mapping_from_lines.restype = C.c_int64
        V = C.c_void_p
        L.ko_ssp_incremental.argtypes = [P(KoGraph), V, V, V, C.c_int64, V, C.c_int64, V, V, V,
                                         P(C.c_int64), P(C.c_int64), P(C.c_int64), P(C.c_double)]
        L.ko_reference_path_incremental.argtypes = [P(KoGraph), V, C.c_int64, V, V, V, C.c_int64, V, C.c_int64, V,
                                                    V, V, P(C.c_int64), P(C.c_int64), P(C.c_int64),
                                                    P(C.c_double)]
        L.ko_export_changes.argtypes = [V, C.c_int64, C.c_char_p, C.c_int64]
        L.ko_export_changes.restype = C.c_int64
        L.ko_parse_changes.argtypes = [C.c_char_p, C.c_int64, V, C.c_int64]
        L.ko_parse_changes.restype = C.c_int64
        _LIB = L
    return _LIB


class _Holder:
    """Keeps numpy arrays alive behind a KoGraph view."""

    def __init__(self, g):
        p64 = lambda a: np.ascontiguousarray(a, np.int64)
        self.ntype = np.ascontiguousarray(g.ntype, np.int32)
        self.supply, self.src, self.dst = p64(g.supply), p64(g.src), p64(g.dst)
        self.low, self.cap, self.cost = p64(g.low), p64(g.cap), p64(g.cost)
        P = lambda a, t: a.ctypes.data_as(C.POINTER(t))
        self.kg = KoGraph(self.ntype.shape[0], self.src.shape[0], P(self.ntype, C.c_int32),
                          P(self.supply, C.c_int64), P(self.src, C.c_int64), P(self.dst, C.c_int64),
                          P(self.low, C.c_int64), P(self.cap, C.c_int64), P(self.cost, C.c_int64))


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_int64))


def ssp(g):
    """Successive shortest path → (status, cost, flow_value, flows[m], augmentations)."""
    h = _Holder(g)
    flow = np.zeros(h.src.shape[0], np.int64)
    cost, fv, aug = C.c_int64(), C.c_int64(), C.c_int64()
    st = lib().ko_ssp(C.byref(h.kg), _p(flow), C.byref(cost), C.byref(fv), C.byref(aug))
    return st, cost.value, fv.value, flow, aug.value


def cost_scaling(g, alpha: int = 12):
    h = _Holder(g)
    flow = np.zeros(h.src.shape[0], np.int64)
    cost, fv = C.c_int64(), C.c_int64()
    st = lib().ko_cost_scaling(C.byref(h.kg), alpha, _p(flow), C.byref(cost), C.byref(fv))
    return st, cost.value, fv.value, flow


def verify(g, flow):
    """→ (status 0 ok / 1 capacity / 2 conservation, cost, Σ positive supply)."""
    h = _Holder(g)
    f = np.ascontiguousarray(flow, np.int64)
    cost, fv = C.c_int64(), C.c_int64()
    st = lib().ko_verify(C.byref(h.kg), _p(f), C.byref(cost), C.byref(fv))
    return st, cost.value, fv.value


def reference_path(g):
    """export → parse → SSP → f lines → BFS mapping; → (status, cost, flow, mapped, ms[5])."""
    h = _Holder(g)
    cost, fv, nm = C.c_int64(), C.c_int64(), C.c_int64()
    ms = (C.c_double * 5)()
    st = lib().ko_reference_path(C.byref(h.kg), C.byref(cost), C.byref(fv), C.byref(nm), ms)
    return st, cost.value, fv.value, nm.value, list(ms)


def export_dimacs(g) -> str:
    h = _Holder(g)
    need = lib().ko_export_dimacs(C.byref(h.kg), None, 0)
    buf = C.create_string_buffer(int(need) + 1)
    ln = lib().ko_export_dimacs(C.byref(h.kg), buf, need + 1)
    return buf.raw[:ln].decode()


def bfs_mapping(g, flow, cost: int = 0):
    """Reference-faithful parseFlowToMapping over the f lines of `flow`."""
    h = _Holder(g)
    f = np.ascontiguousarray(flow, np.int64)
    need = lib().ko_flow_lines(C.byref(h.kg), _p(f), cost, None, 0)
    buf = C.create_string_buffer(int(need) + 1)
    ln = lib().ko_flow_lines(C.byref(h.kg), _p(f), cost, buf, need + 1)
    tk = np.zeros(h.ntype.shape[0] + 1, np.int64)
    pu = np.zeros(h.ntype.shape[0] + 1, np.int64)
    k = lib().ko_bfs_mapping_from_lines(C.byref(h.kg), buf, ln, _p(tk), _p(pu))
    if k < 0:
        raise RuntimeError("Task Node to Resource Node should be 1:1 mapping")
    return dict(zip(tk[:k].tolist(), pu[:k].tolist()))


def bfs_mapping_from_text(g, text: str):
    """Reference-faithful parseFlowToMapping over an "f"/"s"/"c EOI" text block
    (e.g. a solver daemon's output); raises like solver.go:223-225."""
    h = _Holder(g)
    raw = text.encode()
    tk = np.zeros(h.ntype.shape[0] + 1, np.int64)
    pu = np.zeros(h.ntype.shape[0] + 1, np.int64)
    k = lib().ko_bfs_mapping_from_lines(C.byref(h.kg), raw, len(raw), _p(tk), _p(pu))
    if k < 0:
        raise RuntimeError("Task Node to Resource Node should be 1:1 mapping")
    return dict(zip(tk[:k].tolist(), pu[:k].tolist()))


DELTA_DT = np.dtype({"names": ["kind", "type", "id", "src", "dst", "low", "cap", "cost", "old_cost", "excess"],
                     "formats": ["<i4", "<i4", "<u8", "<u8", "<u8", "<u8", "<u8", "<i8", "<i8", "<i8"],
                     "offsets": [0, 4, 8, 16, 24, 32, 40, 48, 56, 64], "itemsize": 72})


class IncrementalSSP:
    """Flowlessly's daemon mode restated (ko_ssp_incremental): each round re-solves
    from the previous round's flow (carried by (src, dst)) and potentials (by node
    id). ``round(g, deltas, fresh_ids)`` runs the whole later-Solve reference path:
    the change block as text and parsed back, the incremental SSP, the "f" lines
    and the BFS mapping (ko_reference_path_incremental). The first call (no
    previous state) is a cold SSP."""

    def __init__(self):
        self.src = self.dst = self.flow = self.pot = None
        self.last = None

    def round(self, g, deltas=None, fresh_ids=()):
        h = _Holder(g)
        n, m = h.ntype.shape[0], h.src.shape[0]
        flow = np.zeros(m, np.int64)
        pot = np.zeros(n, np.int64)
        cost, fv, nm = C.c_int64(), C.c_int64(), C.c_int64()
        ms = (C.c_double * 6)()
        if self.pot is None:
            self.src = np.zeros(0, np.int64)
            self.dst = np.zeros(0, np.int64)
            self.flow = np.zeros(0, np.int64)
            self.pot = np.zeros(0, np.int64)
        fresh = np.zeros(n, np.uint8)
        ids = np.asarray(list(fresh_ids), np.int64)
        if ids.size:
            fresh[ids - 1] = 1
        d = np.ascontiguousarray(deltas if deltas is not None else np.zeros(0, DELTA_DT), DELTA_DT)
        cp = lambda a: a.ctypes.data
        st = lib().ko_reference_path_incremental(
            C.byref(h.kg), cp(d), d.shape[0], cp(self.src), cp(self.dst), cp(self.flow), self.src.shape[0],
            cp(self.pot), self.pot.shape[0], cp(fresh), cp(flow), cp(pot), C.byref(cost), C.byref(fv),
            C.byref(nm), ms)
        if st < 0:
            raise RuntimeError(f"ko_reference_path_incremental failed ({st})")
        self.src, self.dst, self.flow, self.pot = h.src.copy(), h.dst.copy(), flow, pot
        self.last = {"status": st, "cost": cost.value, "flow": fv.value, "mapped": nm.value,
                     "ms": dict(zip(("export", "parse", "carry", "saturate", "augment", "flines_bfs"), list(ms)))}
        return st, cost.value, fv.value, flow

    def export_changes(self, deltas) -> str:
        d = np.ascontiguousarray(deltas, DELTA_DT)
        need = lib().ko_export_changes(d.ctypes.data, d.shape[0], None, 0)
        buf = C.create_string_buffer(int(need) + 1)
        ln = lib().ko_export_changes(d.ctypes.data, d.shape[0], buf, need + 1)
        return buf.raw[:ln].decode()


def parse_changes(text: str) -> np.ndarray:
    raw = text.encode()
    out = np.zeros(raw.count(b"\n") + 1, DELTA_DT)
    k = lib().ko_parse_changes(raw, len(raw), out.ctypes.data, out.shape[0])
    if k < 0:
        raise ValueError("malformed change block")
    return out[:k]


def gen_quincy(T, M, R, J, seed):
    """The C generator's arrays (to check the numpy twin bit-for-bit)."""
    n, m = C.c_int64(), C.c_int64()
    lib().ko_quincy_sizes(T, M, R, J, C.byref(n), C.byref(m))

    class G:
        pass

    g = G()
    g.ntype = np.zeros(n.value, np.int32)
    for k in ("supply",):
        setattr(g, k, np.zeros(n.value, np.int64))
    for k in ("src", "dst", "low", "cap", "cost"):
        setattr(g, k, np.zeros(m.value, np.int64))
    h = _Holder(g)
    st = lib().ko_gen_quincy(T, M, R, J, seed, C.byref(h.kg))
    if st:
        raise ValueError("ko_gen_quincy failed")
    for k in ("ntype", "supply", "src", "dst", "low", "cap", "cost"):
        setattr(g, k, getattr(h, k))
    return g
