"""Time the host graph store (ks_apply_deltas, the compaction inside ks_solve)
on the config-4 delta stream, with a stub engine (tools/hostbench/stub_engine.cpp)."""
import ctypes as C
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["KS_PRELOAD_TORCH"] = "0"
from ksched_amd import churn, native  # noqa: E402

so = "/tmp/ks_hostonly.so"
subprocess.run(["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-I" + os.path.join(ROOT, "include"),
                os.path.join(ROOT, "ksched_amd/csrc/ks_host.cpp"), os.path.join(ROOT, "tools/hostbench/stub_engine.cpp"),
                "-o", so], check=True)
L = C.CDLL(so)
L.ks_create.restype = C.c_void_p
L.ks_create.argtypes = [C.c_int, C.c_void_p]
for f in ("ks_load_graph", "ks_apply_deltas", "ks_solve"):
    getattr(L, f).restype = C.c_int
L.ks_load_graph.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
L.ks_apply_deltas.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
L.ks_solve.argtypes = [C.c_void_p, C.c_void_p]
h = L.ks_create(0, None)
T, M, R, J = 100_000, 10_000, 250, 1_000
cell = churn.Cell(T, M, R, J, 3)
g = cell.graph()
import numpy as np  # noqa: E402
nodes = np.zeros(g.n, native.NODE_DT)
nodes["id"] = np.arange(1, g.n + 1)
nodes["excess"], nodes["type"] = g.supply, g.ntype
arcs = np.zeros(g.m, native.ARC_DT)
arcs["src"], arcs["dst"], arcs["low"], arcs["cap"], arcs["cost"] = g.src, g.dst, g.low, g.cap, g.cost
t = time.perf_counter(); assert L.ks_load_graph(h, nodes.ctypes.data, g.n, arcs.ctypes.data, g.m) == 0
print(f"load_graph {1e3*(time.perf_counter()-t):.1f} ms")
res = (C.c_char * 512)()
t = time.perf_counter(); assert L.ks_solve(h, res) == 0
print(f"first solve (compaction+upload) {1e3*(time.perf_counter()-t):.1f} ms")
# a mapping that places the first 95% of tasks on PUs round-robin (stands in for a solve)
def fill(tasks):
    free = cell.slots - cell.running_on
    slots = np.repeat(cell.PU0 + np.arange(M), np.maximum(free, 0))
    k = min(tasks.shape[0], slots.shape[0])
    return dict(zip(tasks[:k].tolist(), slots[:k].tolist()))


mp = fill(cell.task_ids(cell.WAIT))
for rnd in range(4):
    d = cell.step(mp, done=5000, arrive=5000)
    t = time.perf_counter(); assert L.ks_apply_deltas(h, d.ctypes.data, d.shape[0]) == 0
    ta = time.perf_counter(); assert L.ks_solve(h, res) == 0
    tb = time.perf_counter()
    print(f"round {rnd+1}: {d.shape[0]} deltas apply {1e3*(ta-t):.1f} ms, compaction {1e3*(tb-ta):.1f} ms")
    mp = fill(cell.task_ids(cell.WAIT))
