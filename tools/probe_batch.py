"""Diagnostic for ks_solve_many: first solves run concurrently on fresh contexts
(the bench's warmup), compared with sequential solves of the same graphs."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
from ksched_amd import gen, native  # noqa: E402

T, M, R, J, _ = gen.CONFIGS["config2"]
num = int(sys.argv[1]) if len(sys.argv) > 1 else 64
workers = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,4").split(",")]
graphs = [gen.quincy(T, M, R, J, 1000 + k) for k in range(num)]

ref = []
with native.Context(0) as c:
    for g in graphs:
        c.load_graph(g)
        ref.append(c.solve().cost)
print("reference costs computed", flush=True)

for w in workers:
    for trial in range(2):
        ctxs = [native.Context(0) for _ in graphs]
        for c, g in zip(ctxs, graphs):
            c.load_graph(g)
        t0 = time.perf_counter()
        try:
            res = native.solve_many(ctxs, workers=w)
            bad = [k for k, r in enumerate(res) if r.cost != ref[k]]
            print("fresh contexts, workers", w, "trial", trial, "ms", round(1e3 * (time.perf_counter() - t0), 1),
                  "mismatch", bad, flush=True)
        except native.KsError as e:
            print("fresh contexts, workers", w, "trial", trial, "error", e, flush=True)
        try:
            res = native.solve_many(ctxs, workers=w)
            bad = [k for k, r in enumerate(res) if r.cost != ref[k]]
            print("   second solve mismatch", bad, flush=True)
        except native.KsError as e:
            print("   second solve error", e, flush=True)
        for c in ctxs:
            c.close()
