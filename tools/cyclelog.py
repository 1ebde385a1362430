#!/usr/bin/env python3
"""One config-3 solve (after a warm-up) with the engine's cycle log on, options
from the command line: python tools/cyclelog.py [k=v,...] [--config4]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ksched_amd import churn, gen, native  # noqa: E402

opts = {}
for kv in filter(None, (sys.argv[1] if len(sys.argv) > 1 and "=" in sys.argv[1] and not sys.argv[1].startswith("--") else "").split(",")):
    k, v = kv.split("=")
    opts[k] = int(v)
cfg = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--config=")), "config3")
T, M, R, J, seed = gen.CONFIGS["config3"]
if "--config4" in sys.argv:
    cell = churn.Cell(T, M, R, J, seed)
    ctx = native.Context(0, **opts)
    ctx.load_graph(cell.graph())
    ctx.solve()
    mp = ctx.task_mapping()
    for i in range(2):
        ctx.apply_deltas(cell.step(mp, done=T // 20, arrive=T // 20))
        ctx.solve()
        mp = ctx.task_mapping()
    ctx.close()
    ctx = native.Context(0, log_cycles=1, **opts)
    ctx.load_graph(cell.graph())
    ctx.solve()
    print("config4 round 3 graph:", ctx.solve().raw["ms"], file=sys.stderr)
else:
    g = gen.quincy(*gen.CONFIGS[cfg])
    ctx = native.Context(0, **opts)
    ctx.load_graph(g)
    ctx.solve()
    ctx.close()
    ctx = native.Context(0, log_cycles=1, **opts)
    ctx.load_graph(g)
    r = ctx.solve()
    print(cfg + ":", r.cost, r.raw["ms"], file=sys.stderr)
