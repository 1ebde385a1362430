#!/usr/bin/env python3
"""Quick GPU check of the cell solver (ks_cell.hip) against the committed goldens,
beside the multi-kernel engine on the same graphs (cell_nodes = -1).

    python tools/cell_check.py [--reps N] [--graphs K]

Prints one line per graph: golden cost, each path's cost and solve ms, the cell
solver's in-kernel ticks, phases, updates, sweeps and Bellman-Ford rounds."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ksched_amd import gen, native  # noqa: E402


def graph_of(e):
    if e["family"] == "trivial":
        return gen.trivial(*e["params"])
    return gen.quincy(*e["params"], e["seed"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--graphs", type=int, default=8)
    ap.add_argument("--engine", type=int, default=1, help="also time the multi-kernel engine")
    ap.add_argument("--min-n", type=int, default=0)
    ap.add_argument("--log", type=int, default=0, help="ks_opts.log_cycles on the cell path (per-op times on stderr)")
    ap.add_argument("--opts", default="{}", help="JSON ks_opts overrides for the cell path, e.g. '{\"gu_interval\": 48}'")
    args = ap.parse_args()
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "goldens.json")))["graphs"]
    sel = [e for e in gold if args.min_n <= e["n"] <= 14000][: args.graphs]
    bad = 0
    for e in sel:
        g = graph_of(e)
        row = {"family": e["family"], "params": e["params"], "seed": e["seed"], "n": g.n, "gold": e["cost"]}
        for name, opts in (("cell", {"log_cycles": args.log, "cell_nodes": 1 << 16, **json.loads(args.opts)}), ("engine", {"cell_nodes": -1})):
            if name == "engine" and not args.engine:
                continue
            ctx = native.Context(0, **opts)
            ctx.load_graph(g)
            ts, r = [], None
            for _ in range(args.reps):
                t0 = time.perf_counter()
                r = ctx.solve()
                ts.append(1e3 * (time.perf_counter() - t0))
            ok = r.cost == e["cost"] and r.flow == e["flow"]
            bad += not ok
            row[name] = {"cost": r.cost, "ok": ok, "ms": [round(x, 2) for x in ts], "solver": r.raw["solver"],
                         "phases": r.raw["phases"], "updates": r.raw["global_updates"], "sweeps": r.raw["sweeps"],
                         "bf_rounds": r.raw["gu_iterations"], "recoveries": r.raw["recoveries"],
                         "kernel_ms": round(r.raw["ms_cell_kernel"], 3), "ticks_max": r.raw["cell_ticks_max"]}
            ctx.close()
        print(json.dumps(row), flush=True)
    print("BAD", bad, flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
