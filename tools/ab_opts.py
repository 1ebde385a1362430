#!/usr/bin/env python3
"""Interleaved A/B of solver options (ks_opts fields) — or, with --variant TAG, of the
default library against libksmcmf_TAG.so (same options) — on one GPU: config-3 solves
and config-4 churn rounds, every result checked against the golden / the other
variant. Each variant has its own context on the same graph; solves alternate
A, B, A, B … so clock and thermal drift hit both alike.

    python tools/ab_opts.py --a "" --b "bf_bound=-1" [--solves 20] [--rounds 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ksched_amd import churn, gen, native  # noqa: E402


def parse(spec):
    out = {}
    for kv in filter(None, (x.strip() for x in spec.split(","))):
        k, v = kv.split("=")
        out[k] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default="")
    ap.add_argument("--b", default="")
    ap.add_argument("--solves", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--config", default="config3", help="solves: gen.CONFIGS name (config2, config3)")
    ap.add_argument("--variant", default="", help="b runs libksmcmf_<variant>.so (a: the default library)")
    a = ap.parse_args()
    va, vb = parse(a.a), parse(a.b)
    libs = {}
    if a.variant:
        os.environ.pop("KS_LIB_VARIANT", None)
        native._LIB = None
        libs["a"] = native.load()
        os.environ["KS_LIB_VARIANT"] = a.variant
        native._LIB = None
        libs["b"] = native.load()

    def make(k, v):
        if libs:
            native._LIB = libs[k]
        return native.Context(0, **v)
    T, M, R, J, seed = gen.CONFIGS["config3"]
    out = {"a": va, "b": vb}
    if a.solves:
        g = gen.quincy(*gen.CONFIGS[a.config])
        ref = None
        ctx = {k: make(k, v) for k, v in (("a", va), ("b", vb))}
        for c in ctx.values():
            c.load_graph(g)
            c.solve()
        ms = {"a": [], "b": []}
        upd = {"a": [], "b": []}
        for i in range(a.solves):
            for k in (("a", "b") if i % 2 == 0 else ("b", "a")):
                t0 = time.perf_counter()
                r = ctx[k].solve()
                ms[k].append(1e3 * (time.perf_counter() - t0))
                upd[k].append(r.raw["global_updates"])
                ref = ref or (r.cost, r.flow)
                if (r.cost, r.flow) != ref or (a.config == "config3" and r.cost != 3257656):
                    raise SystemExit(f"{a.config} variant {k}: cost {r.cost} flow {r.flow} (reference {ref})")
        for k in ("a", "b"):
            x = np.array(ms[k])
            print(f"{a.config} {k}: median {np.median(x):.2f} mean {x.mean():.2f} "
                  f"min {x.min():.2f} ms, updates {np.mean(upd[k]):.1f}")
        out[a.config] = {k: [round(x, 2) for x in ms[k]] for k in ms}
        for c in ctx.values():
            c.close()
    if a.rounds:
        # one churn stream (driven by variant a's mappings) applied to both contexts:
        # the same graph every round, so the costs must agree exactly
        cell = churn.Cell(T, M, R, J, seed)
        ctx = {k: make(k, v) for k, v in (("a", va), ("b", vb))}
        g = cell.graph()
        for k in ("a", "b"):
            ctx[k].load_graph(g)
            ctx[k].solve()
        mp = ctx["a"].task_mapping()
        ms = {"a": [], "b": []}
        for i in range(a.rounds):
            d = cell.step(mp, done=T // 20, arrive=T // 20)
            costs = {}
            for k in (("a", "b") if i % 2 == 0 else ("b", "a")):
                ctx[k].apply_deltas(d)
                t0 = time.perf_counter()
                r = ctx[k].solve()
                ms[k].append(1e3 * (time.perf_counter() - t0))
                costs[k] = (r.cost, r.flow)
            if costs["a"] != costs["b"]:
                raise SystemExit(f"config4 round {i + 1}: costs differ {costs}")
            mp = ctx["a"].task_mapping()
        for k in ("a", "b"):
            x = np.array(ms[k])
            print(f"config4 {k}: solve median {np.median(x):.2f} mean {x.mean():.2f} ms over {a.rounds} rounds")
        out["config4"] = {k: [round(x, 2) for x in ms[k]] for k in ms}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
