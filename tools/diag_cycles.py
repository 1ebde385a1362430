#!/usr/bin/env python3
"""Per-phase / per-cycle breakdown of config-3 solves and config-4 rounds from
the engine's cycle log (ks_opts.log_cycles = 1: one stderr line per update
cycle). Usage: python tools/diag_cycles.py OUT_DIR [--solves K] [--rounds R]"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PAT = re.compile(r"cycle phase (\d+) eps (\d+) bf (\d+) bf_ms ([\d.]+) sw_ms ([\d.]+) active (\d+) n_exc (\d+)")


def summarize(path):
    phases = {}
    solves = 0
    for line in open(path):
        if line.startswith("solve phases"):
            solves += 1
        m = PAT.search(line)
        if not m:
            continue
        ph, eps, bf, bfm, swm, act, nx = m.groups()
        p = phases.setdefault(int(ph), {"eps": int(eps), "cycles": 0, "bf_rounds": 0, "bf_ms": 0.0, "sw_ms": 0.0,
                                        "tail_cycles": 0})
        p["cycles"] += 1
        p["bf_rounds"] += int(bf)
        p["bf_ms"] += float(bfm)
        p["sw_ms"] += float(swm)
        p["tail_cycles"] += int(nx) <= 64
    for k in sorted(phases):
        p = phases[k]
        print(f"phase {k} eps {p['eps']}: cycles {p['cycles'] / max(1, solves):.1f}  tail cycles "
              f"{p['tail_cycles'] / max(1, solves):.1f}  bf rounds {p['bf_rounds'] / max(1, solves):.0f}  "
              f"bf ms {p['bf_ms'] / max(1, solves):.2f}  sweep ms {p['sw_ms'] / max(1, solves):.2f}")


def run(args):
    from ksched_amd import churn, gen, native
    T, M, R, J, seed = gen.CONFIGS["config3"]
    cell = churn.Cell(T, M, R, J, seed)
    ctx = native.Context(0, log_cycles=1)
    ctx.load_graph(cell.graph())
    for i in range(args.solves):
        r = ctx.solve()
        print(f"# config3 solve {i}: {r.raw['ms']['total']:.2f} ms cost {r.cost} phases {r.raw['phases']} "
              f"updates {r.raw['global_updates']} sweeps {r.raw['sweeps']} bf {r.raw['gu_iterations']}",
              file=sys.stderr, flush=True)
    mp = ctx.task_mapping()
    for i in range(args.rounds):
        d = cell.step(mp, done=T // 20, arrive=T // 20)
        ctx.apply_deltas(d)
        r = ctx.solve()
        mp = ctx.task_mapping()
        print(f"# config4 round {i + 1}: {r.raw['ms']['total']:.2f} ms cost {r.cost} phases {r.raw['phases']} "
              f"updates {r.raw['global_updates']} sweeps {r.raw['sweeps']} bf {r.raw['gu_iterations']}",
              file=sys.stderr, flush=True)
    ctx.close()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--solves", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--inner", action="store_true")
    ap.add_argument("--summarize", action="store_true")
    a = ap.parse_args()
    if a.inner:
        run(a)
    elif a.summarize:
        summarize(os.path.join(a.out, "cycles3.log"))
        summarize(os.path.join(a.out, "cycles4.log"))
    else:
        os.makedirs(a.out, exist_ok=True)
        for name, extra in (("cycles3.log", ["--rounds", "0"]), ("cycles4.log", ["--solves", "1", "--rounds",
                                                                                  str(a.rounds)])):
            with open(os.path.join(a.out, name), "w") as f:
                subprocess.run([sys.executable, __file__, a.out, "--inner", *extra] +
                               (["--solves", str(a.solves)] if name == "cycles3.log" else []),
                               stderr=f, check=True, timeout=600)
        print("== config 3 (per solve)")
        summarize(os.path.join(a.out, "cycles3.log"))
        print("== config 4 (the initial solve + rounds, per solve)")
        summarize(os.path.join(a.out, "cycles4.log"))
