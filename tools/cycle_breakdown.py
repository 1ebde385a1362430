#!/usr/bin/env python3
"""Per-cycle time model of ONE solve: rocprofv3 kernel trace (last solve in the
trace) joined with the engine's KS_TRACE per-sweep visit counts.

    python tools/cycle_breakdown.py <rocprof dir> <trace.jsonl>

A cycle = [k_gu_init] k_bf_round* k_gu_max k_gu_apply k_sweep*; prints, per
cycle bucket of total sweep visits, the count of cycles and the mean time spent
in BF rounds, sweeps and the rest."""
import csv
import glob
import json
import re
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
tr = [json.loads(l) for l in open(sys.argv[2])]
visits = tr[-1]["visits"]


def short(n):
    m = re.search(r"(k_\w+)(<\w+>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:30]


ks = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
# last solve: from the last k_make_keys pair onwards
starts = [i for i, k in enumerate(ks) if k[0] == "k_make_keys"]
ks = ks[starts[-2]:] if len(starts) >= 2 else ks
cycles = []
cur = None
sweep_i = 0
for name, t0, t1 in ks:
    d = (t1 - t0) / 1e3
    if name in ("k_gu_init",) or (name.startswith("k_bf_round<false>") and cur is not None and cur["sw_n"] > 0):
        cur = {"bf": 0.0, "bf_n": 0, "sw": 0.0, "sw_n": 0, "other": 0.0, "visits": 0, "t0": t0, "t1": t1}
        cycles.append(cur)
    if cur is None:
        continue
    cur["t1"] = t1
    if name.startswith("k_bf_round<false>"):
        cur["bf"] += d
        cur["bf_n"] += 1
    elif name == "k_sweep":
        cur["sw"] += d
        cur["sw_n"] += 1
        if sweep_i < len(visits):
            cur["visits"] += visits[sweep_i]
        sweep_i += 1
    else:
        cur["other"] += d
buckets = [(0, 0), (1, 100), (101, 1000), (1001, 10000), (10001, 10**9)]
print(f"cycles {len(cycles)}  sweeps matched {sweep_i} of {len(visits)}")
print(f"{'visits':>14} {'cyc':>4} {'bf_n':>6} {'bf_us':>8} {'sw_us':>8} {'other':>7} {'wall_us':>8} {'tot_ms':>7}")
for lo, hi in buckets:
    cs = [c for c in cycles if lo <= c["visits"] <= hi]
    if not cs:
        continue
    n = len(cs)
    wall = sum((c["t1"] - c["t0"]) / 1e3 for c in cs)
    print(f"{lo:>6}-{hi:<7} {n:4d} {sum(c['bf_n'] for c in cs)/n:6.1f} {sum(c['bf'] for c in cs)/n:8.1f} "
          f"{sum(c['sw'] for c in cs)/n:8.1f} {sum(c['other'] for c in cs)/n:7.1f} {wall/n:8.1f} {wall/1e3:7.2f}")
