#!/usr/bin/env python3
"""Bellman-Ford round durations by position within an update (rocprofv3 kernel trace)."""
import collections
import csv
import glob
import re
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    m = re.search(r"(k_\w+)(<\w+>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:30]


prev, idx = None, 0
stats = collections.defaultdict(list)
for r in rows:
    s = short(r["Kernel_Name"])
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if s.startswith("k_bf_round"):
        idx = 0 if prev in ("k_gu_init", "k_pr_init") else (idx + 1 if prev and prev.startswith("k_bf_round") else 99)
        b = "r0" if idx == 0 else "r1-3" if idx < 4 else "r4-15" if idx < 16 else "r16-31" if idx < 32 else "r32+"
        stats[f"{s} {b}"].append(dur)
    elif s == "k_sweep":
        stats["sweep"].append(dur)
    prev = s
for k in sorted(stats):
    d = sorted(stats[k])
    n = len(d)
    print(f"{k:28s} n={n:6d} p50 {d[n//2]:7.1f} p90 {d[9*n//10]:7.1f} max {d[-1]:7.1f} tot {sum(d)/1e3:7.1f}ms")
