#!/usr/bin/env python3
"""Kernel-time histogram by duration bin (rocprofv3 kernel trace): where the
solve's device time goes — many short launches or a few long ones."""
import collections
import csv
import glob
import re
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
bins = [0, 4, 6, 8, 10, 15, 20, 30, 50, 100, 1e9]
agg = collections.defaultdict(lambda: [[0, 0.0] for _ in bins])
for r in rows:
    m = re.search(r"(k_\w+)(<\w+>)?", r["Kernel_Name"])
    name = (m.group(1) + (m.group(2) or "")) if m else "other"
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for i in range(len(bins) - 1):
        if bins[i] <= d < bins[i + 1]:
            agg[name][i][0] += 1
            agg[name][i][1] += d
for name in ("k_sweep", "k_bf_round<false>"):
    tot = sum(x[1] for x in agg[name])
    print(name, f"total {tot/1e3:.1f} ms")
    for i in range(len(bins) - 1):
        n, t = agg[name][i]
        if n:
            print(f"   {bins[i]:>4}-{bins[i+1]:<6} us: n={n:6d} time {t/1e3:7.2f} ms ({100*t/tot:5.1f}%)")
