#!/usr/bin/env python3
"""Per-kernel duration distribution from a rocprofv3 kernel_trace.csv."""
import collections
import csv
import glob
import sys

path = sys.argv[1]
f = glob.glob(f"{path}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
d = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].replace("ks::(anonymous namespace)::", "")
    name = name.split("(")[0] if not name.startswith("void ks") else name.split("(ks")[0]
    d[name[:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v2 = sorted(v)
    n = len(v2)
    print(f"{k:48s} n={n:6d} tot={sum(v2)/1e3:9.2f}ms p10={v2[n//10]:8.1f} p50={v2[n//2]:8.1f} "
          f"p90={v2[9*n//10]:8.1f} max={v2[-1]:8.1f}")
