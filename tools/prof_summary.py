#!/usr/bin/env python3
"""Summarise a rocprofv3 run (rocpd .db or *_kernel_stats.csv) into a small CSV.

    python tools/prof_summary.py gpurun_out/<tag>/prof > profiles/<name>.csv
"""
import csv
import glob
import os
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = name.replace("ks::(anonymous namespace)::", "ks::")
    name = re.sub(r"\(.*", "", name) if name.startswith("ks::") else name
    if "rocprim" in name:
        m = re.search(r"detail::(\w+?)(_kernel|<)", name)
        name = "rocprim::" + (m.group(1) if m else "kernel")
    return name


def rows_from(path):
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    csvs = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
    if csvs:
        for r in csv.DictReader(open(csvs[0])):
            yield short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3, \
                float(r["Percentage"])
    elif dbs:
        c = sqlite3.connect(dbs[0])
        for name, calls, tot, avg, pct in c.execute("select * from top_kernels"):
            yield short(name), calls, tot, avg, pct  # rocpd views report microseconds


def main():
    agg = {}
    for name, calls, tot, avg, pct in rows_from(sys.argv[1]):
        a = agg.setdefault(name, [0, 0.0, 0.0])
        a[0] += calls
        a[1] += tot
        a[2] += pct
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "calls", "total_us", "avg_us", "pct"])
    for name, (calls, tot, pct) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        w.writerow([name, calls, round(tot, 1), round(tot / calls, 3), round(pct, 2)])


if __name__ == "__main__":
    main()
