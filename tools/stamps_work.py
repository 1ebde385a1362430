#!/usr/bin/env python3
"""Per-launch work vs span from a KS_STAMPS file (tools/stamps.py --out): for the
Bellman-Ford rounds, how many relaxations each launch did and how long its
working blocks took, bucketed by work. Usage: python tools/stamps_work.py FILE SOLVES"""
import sys

import numpy as np

rows = np.loadtxt(sys.argv[1], dtype=np.int64, ndmin=2)
solves = int(sys.argv[2]) if len(sys.argv) > 2 else 1
for name, sel in (("sweep", rows[:, 0] < 4096), ("bf", rows[:, 0] >= 4096)):
    x = rows[sel]
    span = (x[:, 2] - x[:, 1]) * 0.01
    work = x[:, 10]
    print(f"== {name}: {len(x) / solves:.0f} working launches per solve, {span.sum() / 1e3 / solves:.2f} ms of spans, "
          f"{work.sum() / solves:.0f} units")
    edges = [0, 16, 64, 256, 1024, 4096, 16384, 65536, 1 << 40]
    for lo, hi in zip(edges[:-1], edges[1:]):
        m = (work >= lo) & (work < hi)
        if m.any():
            print(f"  work [{lo:6d},{hi if hi < 1 << 40 else 'inf'}): launches {m.sum() / solves:7.1f}  "
                  f"span p50 {np.median(span[m]):6.1f} us  sum {span[m].sum() / 1e3 / solves:6.2f} ms  "
                  f"units {work[m].sum() / solves:10.0f}")
