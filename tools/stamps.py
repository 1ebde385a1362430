#!/usr/bin/env python3
"""Critical-path diagnostic for the solver's sweep / BF-round launches.

Needs the KS_STAMPS build variant (ksched_amd/libksmcmf_stamps.so, built with
`_build.build_variant("stamps", ["KS_STAMPS=1"])`). Solves one Quincy workload
and, per launch, reports the span from the earliest block start to the latest
end of a block that did work, tagged with the kind of that last block:
1 hub chunk, 2 chunked node, 3 + c window class c (BF rounds: 1 hub, 3 other).

    KS_LIB_VARIANT=stamps python tools/stamps.py [config3] [--solves 2]
"""
import argparse
import os
import sys
from collections import defaultdict

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("KS_LIB_VARIANT", "stamps")

from ksched_amd import gen, native  # noqa: E402

KINDS = {0: "idle", 1: "hub", 2: "chunked", 3: "cls0(4)", 4: "cls1(8)", 5: "cls2(16)", 6: "cls3(32)", 7: "cls4(64)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="config3")
    ap.add_argument("--solves", type=int, default=2)
    ap.add_argument("--out", default="gpurun_out/stamps.txt")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    T, M, R, J, seed = gen.CONFIGS[a.config]
    g = gen.quincy(T, M, R, J, seed)
    ctx = native.Context(0, warm_start=0)
    ctx.load_graph(g)
    ctx.solve()                      # warm-up (no stamps)
    if os.path.exists(a.out):
        os.remove(a.out)
    os.environ["KS_STAMPS_OUT"] = a.out
    r = None
    for _ in range(a.solves):
        r = ctx.solve()
    print(f"cost {r.cost} flow {r.flow}")
    rows = np.loadtxt(a.out, dtype=np.int64, ndmin=2)
    for name, sel in (("sweep", rows[:, 0] < 4096), ("bf", rows[:, 0] >= 4096)):
        x = rows[sel]
        if not len(x):
            continue
        span = (x[:, 2] - x[:, 1]) * 0.01      # s_memrealtime: 100 MHz → 10 ns ticks
        print(f"{name}: launches with work {len(x)} (over {a.solves} solves), span p10/p50/p90 "
              f"{np.percentile(span, 10):.1f}/{np.percentile(span, 50):.1f}/{np.percentile(span, 90):.1f} us, "
              f"sum {span.sum() / 1e3 / a.solves:.2f} ms/solve")
        late = x[:, 4] * 0.01
        print(f"   latest working-block start after first: p50 {np.median(late):.1f} us p90 {np.percentile(late, 90):.1f} us")
        by = defaultdict(list)
        for k, s in zip(x[:, 3], span):
            by[int(k)].append(s)
        for k in sorted(by):
            v = np.array(by[k])
            print(f"   last block {KINDS.get(k, k):10s} n={len(v):6d} span p50 {np.median(v):6.1f} us "
                  f"p90 {np.percentile(v, 90):6.1f} us sum {v.sum() / 1e3 / a.solves:7.2f} ms/solve")
        for k in range(1, 8):
            d = x[:, 4 + k] * 0.01
            d = d[d > 0]
            if len(d):
                print(f"   longest {KINDS[k]:10s} block: in {len(d):5d} launches, p50 {np.median(d):6.1f} us "
                      f"p90 {np.percentile(d, 90):6.1f} us")
    for name, sel, unit in (("sweep", rows[:, 0] < 4096, "active nodes"), ("bf", rows[:, 0] >= 4096, "arc scans")):
        x = rows[sel]
        span = (x[:, 2] - x[:, 1]) * 0.01
        work = x[:, 12]
        print(f"{name}: time by {unit} per launch")
        edges = [0, 16, 64, 256, 1024, 4096, 16384, 65536, 1 << 40]
        for lo, hi in zip(edges[:-1], edges[1:]):
            m = (work >= lo) & (work < hi)
            if m.any():
                print(f"   [{lo:6d}, {hi if hi < 1 << 40 else 'inf'}): launches {m.sum():5d} "
                      f"span p50 {np.median(span[m]):6.1f} us, sum {span[m].sum() / 1e3 / a.solves:6.2f} ms/solve")
    ctx.close()


if __name__ == "__main__":
    main()
