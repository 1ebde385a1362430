#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV (per-dispatch start/end): per kernel
the duration distribution, and the idle gaps between consecutive dispatches.

    python tools/kernel_trace.py <dir with *kernel_trace.csv> [--kernels k_sweep,k_bf_round]
"""
import csv
import glob
import os
import re
import sys

import numpy as np


def main():
    d = sys.argv[1]
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                m = re.search(r"(k_\w+)(<([\w, ]+)>)?\(", name)
                if m:   # the record-layout parameter (true/false last) is dropped: k_bf_round<false, true> → k_bf_round<false>
                    targs = [t.strip() for t in (m.group(3) or "").split(",") if t.strip()]
                    if m.group(1) in ("k_bf_round",) and len(targs) == 2:
                        targs = targs[:1]
                    elif m.group(1) in ("k_sweep", "k_saturate", "k_augment", "k_aug_hub", "k_fs_round", "k_fs_trace"):
                        targs = []
                    short = m.group(1) + (f"<{', '.join(targs)}>" if targs else "")
                else:
                    short = name.replace("(anonymous namespace)", "")[:40]
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
    rows.sort()
    st = np.array([r[0] for r in rows], np.int64)
    en = np.array([r[1] for r in rows], np.int64)
    names = np.array([r[2] for r in rows])
    dur = (en - st) / 1e3
    gaps = np.maximum(0, st[1:] - en[:-1]) / 1e3
    print(f"dispatches {len(rows)}, busy {dur.sum() / 1e3:.2f} ms, span {(en.max() - st.min()) / 1e6:.2f} ms")
    for k in sorted(set(names), key=lambda k: -dur[names == k].sum()):
        x = dur[names == k]
        if x.sum() < 100:
            continue
        q = np.percentile(x, [10, 50, 90, 99])
        print(f"{k[:40]:40s} n={len(x):6d} sum={x.sum() / 1e3:8.2f}ms p10={q[0]:6.1f} p50={q[1]:6.1f} "
              f"p90={q[2]:6.1f} p99={q[3]:6.1f} us; <2us: {(x < 2).sum()}")
    for k in ("k_bf_round<false>", "k_sweep"):
        x = dur[names == k]
        if not len(x):
            continue
        print(f"{k}: device time by launch duration")
        edges = [0, 3, 6, 10, 15, 25, 40, 70, 120, 1e9]
        for lo, hi in zip(edges[:-1], edges[1:]):
            m = (x >= lo) & (x < hi)
            if m.any():
                print(f"   [{lo:4.0f}, {hi:4.0f}) us: n={m.sum():6d} sum={x[m].sum() / 1e3:7.2f} ms")
    if "--seq" in sys.argv:   # the Bellman-Ford round durations of each update, in launch order
        cur = []
        for k, d in zip(names, dur):
            if k == "k_gu_init":
                if cur:
                    print("update:", " ".join(f"{v:.0f}" for v in cur))
                cur = []
            elif k == "k_bf_round<false>" and d >= 3:
                cur.append(d)
    if "--cycles" in sys.argv:   # one line per cycle: span, host gap before it, device time by kernel kind
        kinds = {"k_bf_round<false>": "bf", "k_sweep": "sw", "k_augment": "aug", "k_aug_hub": "hub"}
        starts = [i for i, k in enumerate(names) if k == "k_gu_init"]
        print("cycle span_us host_gap_us bf_n bf_us bf_work_n sw_us aug_us other_us idle_us")
        for c, i0 in enumerate(starts):
            i1 = starts[c + 1] if c + 1 < len(starts) else len(names)
            ends = [j for j in range(i0, i1) if names[j] == "k_cycle_end"]
            if not ends:
                continue
            j1 = ends[0] + 1
            span = (en[j1 - 1] - st[i0]) / 1e3
            hgap = (st[i0] - en[i0 - 1]) / 1e3 if i0 > 0 else 0.0
            acc = {"bf": 0.0, "sw": 0.0, "aug": 0.0, "hub": 0.0, "other": 0.0}
            nbf = nbfw = 0
            for j in range(i0, j1):
                kd = kinds.get(names[j], "other")
                acc[kd] += dur[j]
                if kd == "bf":
                    nbf += 1
                    nbfw += dur[j] >= 3
            busy = sum(acc.values())
            print(f"{c} {span:.0f} {hgap:.0f} {nbf} {acc['bf']:.0f} {nbfw} {acc['sw']:.0f} "
                  f"{acc['aug'] + acc['hub']:.0f} {acc['other']:.0f} {span - busy:.0f}")
    print(f"gaps: n={len(gaps)} sum={gaps.sum() / 1e3:.2f} ms p50={np.median(gaps):.2f} p90={np.percentile(gaps, 90):.2f} us")


if __name__ == "__main__":
    main()
