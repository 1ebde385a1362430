#!/usr/bin/env python3
"""Per-kernel sums of one rocprofv3 --pmc counter pass (counter_collection.csv).

    python tools/pmc_per_kernel.py <pass dir> [<pass dir> ...]
prints {kernel: {counter: total, "dispatches": n}} as JSON.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    """k_bf_round<false, true>(…) → k_bf_round<false>; k_sweep<true>(…) → k_sweep: the
    record-layout template argument (round 5, the last one) is dropped."""
    m = re.search(r"(k_\w+)(<([\w, ]+)>)?\(", name)
    if not m:
        return name.split("(")[0][-60:]
    targs = [t.strip() for t in (m.group(3) or "").split(",") if t.strip()]
    if m.group(1) == "k_bf_round" and len(targs) == 2:
        targs = targs[:1]
    elif m.group(1) in ("k_sweep", "k_saturate", "k_augment", "k_aug_hub", "k_fs_round", "k_fs_trace",
                        "k_cyc_cancel"):
        targs = []
    return m.group(1) + (f"<{', '.join(targs)}>" if targs else "")


def main():
    out = defaultdict(dict)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            seen = defaultdict(set)
            for r in csv.DictReader(open(f)):
                k = short(r["Kernel_Name"])
                c = r["Counter_Name"]
                out[k][c] = out[k].get(c, 0.0) + float(r["Counter_Value"])
                seen[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            counters = defaultdict(set)
            for r in csv.DictReader(open(f)):
                counters[short(r["Kernel_Name"])].add(r["Counter_Name"])
            for k, s in seen.items():
                out[k]["dispatches"] = max(out[k].get("dispatches", 0), len(s))
                for c in counters[k]:   # each pass is its own run: per-launch values use its own count
                    out[k][c + "_dispatches"] = out[k].get(c + "_dispatches", 0) + len(s)
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
