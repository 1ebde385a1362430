#!/usr/bin/env python3
"""Per-kernel mean PMC value per dispatch from rocprofv3 --pmc counter_collection CSVs.

    python tools/pmc_summary.py <dir-with-FETCH_SIZE-run> <dir-with-WRITE_SIZE-run> > profiles/pmc_traffic.json
"""
import collections
import csv
import glob
import json
import re
import sys


def load(path):
    f = glob.glob(f"{path}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        if not m:
            continue
        k = m.group(1)
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(cnt[k]) for c, v in d.items()} for k, d in acc.items()}, {k: len(v) for k, v in cnt.items()}


fetch, nf = load(sys.argv[1])
write, nw = load(sys.argv[2])
out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), mean per dispatch; "
                 "FETCH_SIZE/WRITE_SIZE in KB as rocprofv3 derives them; gfx950 FETCH_SIZE is uncalibrated "
                 "for 4-8 B gathers (MI355X_MICROARCH.md HBM section), reported raw",
       "unit": "bytes"}
for k in sorted(set(fetch) | set(write)):
    fr = fetch.get(k, {}).get("FETCH_SIZE", 0.0) * 1024.0
    wr = write.get(k, {}).get("WRITE_SIZE", 0.0) * 1024.0
    out[k] = {"fetch_bytes_per_launch": round(fr, 1), "write_bytes_per_launch": round(wr, 1),
              "bytes_per_launch": round(fr + wr, 1), "dispatches": nf.get(k, 0)}
print(json.dumps(out, indent=1))
