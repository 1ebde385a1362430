#!/usr/bin/env python3
"""Per-variant summary of an ab.sh run: ms/step, and the per-launch device time of
k_sweep and k_bf_round (event-timed, all timed steps) — launch counts vary run to
run with the solver's race order, per-launch time does not.

    python tools/ab_summary.py gpurun_out/<tag>
"""
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    rows = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        name = os.path.basename(f).rsplit(".", 2)[0]
        try:
            j = json.load(open(f))
        except Exception:
            continue
        ok = j.get("roofline", {}).get("other_kernel")
        if not ok:
            continue
        sw, bf = ok["k_sweep"], ok["k_bf_round"]
        steps = j["steps"]
        rows[name].append((j["ms_per_step"], 1e3 * sw["ms_per_step"] * steps / max(1, sw["launches"]),
                           1e3 * bf["ms_per_step"] * steps / max(1, bf["launches"]),
                           sw["launches"] / steps, bf["launches"] / steps))
    for name, r in rows.items():
        n = len(r)
        avg = [sum(x[i] for x in r) / n for i in range(5)]
        print(f"{name:40s} runs {n}  ms/step {avg[0]:7.2f}  sweep {avg[1]:6.2f} us x {avg[3]:6.0f}  "
              f"bf {avg[2]:6.2f} us x {avg[4]:6.0f}")


if __name__ == "__main__":
    main()
