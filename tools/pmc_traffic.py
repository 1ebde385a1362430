#!/usr/bin/env python3
"""Build profiles/<tag>_pmc_traffic.json from gpu_pmc.sh's passes and the
calibration run (gpu_calib.sh): per kernel, raw FETCH_SIZE + WRITE_SIZE bytes
per launch, the calibrated range, and atomic request counts / rates.

    python tools/pmc_traffic.py gpurun_out/<pmc tag> gpurun_out/<calib tag>|<profile.json> DATE > profiles/<tag>_pmc_<workload>.json

The workload (config2..config5) is the one gpu_pmc.sh profiled (its workload.txt).
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_per_kernel  # noqa: E402


def per_kernel(dirs):
    import io
    from contextlib import redirect_stdout
    buf = io.StringIO()
    argv = sys.argv
    sys.argv = ["x"] + dirs
    with redirect_stdout(buf):
        pmc_per_kernel.main()
    sys.argv = argv
    return json.loads(buf.getvalue())


def main():
    pmc, cal, date = sys.argv[1], sys.argv[2], sys.argv[3]
    k = per_kernel([os.path.join(pmc, p) for p in ("fetch", "write", "atom", "ta", "valu") if os.path.isdir(os.path.join(pmc, p))])
    if cal.endswith(".json"):   # a committed profile's calibration (the calibration is a one-off)
        calib = json.load(open(cal))["calibration"]
    else:
        c = per_kernel([os.path.join(cal, "pmc_FETCH_SIZE"), os.path.join(cal, "pmc_WRITE_SIZE")])
        known = json.load(open(os.path.join(cal, "calib_FETCH_SIZE.json")))
        calib = {
            "stream8_fetch_per_byte": c["k_stream8"]["FETCH_SIZE"] * 1024 / known["k_stream8"],
            "stream4_fetch_per_byte": c["k_stream4"]["FETCH_SIZE"] * 1024 / known["k_stream4"],
            "gather8_fetch_bytes_per_load": c["k_gather8"]["FETCH_SIZE"] * 1024 / known["k_gather8_loads"],
            "store8_write_per_byte": c["k_store8"]["WRITE_SIZE"] * 1024 / known["k_store8"],
            "atomic8_write_bytes_per_op": c["k_atomic8"]["WRITE_SIZE"] * 1024 / known["k_atomic8_ops"],
        }
    times = {}
    stats = os.path.join(pmc, "kernel_stats.csv")
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            name = r.get("kernel") or r.get("Name") or ""
            for key in ("k_sweep", "k_bf_round", "k_saturate", "k_fs_round", "k_cell"):
                if key + "<" in name or key + "(" in name or name.endswith(key):
                    times.setdefault(key, {"calls": 0, "total_us": 0.0})
                    times[key]["calls"] += int(float(r.get("calls", 0)))
                    times[key]["total_us"] += float(r.get("total_us", 0.0))
    wl_path = os.path.join(pmc, "workload.txt")
    wl = open(wl_path).read().strip() if os.path.exists(wl_path) else "config3"
    desc = {"config3": "config 3 (bench.py --steps 1 --warmup 0): one full solve",
            "config2": "config 2 (bench.py --config config2 --steps 3 --warmup 0): three full solves",
            "config4": "config 4 (bench.py --workload incremental --steps 3 --warmup 0): initial solve + 3 churn rounds",
            "config5": "config 5 (bench.py --workload batch --steps 1 --warmup 0): warm-up + one batch solve"}[wl]
    out = {"date": date, "workload": desc, "workload_key": wl,
           "note": "raw = (FETCH_SIZE + WRITE_SIZE) per launch from separate rocprofv3 --pmc passes; gfx950 "
                   "FETCH_SIZE tallies coalesced 4/8-B streams at 1/2 of their bytes and a random 8-B gather at "
                   "64 B (tools/calib/calib_fetch.hip), so the calibrated range is [raw, 2*FETCH + WRITE]; "
                   "WRITE_SIZE counts 32 B per 8-B atomic",
           "calibration": {kk: round(v, 4) for kk, v in calib.items()}, "kernels": {}}
    merged = {}
    for name, v in k.items():
        base = "k_bf_round" if name.startswith("k_bf_round") else name
        m = merged.setdefault(base, {"dispatches": 0, "FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0, "TCC_ATOMIC_sum": 0.0,
                                     "TCC_EA0_ATOMIC_sum": 0.0, "TA_FLAT_ATOMIC_WAVEFRONTS_sum": 0.0})
        m["dispatches"] += int(v.get("dispatches", 0))
        for ckey in ("FETCH_SIZE", "WRITE_SIZE", "TCC_ATOMIC_sum", "TCC_EA0_ATOMIC_sum",
                     "TA_FLAT_ATOMIC_WAVEFRONTS_sum"):
            m[ckey] += float(v.get(ckey, 0.0))
            m[ckey + "_n"] = m.get(ckey + "_n", 0) + int(v.get(ckey + "_dispatches", 0))
    for name, m in merged.items():
        per = {c: m[c] / max(1, m.get(c + "_n", 0)) for c in ("FETCH_SIZE", "WRITE_SIZE", "TCC_ATOMIC_sum",
                                                              "TCC_EA0_ATOMIC_sum", "TA_FLAT_ATOMIC_WAVEFRONTS_sum")}
        fetch, write = per["FETCH_SIZE"] * 1024, per["WRITE_SIZE"] * 1024
        rec = {"dispatches_per_pass": {c: m.get(c + "_n", 0) for c in ("FETCH_SIZE", "WRITE_SIZE", "TCC_ATOMIC_sum",
                                                                       "TA_FLAT_ATOMIC_WAVEFRONTS_sum")},
               "raw_fetch_bytes_per_launch": round(fetch, 1), "raw_write_bytes_per_launch": round(write, 1),
               "raw_bytes_per_launch": round(fetch + write, 1),
               "calibrated_bytes_per_launch": [round(fetch + write, 1), round(2 * fetch + write, 1)],
               "tcc_atomic_per_launch": round(per["TCC_ATOMIC_sum"], 1),
               "ea_atomic_per_launch": round(per["TCC_EA0_ATOMIC_sum"], 1),
               "ta_flat_atomic_wavefronts_per_launch": round(per["TA_FLAT_ATOMIC_WAVEFRONTS_sum"], 1)}
        src = k.get(name, {})
        if src.get("SQ_INSTS_VALU") is not None and src.get("SQ_BUSY_CU_CYCLES"):
            nv = max(1, int(src.get("SQ_INSTS_VALU_dispatches", 1)))
            ipc = src["SQ_INSTS_VALU"] / src["SQ_BUSY_CU_CYCLES"]
            rec["valu"] = {"insts_per_launch": round(src["SQ_INSTS_VALU"] / nv, 1),
                           "busy_cu_cycles_per_launch": round(src["SQ_BUSY_CU_CYCLES"] / nv, 1),
                           "valu_per_cu_cycle": round(ipc, 4),
                           "peak_per_cu_cycle": 2.0,
                           "frac": round(ipc / 2.0, 4),
                           "note": "SQ_INSTS_VALU (wave64 VALU instructions) / SQ_BUSY_CU_CYCLES (cycles the CUs "
                                   "running the kernel were busy, summed over CUs); a CDNA4 CU issues at most 2 "
                                   "wave64 VALU per cycle (4 SIMD-32, a wave64 instruction over 2 cycles; "
                                   "MI355X_MICROARCH.md)"}
        t = times.get(name)
        if t and t["total_us"] > 0:
            rec["device_us_total"] = round(t["total_us"], 1)
            rec["trace_calls"] = t["calls"]
            rec["avg_launch_us"] = round(t["total_us"] / max(1, t["calls"]), 3)
            if rec.get("valu"):
                # CU utilisation: busy CU-cycles over all 256 CUs'
                # cycles while the kernel runs, at the 2.4 GHz peak engine clock (a lower
                # bound if the clock ran lower); GRBM_GUI_ACTIVE as measured, for reference
                busy = rec["valu"]["busy_cu_cycles_per_launch"]
                rec["valu"]["cu_busy_frac_at_peak_clock"] = round(busy / (256 * rec["avg_launch_us"] * 2400.0), 4)
                if src.get("GRBM_GUI_ACTIVE"):
                    rec["valu"]["grbm_gui_active_per_launch"] = round(src["GRBM_GUI_ACTIVE"] / nv, 1)
            # 64-bit atomics per second while the kernel runs: per-launch requests ÷ mean launch time
            rec["tcc_atomics_per_s"] = round(per["TCC_ATOMIC_sum"] / (rec["avg_launch_us"] / 1e6), 1)
        out["kernels"][name] = rec
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
