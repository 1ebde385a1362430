#!/usr/bin/env python3
"""bench.py — MCMF solve latency and arcs/s on Quincy-shaped cell graphs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload full|incremental|batch]

* ``full`` (default, the headline line): config 3 (100k tasks × 10k machines),
  one full device re-solve per step. N > 1 runs under torch.distributed (one
  rank per GPU, RCCL): every rank solves its own independent cell graph
  (seed + rank), the north star's sharding of independent graphs; the task→PU
  mappings are gathered over RCCL after the timed region.
  ``value`` = Σ arcs over ranks ÷ max-rank time.
* ``incremental``: config 4 — the config-3 cell under churn (5% completions +
  5% arrivals per round, pins, ageing, capacity refresh); a step is one round:
  ks_apply_deltas + ks_solve + ks_get_task_mapping.
* ``batch``: config 5 — 64 independent config-2 graphs (seeds 1000..1063)
  round-robin over the ranks; each GPU solves its share as ONE device solve of
  their disjoint union (``--batch-mode union``, default) or as concurrent
  contexts (``--batch-mode streams``, ks_solve_many); a step solves every graph
  once. Mappings are gathered over RCCL afterwards.

Inputs are resident in HBM before timing (the first, untimed solve uploads).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from ksched_amd import batch, churn, gen, native  # noqa: E402

METRIC = "MCMF solve latency (ms) + arcs/s at 100k tasks x 10k machines, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (spec)
B_UNIT = 24             # bytes per residual-arc scan / node visit / push / relaxation
B_RELAX = 44            # Bellman-Ford in-arc relaxation as the kernel reads it: ucap, rcap, cost (8 each),
                        # head (4), gathered price and distance of the tail (8 each) — second field
# PMC traffic per workload: (FETCH_SIZE + WRITE_SIZE) per launch of each kernel,
# from rocprofv3 --pmc passes of the same workload (tools/gpu_pmc.sh); the newest
# file for the workload wins
PMC_DIR = os.path.join(ROOT, "profiles")


def pmc_file(workload: str):
    import glob
    cands = sorted(glob.glob(os.path.join(PMC_DIR, f"r*_pmc_{workload}.json")))
    if cands:
        return cands[-1]
    legacy = os.path.join(PMC_DIR, "r03m_pmc_traffic.json")   # round 3: config 3 only
    return legacy if workload == "config3" and os.path.exists(legacy) else None


# kinds of device work a solve reports (ks_result ABI 3): the kernel each one
# times, its launch count and time fields, its algorithmic units
KINDS = {
    "k_sweep": ("sweep_launches", "ms_sweep_kernels", ("arc_scans", "node_visits", "pushes")),
    # both hops of a round: the frontier's in-arcs and, for a task or PU whose distance
    # just dropped, its own in-arcs in the same launch (ks_result.gu_leaf_scans, ABI 5;
    # rounds 1-5 counted the first hop only — the line keeps that figure as *_first_hop)
    "k_bf_round": ("gu_launches", "ms_gu_kernels", ("gu_arc_scans", "gu_leaf_scans")),
    "k_fs_round": ("fs_launches", "ms_fs_kernels", ("fs_arc_scans",)),
    "k_cell": (None, "ms_cell_kernel", ("arc_scans", "node_visits", "pushes", "gu_arc_scans")),
}


def pct(xs, q):
    return round(float(np.percentile(np.asarray(xs, float), q)), 3) if len(xs) else None


def latency_stats(step_ms):
    """p50 / p95 / max of the timed steps (a scheduler's round budget is set by the max)."""
    if not step_ms:
        return None
    return {"p50_ms": pct(step_ms, 50), "p95_ms": pct(step_ms, 95), "max_ms": round(max(step_ms), 3),
            "min_ms": round(min(step_ms), 3), "max_over_median": round(max(step_ms) / float(np.median(step_ms)), 3)}


def roofline_of(results, workload: str):
    """HBM roofline of the dominant kernel (by device time) over the timed steps:
    algorithmic bytes = SURVEY §8(d)'s 24 B per unit × the device counters' units,
    divided by the measured duration of that kernel's launches (ks_result ABI 3):
    k_bf_round by HIP events on the engine's stream — each update's rounds
    bracketed exactly, the finish's batches less their parent-graph searches
    (timed by the device clock, s_memrealtime) — k_sweep by the device clock
    (the first sweep's start to k_cycle_end's: an event between two kernels
    would add a ~5.7 µs gap of its own), k_fs_round by HIP events.
    For k_bf_round the 44 B the relaxation actually reads is reported beside it;
    the forward search (k_fs_round) counts the residual out-arcs it examines.
    The cell solver (k_cell, one launch per solve) does all four kinds of work
    in one kernel: its units are all of them. ``traffic`` (PMC bytes per launch)
    cannot be collected inside this run (rocprofv3 --pmc is its own pass): it is
    read from the newest profile of the SAME workload, named in traffic_source."""
    n_res = max(1, len(results))
    kinds = {}
    for kname, (nkey, mskey, ukeys) in KINDS.items():
        rs = [r for r in results if (r.raw["solver"] == 1) == (kname == "k_cell")]
        ms = sum(r.raw[mskey] for r in rs)
        n = sum(r.raw[nkey] for r in rs) if nkey else sum(1 for r in rs if r.raw[mskey] > 0)
        units = sum(sum(r.raw[u] for u in ukeys) for r in rs)
        kinds[kname] = {"ms": ms, "launches": n, "units": units}
    kernel = max(kinds, key=lambda k: kinds[k]["ms"])
    ms, n, units = kinds[kernel]["ms"], kinds[kernel]["launches"], kinds[kernel]["units"]
    b = B_UNIT * units
    achieved = b / (ms / 1e3) / 1e9 if ms > 0 else 0.0
    line = {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
            "bytes_per_unit": B_UNIT, "units_per_launch": round(units / max(1, n), 1),
            "bytes_per_launch": round(b / max(1, n), 1), "avg_launch_us": round(1e3 * ms / max(1, n), 3),
            "launches": n, "kernel_ms_per_step": round(ms / n_res, 3),
            "kinds": {k: {"ms_per_step": round(v["ms"] / n_res, 3), "launches": v["launches"], "units": v["units"],
                          "avg_launch_us": round(1e3 * v["ms"] / max(1, v["launches"]), 3)}
                      for k, v in kinds.items() if v["ms"] > 0}}
    if kernel == "k_bf_round":
        a44 = B_RELAX * units / (ms / 1e3) / 1e9 if ms > 0 else 0.0
        line["achieved_44B"] = round(a44, 3)
        line["frac_44B"] = round(a44 / HBM_PEAK_GBS, 6)
        first = sum(r.raw["gu_arc_scans"] for r in results if r.raw["solver"] == 0)
        a1 = B_UNIT * first / (ms / 1e3) / 1e9 if ms > 0 else 0.0
        line["units_per_launch_first_hop"] = round(first / max(1, n), 1)
        line["achieved_first_hop"] = round(a1, 3)
        line["frac_first_hop"] = round(a1 / HBM_PEAK_GBS, 6)
    # SURVEY §8(d) solve-level figure: B_work = 24 B × (arc scans + node visits + pushes)
    # over the whole solve time (and with the Bellman-Ford relaxations added), and the
    # single-pass floor B_pass = 2m·16 + n·24 for scale
    sw_units = sum(r.raw["arc_scans"] + r.raw["node_visits"] + r.raw["pushes"] for r in results)
    bf_units = sum(r.raw["gu_arc_scans"] + r.raw["gu_leaf_scans"] for r in results)
    t_solve = sum(r.raw["ms"]["total"] for r in results) / 1e3
    if t_solve > 0:
        nn, mm = results[-1].raw["n_nodes"], results[-1].raw["n_arcs"]
        bw = B_UNIT * sw_units
        bwa = B_UNIT * (sw_units + bf_units)
        bp = 2 * mm * 16 + nn * 24
        line["solve_level"] = {
            "b_work_bytes": bw, "achieved": round(bw / t_solve / 1e9, 3),
            "frac": round(bw / t_solve / 1e9 / HBM_PEAK_GBS, 6),
            "b_work_with_bf_bytes": bwa, "achieved_with_bf": round(bwa / t_solve / 1e9, 3),
            "frac_with_bf": round(bwa / t_solve / 1e9 / HBM_PEAK_GBS, 6),
            "b_pass_bytes": bp, "b_pass_us_at_peak": round(bp / (HBM_PEAK_GBS * 1e9) * 1e6, 2),
            "note": "SURVEY 8(d): B_work / t_solve over all timed solves; b_pass = one read of the "
                    "residual graph, the floor any iterative solve sits above"}
    pf = pmc_file(workload)
    k = {}
    if pf:
        pmc = json.load(open(pf))
        k = pmc.get("kernels", {}).get(kernel, {})
        line["traffic"] = k.get("raw_bytes_per_launch")
        line["traffic_source"] = {"file": os.path.relpath(pf, ROOT), "date": pmc.get("date"),
                                  "workload": pmc.get("workload"),
                                  "calibrated_bytes_per_launch": k.get("calibrated_bytes_per_launch"),
                                  "atomics_per_launch": k.get("tcc_atomic_per_launch"),
                                  "note": pmc.get("note")}
    if kernel == "k_cell":
        # the cell solver's scans and relaxations are served by LDS and
        # L2, so 24 B per unit is not HBM traffic. Its HBM line is the PMC counter bytes
        # (FETCH_SIZE + WRITE_SIZE per launch) over this run's event-timed launch, and its
        # compute line the VALU issue rate of the same profile (2 wave64 VALU per CU-cycle).
        line["bytes_per_unit"] = None
        line["bytes_per_launch"] = None
        raw = k.get("raw_bytes_per_launch")
        t = ms / max(1, n) / 1e3
        if raw and t > 0:
            line["achieved"] = round(raw / t / 1e9, 3)
            line["frac"] = round(raw / t / 1e9 / HBM_PEAK_GBS, 6)
            line["bytes_source"] = "PMC counter bytes per launch (traffic_source)"
        else:
            line["achieved"], line["frac"] = None, None
        if k.get("valu"):
            line["valu"] = k["valu"]
    return line


GOLDEN_FILE = os.path.join(ROOT, "tests", "golden", "goldens.json")


def golden_of(T, M, R, J, seed):
    """(cost, flow) of a committed golden (networkx network_simplex, generated in the
    build container by tests/golden/gen_goldens.py), or None."""
    if not os.path.exists(GOLDEN_FILE):
        return None
    for e in json.load(open(GOLDEN_FILE))["graphs"]:
        if e.get("family") == "quincy" and list(e.get("params", [])) == [T, M, R, J] and e.get("seed") == seed:
            return int(e["cost"]), int(e["flow"])
    return None


class ParityError(RuntimeError):
    pass


def timed_cpu(fn, reps: int = 5, warmup: int = 1, pin: bool = True):
    """BASELINE.md §3-4 protocol for a CPU baseline: `warmup` untimed runs, then the
    median of `reps` timed runs, the calling thread pinned to one core (taskset-like,
    os.sched_setaffinity) when `pin`. → (median seconds, all times, last result, core)."""
    core = None
    old = None
    if pin and hasattr(os, "sched_setaffinity"):
        old = os.sched_getaffinity(0)
        core = min(old)
        os.sched_setaffinity(0, {core})
    try:
        out = None
        for _ in range(warmup):
            out = fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            out = fn()
            ts.append(time.perf_counter() - t0)
    finally:
        if old is not None:
            os.sched_setaffinity(0, old)
    return float(np.median(ts)), ts, out, core


def host_cores() -> int:
    """Cores this process may use (the GPU box exposes the whole machine's CPUs but
    grants a share: OMP_NUM_THREADS is set to it there)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(env))) if env and env.isdigit() else n


class Dist:
    """torch.distributed over RCCL when launched with WORLD_SIZE > 1.

    KS_BENCH_REHEARSAL=1 (tests only): gloo collectives on host copies and every
    rank on GPU 0, so the N > 1 code path runs on a one-GPU box."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.rehearsal = os.environ.get("KS_BENCH_REHEARSAL") == "1"
        self.dist = self.torch = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            if self.rehearsal:
                self.local = 0
                torch.cuda.set_device(0)
                dist.init_process_group("gloo")
            else:
                torch.cuda.set_device(self.local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            self.dist, self.torch = dist, torch

    def sync(self):
        if self.dist:
            self.torch.cuda.synchronize()
            self.dist.barrier()

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device="cpu" if self.rehearsal else "cuda")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, block, num_graphs: int):
        """RCCL all-gather of a device block (rehearsal: gloo on a host copy)."""
        if self.rehearsal:
            return batch.gather(block.cpu(), num_graphs, self.dist)
        return batch.gather(block, num_graphs, self.dist)

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def opts_of(args) -> dict:
    """ks_opts for the bench's contexts: the flags below, plus --opt key=value (any
    ks_opts field; also KS_BENCH_OPTS="key:value+key:value" for A/B scripts)."""
    o = {}
    pairs = list(args.opt or [])
    env = os.environ.get("KS_BENCH_OPTS")
    if env:
        pairs += [p.replace(":", "=") for p in env.split("+") if p]
    for kv in pairs:
        k, v = kv.split("=", 1)
        o[k.strip()] = int(v)
    if args.alpha:
        o["alpha"] = args.alpha
    if args.gu_interval:
        o["gu_interval"] = args.gu_interval
    if args.price_refine >= 0:
        o["price_refine"] = args.price_refine
    return o


def full_opts(args) -> dict:
    """Every timed full-workload step is a from-scratch solve: no warm start."""
    return dict(opts_of(args), warm_start=0)


def base_line(args, D, value, ms_per_step, config, **extra):
    line = {"metric": METRIC, "value": round(value, 1), "unit": "arcs/s", "n_gpus": D.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64", "data": "synthetic", "config": config}
    line.update(extra)
    return line


# --------------------------------------------------------------------- full
def run_full(args, D):
    T, M, R, J, seed = gen.CONFIGS[args.config]
    g = gen.quincy(T, M, R, J, seed + D.rank)
    ctx = native.Context(D.local, **full_opts(args))
    ctx.load_graph(g)
    import torch
    dev_map = torch.zeros(T, dtype=torch.int64, device=f"cuda:{D.local}") if torch.cuda.is_available() else None

    def step():
        # Solve() → TaskMapping (placement/solver.go:60-90, 183-269): the device solve
        # and the device-side decomposition into the task→PU vector (stays in HBM)
        r = ctx.solve()
        if dev_map is not None:
            ctx.task_pu_device(dev_map.data_ptr(), T)
        return r

    for _ in range(args.warmup):
        step()
    D.sync()
    t0 = time.perf_counter()
    results, step_ms = [], []
    for _ in range(args.steps):
        ts = time.perf_counter()
        results.append(step())
        step_ms.append(1e3 * (time.perf_counter() - ts))
    D.sync()
    elapsed = D.max(time.perf_counter() - t0)
    ms_per_step = 1e3 * elapsed / max(1, args.steps)
    value = D.world * g.m / (ms_per_step / 1e3)

    gather = None
    if D.dist:       # RCCL gather of the task→PU mappings (int64 PU id per task, 0 = unscheduled)
        buf = dev_map.view(1, T)
        tg0 = time.perf_counter()
        out = D.gather(buf, D.world)
        torch.cuda.synchronize()
        gather = {"ms": 1e3 * (time.perf_counter() - tg0), "bytes_per_rank": T * 8,
                  "scheduled": int((out > 0).sum().item())}

    costs = sorted({r.cost for r in results})
    flows = sorted({r.flow for r in results})
    cpu = None
    parity = {"gpu_costs": costs, "flow": results[-1].flow, "steps_checked": len(results)}
    problems = []
    if len(costs) != 1:
        problems.append(f"timed solves disagree on the cost: {costs}")
    if flows != [T]:
        problems.append(f"flow value {flows} != {T} tasks")
    gold = golden_of(T, M, R, J, seed + D.rank)
    if gold is not None:
        parity["golden"] = {"cost": gold[0], "flow": gold[1], "source": "tests/golden/goldens.json"}
        if costs != [gold[0]] or flows != [gold[1]]:
            problems.append(f"cost/flow {costs}/{flows} != golden {gold}")
    if D.rank == 0 and D.world == 1 and args.cpu_baseline == "auto":
        from oracle import ko
        med, ts, out, core = timed_cpu(lambda: ko.reference_path(g), reps=args.cpu_reps)
        st, ccost, cflow, nmap, ms = out
        med2, ts2, out2, _ = timed_cpu(lambda: ko.cost_scaling(g), reps=args.cpu_reps)
        st2, cs_cost, cs_flow, _ = out2
        cpu = {"value": round(g.m / med, 1), "unit": "arcs/s", "cores": 1, "kind": "port",
               "sample": f"the same {args.config} graph through the in-repo restatement of the reference CPU path "
                         f"(DIMACS export -> successive shortest path -> f lines -> BFS mapping), median of "
                         f"{len(ts)} after 1 warm-up, pinned to core {core}",
               "ms": round(1e3 * med, 1), "times_ms": [round(1e3 * x, 1) for x in ts], "median_of": len(ts),
               "pinned_core": core, "phases_ms": [round(x, 1) for x in ms],
               "strong_cpu_cost_scaling": {"value": round(g.m / med2, 1), "unit": "arcs/s", "ms": round(1e3 * med2, 1),
                                           "median_of": len(ts2), "cores": 1}}
        parity.update({"cpu_cost": ccost, "cpu_flow": cflow, "cs_cost": cs_cost})
        if not (costs == [ccost] == [cs_cost] and flows == [cflow] and st == 0 and st2 == 0):
            problems.append(f"GPU {costs}/{flows} vs CPU SSP {ccost}/{cflow} and cost scaling {cs_cost}")
    parity["match"] = not problems
    if problems:
        parity["problems"] = problems
    config = {"workload": f"{args.config}: Quincy-shaped cell graph T={T} M={M} R={R} J={J} "
                          f"(n={g.n}, m={g.m}), step = full device re-solve + device task->PU extraction "
                          f"(Solve() -> TaskMapping), one graph per GPU",
              "tasks": T, "machines": M, "racks": R, "jobs": J, "seed": seed, "n": g.n, "m": g.m,
              "parallelism": f"independent graphs x{D.world}"}
    line = base_line(args, D, value, ms_per_step, config, step_ms=[round(x, 2) for x in step_ms],
                     roofline=roofline_of(results, args.config), cpu_baseline=cpu, parity=parity, gather=gather,
                     latency=latency_stats(step_ms), solve=dict(results[-1].raw))
    ctx.close()
    return line


# -------------------------------------------------------------- incremental
def run_incremental(args, D):
    """Config 4: the config-3 cell solved, then `steps` timed
    churn rounds after `warmup` untimed ones. A round = ks_apply_deltas (in HBM)
    + ks_solve + the task mapping. Rank 0 at N = 1 replays the same rounds through
    the CPU restatement of the reference's incremental mode (the change block as
    text, Flowlessly-style incremental SSP from the previous round's flow and
    potentials, f lines, BFS mapping), with the cold SSP reference path beside it,
    and checks every round's cost and flow against it (outside the timed region)."""
    T, M, R, J, seed = gen.CONFIGS["config3"]
    cell = churn.Cell(T, M, R, J, seed + D.rank)
    # --warm unset: the library's default re-solve mode (from scratch, warm_start 0:
    # the lower worst round in the round-5 interleaved A/B)
    wopt = {} if args.warm is None else {"warm_start": args.warm}
    ctx = native.Context(D.local, **dict(opts_of(args), **wopt))
    g = cell.graph()
    ctx.load_graph(g)
    r0 = ctx.solve()
    mp = ctx.task_mapping_arrays()
    done = arrive = T // 20
    rounds, results = [], []
    t_total = 0.0
    problems = []
    cpu_on = D.rank == 0 and D.world == 1 and args.cpu_baseline == "auto"
    inc = cold_ms = inc_ms = None
    if cpu_on:
        from oracle import ko
        inc = ko.IncrementalSSP()
        t0 = time.perf_counter()
        st, c, f, _ = inc.round(g)                      # the daemon's first (full) solve
        inc_first_ms = 1e3 * (time.perf_counter() - t0)
        if (c, f) != (r0.cost, r0.flow):
            problems.append(f"initial solve: GPU {r0.cost}/{r0.flow} vs CPU {c}/{f}")
        cold_ms, inc_ms, cs_ms = [], [], []
    for i in range(args.warmup + args.steps):
        d = cell.step(mp, done=done, arrive=arrive)
        fresh = list(cell.last_arrived_ids)
        D.sync()
        ts = time.perf_counter()
        ctx.apply_deltas(d)
        ta = time.perf_counter()
        r = ctx.solve()
        tb = time.perf_counter()
        mp = ctx.task_mapping_arrays()   # ks_get_task_mapping's (task, PU) arrays: the TaskMapping
        te = time.perf_counter()
        D.sync()
        dt = D.max(time.perf_counter() - ts)
        sst = ctx.store_stats()
        rec = {"round": i + 1, "timed": i >= args.warmup, "deltas": int(d.shape[0]), "ms": round(1e3 * dt, 3),
               "apply_ms": round(1e3 * (ta - ts), 3), "solve_ms": round(1e3 * (tb - ta), 3),
               "mapping_ms": round(1e3 * (te - tb), 3), "cost": r.cost, "flow": r.flow,
               "warm": r.raw["warm_started"], "phases": r.raw["phases"], "sweeps": r.raw["sweeps"],
               "updates": r.raw["global_updates"], "bf_rounds": r.raw["gu_iterations"],
               "recoveries": r.raw["recoveries"],
               "solve_parts_ms": {k: round(v, 2) for k, v in r.raw["ms"].items()},
               "m": r.raw["n_arcs"], "running": int((cell.state == cell.RUN).sum()),
               "rebuilt": r.raw["rebuilt"], "rebuilds_since_load": sst["rebuilds"],
               "store": {k: sst[k] for k in ("inserted", "updated", "killed", "superseded")}}
        if r.flow != cell.graph().supply[cell.graph().supply > 0].sum():
            problems.append(f"round {i + 1}: flow {r.flow} short of the supply")
        if cpu_on:
            g = cell.graph()
            t0 = time.perf_counter()
            st, c, f, _ = inc.round(g, d, fresh)
            inc_ms.append(1e3 * (time.perf_counter() - t0))
            t0 = time.perf_counter()
            st2, c2, f2, _, _ = ko.reference_path(g)
            cold_ms.append(1e3 * (time.perf_counter() - t0))
            t0 = time.perf_counter()
            st3, c3, f3, _ = ko.cost_scaling(g)
            cs_ms.append(1e3 * (time.perf_counter() - t0))
            rec["cpu"] = {"incremental_ms": round(inc_ms[-1], 1), "cold_ms": round(cold_ms[-1], 1),
                          "cost_scaling_ms": round(cs_ms[-1], 1), "cost": c,
                          "incremental_phases_ms": {k: round(v, 1) for k, v in inc.last["ms"].items()}}
            if not ((r.cost, r.flow) == (c, f) == (c2, f2) == (c3, f3) and st == st2 == st3 == 0):
                problems.append(f"round {i + 1}: GPU {r.cost}/{r.flow} vs CPU incremental {c}/{f}, cold {c2}/{f2}, "
                                f"cost scaling {c3}/{f3}")
        if i >= args.warmup:
            t_total += dt
            results.append(r)
        rounds.append(rec)
    ms_per_step = 1e3 * t_total / max(1, args.steps)
    m_avg = sum(r.raw["n_arcs"] for r in results) / max(1, len(results))
    value = D.world * m_avg / (ms_per_step / 1e3)
    timed = [x for x in rounds if x["timed"]]
    parity = {"rounds_checked": len(rounds) if cpu_on else 0, "flows_checked": len(rounds),
              "match": not problems, "last_round_gpu_cost": rounds[-1]["cost"]}
    if problems:
        parity["problems"] = problems
    cpu = None
    if cpu_on:
        ti = [x for x, rr in zip(inc_ms, rounds) if rr["timed"]]
        tc = [x for x, rr in zip(cold_ms, rounds) if rr["timed"]]
        ts3 = [x for x, rr in zip(cs_ms, rounds) if rr["timed"]]
        med_i, med_c, med_s = float(np.median(ti)), float(np.median(tc)), float(np.median(ts3))
        inc_leg = {"value": round(m_avg / (med_i / 1e3), 1), "unit": "arcs/s", "ms": round(med_i, 1),
                   "times_ms": [round(x, 1) for x in ti], "first_full_solve_ms": round(inc_first_ms, 1), "cores": 1,
                   "sample": "the restatement of the reference's incremental mode (ExportIncremental text -> parse "
                             "-> incremental SSP from the previous round's flow and potentials -> f lines -> BFS "
                             "mapping; Flowlessly daemon, solver.go:30-34,86-89), median per round"}
        cold_leg = {"value": round(m_avg / (med_c / 1e3), 1), "unit": "arcs/s", "ms": round(med_c, 1),
                    "times_ms": [round(x, 1) for x in tc], "cores": 1,
                    "sample": "each timed round's full graph through the cold reference path (export -> SSP -> "
                              "f lines -> BFS), median"}
        # headline: the FASTER of the two reference-path restatements
        head, other, oname = (inc_leg, cold_leg, "cold_reference_path") if med_i <= med_c else \
            (cold_leg, inc_leg, "incremental_reference_path")
        cpu = {"value": head["value"], "unit": "arcs/s", "cores": 1, "kind": "port",
               "sample": f"the same {len(ti)} timed rounds, the faster of two restatements of the reference CPU "
                         f"path: " + head["sample"] + ", 1 thread",
               "ms": head["ms"], "times_ms": head["times_ms"], oname: other,
               "strong_cpu_cost_scaling": {"value": round(m_avg / (med_s / 1e3), 1), "unit": "arcs/s",
                                           "ms": round(med_s, 1), "times_ms": [round(x, 1) for x in ts3],
                                           "cores": 1, "sample": "each timed round's full graph through the "
                                                                 "in-repo single-threaded cost-scaling oracle"}}
    config = {"workload": f"config4: config-3 cell (T={T} M={M}) under churn, {done} completions + "
                          f"{arrive} arrivals per round, pins/ageing/capacity deltas; step = apply deltas + "
                          f"{'warm-started' if any(x['warm'] for x in timed) else 'from-scratch'} re-solve + mapping; {args.steps} timed "
                          f"rounds after {args.warmup}", "tasks": T, "machines": M, "seed": seed,
              "initial_solve_ms": round(r0.raw["ms"]["total"], 3), "rounds": args.steps,
              "round_ms": {"median": round(float(np.median([x["ms"] for x in timed])), 3),
                           "max": round(max(x["ms"] for x in timed), 3)},
              "parallelism": f"independent cells x{D.world}"}
    line = base_line(args, D, value, ms_per_step, config, rounds=rounds, roofline=roofline_of(results, "config4"),
                     latency=latency_stats([x["ms"] for x in timed]),
                     cpu_baseline=cpu, parity=parity)
    ctx.close()
    return line


# -------------------------------------------------------------------- batch
def run_batch(args, D):
    T, M, R, J, _ = gen.CONFIGS["config2"]
    num = args.graphs
    mine = batch.assign(num, D.world, D.rank)
    if D.rehearsal and args.batch_mode == "abi":
        args.batch_mode = "union"    # both ranks on GPU 0: RCCL refuses two ranks per device
    if args.batch_mode == "abi":
        # the C-ABI batch (ks_batch_*): every rank passes all graphs, owns g ≡ rank (mod world),
        # solves the union of its graphs; per-graph rows to rank 0 over RCCL inside libksmcmf
        all_graphs = [gen.quincy(T, M, R, J, 1000 + k) for k in range(num)]
        graphs = [all_graphs[k] for k in mine]
        if D.world > 1:
            uid = [native.Batch.unique_id() if D.rank == 0 else None]
            D.dist.broadcast_object_list(uid, src=0)
            bt = native.Batch(device=D.local, world=D.world, rank=D.rank, uid=uid[0], **full_opts(args))
        else:
            bt = native.Batch(devices=[D.local], **full_opts(args))
        bt.load(all_graphs)
        solve = bt.solve
    elif args.batch_mode == "union":
        graphs = [gen.quincy(T, M, R, J, 1000 + k) for k in mine]
        u, noff, _ = batch.union(graphs)
        ctxs = [native.Context(D.local, **full_opts(args))]
        ctxs[0].load_graph(u)
        solve = lambda: [ctxs[0].solve()]
    else:
        graphs = [gen.quincy(T, M, R, J, 1000 + k) for k in mine]
        ctxs = [native.Context(D.local, **full_opts(args)) for _ in graphs]
        for c, g in zip(ctxs, graphs):
            c.load_graph(g)
        solve = lambda: native.solve_many(ctxs, workers=args.workers)
    for _ in range(args.warmup):
        solve()
    D.sync()
    t0 = time.perf_counter()
    results = []
    step_ms = []
    for _ in range(args.steps):
        ts = time.perf_counter()
        results.extend(solve())
        step_ms.append(1e3 * (time.perf_counter() - ts))
    D.sync()
    elapsed = D.max(time.perf_counter() - t0)
    ms_per_step = 1e3 * elapsed / max(1, args.steps)
    arcs_all = num * gen.quincy_sizes(T, M, R, J)[1]
    value = arcs_all / (ms_per_step / 1e3)

    # after the timed region: per-graph cost/flow and task→PU rows gathered to rank 0
    gather = None
    per_graph = None
    if args.batch_mode == "abi":
        tg0 = time.perf_counter()
        pu, cost, flow = bt.gather(T, root=D.rank == 0)
        gather = {"ms": round(1e3 * (time.perf_counter() - tg0), 3), "via": ("RCCL ncclSend/ncclRecv in libksmcmf" if D.world > 1
                                                                   else "none (world 1: rank 0's own rows, no RCCL call)"),
                  "bytes_per_rank": batch.slots_per_rank(num, D.world) * (T + 2) * 8}
        if D.rank == 0:
            per_graph = cost
            gather.update({"graphs": int(pu.shape[0]), "scheduled": int((pu > 0).sum()),
                           "flow_total": int(flow.sum())})
    else:
        import torch
        if torch.cuda.is_available():
            slots = batch.slots_per_rank(num, D.world)
            buf = torch.zeros(slots, T, dtype=torch.int64, device=f"cuda:{D.local}")
            tg0 = time.perf_counter()
            if args.batch_mode == "union":
                ctxs[0].task_pu_device(buf.data_ptr(), len(mine) * T)
                off = torch.as_tensor(noff[:len(mine)], device=buf.device).view(-1, 1)
                part = buf[:len(mine)]
                part.sub_(torch.where(part > 0, off, torch.zeros_like(off)))
            else:
                for i, c in enumerate(ctxs):
                    c.task_pu_device(buf[i].data_ptr(), T)
            full = D.gather(buf, num) if D.dist else buf[:num]
            torch.cuda.synchronize()
            gather = {"ms": round(1e3 * (time.perf_counter() - tg0), 3), "bytes_per_rank": slots * T * 8,
                      "graphs": int(full.shape[0]), "scheduled": int((full > 0).sum().item())}
        if args.batch_mode == "union":
            per_graph = batch.split_costs(u, noff, ctxs[0].flows())
        else:
            per_graph = np.asarray([r.cost for r in results[-len(ctxs):]], np.int64)
    cpu = None
    parity = {"total_cost": int(per_graph.sum()) if per_graph is not None else None}
    if args.batch_mode == "streams":   # per-cell solve latency (each context's own solve)
        cell_ms = [r.raw["ms"]["total"] for r in results[-len(ctxs):]]
        extra_cells = {"median_ms": round(float(np.median(cell_ms)), 3), "max_ms": round(max(cell_ms), 3),
                       "min_ms": round(min(cell_ms), 3), "cells": len(cell_ms),
                       "note": "host wall time of each context's ks_solve while the cells ran concurrently"}
    else:
        extra_cells = None
    if D.rank == 0 and D.world == 1 and args.cpu_baseline == "auto":
        from concurrent.futures import ThreadPoolExecutor
        from oracle import ko
        cores = host_cores()
        every = [gen.quincy(T, M, R, J, 1000 + k) for k in range(num)]

        def all_graphs_cpu():
            with ThreadPoolExecutor(cores) as ex:
                return list(ex.map(ko.reference_path, every))
        med, ts, outs, _ = timed_cpu(all_graphs_cpu, reps=args.cpu_reps, pin=False)

        def all_graphs_cs():
            with ThreadPoolExecutor(cores) as ex:
                return list(ex.map(ko.cost_scaling, every))
        med_s, ts_s, outs_s, _ = timed_cpu(all_graphs_cs, reps=args.cpu_reps, pin=False)
        m2 = gen.quincy_sizes(T, M, R, J)[1]
        cpu = {"value": round(num * m2 / med, 1), "unit": "arcs/s", "cores": cores, "kind": "port",
               "sample": f"all {num} graphs through the restatement of the reference CPU path (export -> SSP -> "
                         f"f lines -> BFS), one graph per thread on {cores} threads (the host cores this process "
                         f"may use), median of {len(ts)} after 1 warm-up",
               "ms": round(1e3 * med, 1), "times_ms": [round(1e3 * x, 1) for x in ts], "median_of": len(ts),
               "strong_cpu_cost_scaling": {"value": round(num * m2 / med_s, 1), "unit": "arcs/s", "cores": cores,
                                           "ms": round(1e3 * med_s, 1), "times_ms": [round(1e3 * x, 1) for x in ts_s],
                                           "median_of": len(ts_s),
                                           "sample": f"all {num} graphs through the in-repo cost-scaling oracle, one "
                                                     f"graph per thread on {cores} threads"}}
        parity.update({"checked_graphs": num,
                       "match": bool(per_graph is not None and all(o[1] == int(c) == s[1] for o, c, s in
                                                                   zip(outs, per_graph, outs_s)))})
        if not parity["match"]:
            parity["problems"] = ["a graph's GPU cost differs from the CPU reference path"]
    mode = {"abi": "C-ABI batch (union per device, RCCL gather inside libksmcmf)",
            "union": "one device solve of their disjoint union",
            "streams": f"one context each, solved concurrently ({args.workers} workers/GPU)"}[args.batch_mode]
    config = {"workload": f"config5: {num} independent config-2 graphs (T={T} M={M}, seeds 1000..{999 + num}) "
                          f"round-robin over {D.world} GPU(s), {mode}; step = every graph solved once",
              "graphs": num, "tasks": T, "machines": M, "graphs_per_gpu": len(mine), "mode": args.batch_mode,
              "parallelism": f"graph sharding x{D.world}"}
    line = base_line(args, D, value, ms_per_step, config, step_ms=[round(x, 2) for x in step_ms],
                     scaling="strong",   # a fixed 64 graphs shared by the ranks
                     roofline=roofline_of(results, "config5"), cpu_baseline=cpu, gather=gather, parity=parity,
                     latency=latency_stats(step_ms), cell_latency=extra_cells, solve=dict(results[-1].raw))
    if args.batch_mode == "abi":
        bt.close()
    else:
        for c in ctxs:
            c.close()
    return line


def main():
    # stdout carries exactly one JSON line (rank 0): anything else a library prints
    # there (RCCL's version banner at communicator init) goes to stderr instead
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 5; incremental: 10 rounds)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 2; incremental: 1)")
    ap.add_argument("--workload", default="full", choices=["full", "incremental", "batch"])
    ap.add_argument("--config", default="config3", choices=sorted(gen.CONFIGS))
    ap.add_argument("--graphs", type=int, default=64)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--batch-mode", default="abi", choices=["abi", "union", "streams"])
    ap.add_argument("--warm", type=int, default=None,
                    help="incremental workload: ks_opts.warm_start of the re-solves (default: the library's)")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-reps", type=int, default=5, help="CPU baseline: median of this many after 1 warm-up")
    ap.add_argument("--alpha", type=int, default=0)
    ap.add_argument("--gu-interval", type=int, default=0)
    ap.add_argument("--price-refine", type=int, default=-1)
    ap.add_argument("--opt", action="append", help="ks_opts field=value (repeatable)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 10 if args.workload == "incremental" else 5    # config 4 is 10 rounds
    if args.warmup is None:
        args.warmup = 1 if args.workload == "incremental" else 2

    D = Dist()
    run = {"full": run_full, "incremental": run_incremental, "batch": run_batch}[args.workload]
    line = run(args, D)
    # the exit status doubles as a correctness gate: any rank whose solves disagree
    # with the golden / CPU reference / each other fails the run (after the line)
    ok = bool((line.get("parity") or {}).get("match", True))
    bad = D.max(0.0 if ok else 1.0) > 0
    if D.rank == 0:
        print(json.dumps(line), file=json_out, flush=True)
    D.close()
    if bad:
        print("bench.py: PARITY FAILURE: " + json.dumps((line.get("parity") or {}).get("problems")), file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
