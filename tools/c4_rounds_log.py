#!/usr/bin/env python3
"""Config-4 rounds with the cycle log on (stderr → FILE): per round, the solve
time and the cycle kinds per phase. python tools/c4_rounds_log.py FILE [rounds]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ksched_amd import churn, gen, native  # noqa: E402

log = sys.argv[1]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
fd = os.open(log, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
os.dup2(fd, 2)
T, M, R, J, seed = gen.CONFIGS["config3"]
cell = churn.Cell(T, M, R, J, seed)
ctx = native.Context(0, log_cycles=1)
ctx.load_graph(cell.graph())
ctx.solve()
mp = ctx.task_mapping_arrays()
for i in range(rounds):
    ctx.apply_deltas(cell.step(mp, done=T // 20, arrive=T // 20))
    print(f"=== round {i + 1}", file=sys.stderr, flush=True)
    r = ctx.solve()
    print(f"=== round {i + 1} solve_ms {r.raw['ms']['total']:.2f} sweeps {r.raw['sweeps']}", file=sys.stderr, flush=True)
    print(f"round {i + 1} {r.raw['ms']['total']:.2f} ms sweeps {r.raw['sweeps']}", flush=True)
    mp = ctx.task_mapping_arrays()
