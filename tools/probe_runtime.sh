#!/bin/bash
# Which HIP runtime libksmcmf binds to, and the full-solve latency under each:
# torch imported first (shared torch runtime) vs the library alone (/opt/rocm).
set -o pipefail
OUT=gpurun_out/${1:-rt}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u - > "$OUT/probe.log" 2>&1 <<'EOF' || { echo probe failed; tail -30 "$OUT/probe.log"; exit 1; }
import os, sys
sys.path.insert(0, os.getcwd())
from ksched_amd import native, gen
import torch
x = torch.zeros(4, device="cuda")
c = native.Context(0)
c.load_graph(gen.quincy(1000, 100, 5, 10, 1))
r = c.solve()
print("torch-first ok", r.cost, x.sum().item())
maps = [l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l]
print(sorted(set(maps)))
EOF
cat "$OUT/probe.log"
for pre in 1 0; do
    KS_PRELOAD_TORCH=$pre timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --cpu-baseline off \
        > "$OUT/bench_pre$pre.json" 2> "$OUT/bench_pre$pre.err" || { echo "bench pre=$pre failed"; tail -20 "$OUT/bench_pre$pre.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_pre$pre.json')); print('preload', $pre, 'ms/step', d['ms_per_step'], d['step_ms'])"
done
