#!/bin/bash
# Quick GPU iteration: parity tests (fast subset unless FULL=1) then one bench line.
set -o pipefail
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --cpu-baseline off ${@:2} > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); s=d['solve']; print('ms/step', d['ms_per_step'], 'cost', s['total_cost'], 'phases', s['phases'], 'sweeps', s['sweeps'], 'gus', s['global_updates'], 'bf_rounds', s['gu_iterations'], 'bf_launches', s['gu_launches'], s['ms'])"
