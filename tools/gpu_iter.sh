#!/bin/bash
# One iteration: GPU parity tests, a bench line, and a kernel-duration breakdown.
set -o pipefail
OUT=gpurun_out/${1:-iter}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u bench.py --steps 8 --warmup 1 --cpu-baseline off ${@:2} > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); s=d['solve']; print('ms/step', d['ms_per_step'], 'steps', d['step_ms'], 'cost', s['total_cost'], 'phases', s['phases'], 'sweeps', s['sweeps'], 'gus', s['global_updates'], 'bf_rounds', s['gu_iterations'], 'bf_launches', s['gu_launches'], s['ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
    python -u bench.py --steps 2 --warmup 1 --cpu-baseline off ${@:2} > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
    || { echo "rocprof failed"; tail -30 "$OUT/bench_prof.err"; exit 1; }
python tools/kdist.py "$OUT/prof" | head -8
