#!/bin/bash
# GPU tests + config-5 bench in both batch modes.
set -o pipefail
OUT=gpurun_out/${1:-batch}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for mode in union streams; do
    timeout -k 10 300 python -u bench.py --workload batch --batch-mode $mode --steps 5 --warmup 2 --cpu-baseline ${CPU:-off} \
        > "$OUT/bench_$mode.json" 2> "$OUT/bench_$mode.err" || { echo "bench $mode failed"; tail -30 "$OUT/bench_$mode.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_$mode.json')); print('$mode', d['ms_per_step'], d['value'], d['step_ms'], d['parity'], d['gather'], (d.get('cpu_baseline') or {}).get('value'), d['solve']['phases'], d['solve']['sweeps'], d['solve']['ms'])"
done
