#!/bin/bash
# GPU tests + incremental bench (warm vs from-scratch) + batch union bench.
set -o pipefail
OUT=gpurun_out/${1:-incr}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for w in 1 0; do
    timeout -k 10 300 python -u bench.py --workload incremental --warm $w --steps 5 --warmup 2 --cpu-baseline off \
        > "$OUT/incr_w$w.json" 2> "$OUT/incr_w$w.err" || { echo "incr $w failed"; tail -30 "$OUT/incr_w$w.err"; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/incr_w$w.json')); print('warm', $w, 'ms/step', d['ms_per_step'])
for r in d['rounds']: print('  ', {k: r[k] for k in ('round','deltas','ms','apply_ms','solve_ms','cost','warm','phases','sweeps','updates','bf_rounds','solve_parts_ms')})"
done
timeout -k 10 300 python -u bench.py --workload batch --steps 5 --warmup 2 --cpu-baseline off > "$OUT/batch.json" 2> "$OUT/batch.err" \
    || { echo "batch failed"; tail -30 "$OUT/batch.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/batch.json')); print('batch union', d['ms_per_step'], d['value'], d['step_ms'], d['parity'], d['solve']['phases'], d['solve']['sweeps'], d['solve']['ms'])"
