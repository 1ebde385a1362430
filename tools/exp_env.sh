#!/bin/bash
# Sweep an env variable over values on config3 (3 repeats each, 5 steps).
set -o pipefail
OUT=gpurun_out/${1:-env}; VAR=$2; VALS=$3
mkdir -p "$OUT"
for r in 1 2; do for val in $VALS; do
  env $VAR=$val timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --cpu-baseline off ${@:4} > "$OUT/b_${val}_$r.json" 2>"$OUT/b_${val}_$r.err" || { tail -5 "$OUT/b_${val}_$r.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_${val}_$r.json')); s=d['solve']; print('$VAR=$val', d['ms_per_step'], 'ph', s['phases'], 'sw', s['sweeps'], 'gus', s['global_updates'], 'bfr', s['gu_iterations'], 'pr_ms', round(s['ms']['global_update'],2))"
done; done
