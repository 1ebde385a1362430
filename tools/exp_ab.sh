#!/bin/bash
# A/B of an env switch on config3: runs bench with VAR=a and VAR=b, 3 repeats each.
set -o pipefail
OUT=gpurun_out/${1:-ab}; VAR=$2; A=$3; B=$4
mkdir -p "$OUT"
for r in 1 2 3; do for val in $A $B; do
  env $VAR=$val timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --cpu-baseline off ${@:5} > "$OUT/b_${val}_$r.json" 2>"$OUT/b_${val}_$r.err" || { tail -5 "$OUT/b_${val}_$r.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/b_${val}_$r.json')); s=d['solve']; print('$VAR=$val', d['ms_per_step'], 'ph', s['phases'], 'sw', s['sweeps'], 'gus', s['global_updates'], 'bfr', s['gu_iterations'])"
done; done
KS_TRACE=$OUT/trace.jsonl timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --cpu-baseline off ${@:5} > /dev/null
