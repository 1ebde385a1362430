#!/bin/bash
# alpha x gu_interval grid on config3 (and config2) — one bench line each.
set -o pipefail
OUT=gpurun_out/${1:-grid}
mkdir -p "$OUT"
CFG=${2:-config3}
for a in ${ALPHAS:-8 16 32 64}; do
  for gi in ${GIS:-8 16 32}; do
    timeout -k 10 120 python -u bench.py --config $CFG --steps 3 --warmup 1 --cpu-baseline off --alpha $a --gu-interval $gi \
      > "$OUT/b_${CFG}_${a}_${gi}.json" 2> "$OUT/b_${CFG}_${a}_${gi}.err" || { echo "fail a=$a gi=$gi"; tail -5 "$OUT/b_${CFG}_${a}_${gi}.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/b_${CFG}_${a}_${gi}.json')); s=d['solve']; print('$CFG alpha=$a gi=$gi', d['ms_per_step'], 'ph', s['phases'], 'sw', s['sweeps'], 'gus', s['global_updates'], 'bfr', s['gu_iterations'], 'cost', s['total_cost'])" | tee -a "$OUT/grid.txt"
  done
done
