#!/bin/bash
# Parameter exploration on the GPU box: trace one solve, then alpha x gu_interval grid.
set -o pipefail
OUT=gpurun_out/${1:-exp}
mkdir -p "$OUT"
KS_TRACE=$OUT/trace.jsonl timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --cpu-baseline off > "$OUT/trace_bench.json" || exit 1
for a in 8 16 32 64; do
  for gi in 8 16 48 128; do
    timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --cpu-baseline off --alpha $a --gu-interval $gi --batch 8 \
      | python -c "import json,sys; d=json.load(sys.stdin); s=d['solve']; print($a, $gi, d['ms_per_step'], s['sweeps'], s['global_updates'], s['gu_iterations'], s['phases'])" \
      >> "$OUT/grid.txt" || exit 1
  done
done
cat "$OUT/grid.txt"
