#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-stamp}
mkdir -p "$OUT"
for sw in ${SWEEPS:-100 400 800 1200 1600 2000}; do
  KS_STAMP=$sw:$OUT/stamp_$sw.txt KS_TRACE=$OUT/trace_$sw.jsonl timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --cpu-baseline off > /dev/null || exit 1
done
ls $OUT
