#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-trace}
mkdir -p "$OUT"
KS_TRACE=$OUT/trace.jsonl timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --cpu-baseline off ${@:2} > "$OUT/trace_bench.json" || exit 1
tail -c 600 "$OUT/trace_bench.json"
