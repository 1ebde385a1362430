#!/bin/bash
# One traced + profiled full solve and its per-cycle time model.
set -o pipefail
OUT=gpurun_out/${1:-cyc}
mkdir -p "$OUT"
export TMPDIR=/tmp
rm -f "$OUT/trace.jsonl"
KS_TRACE=$OUT/trace.jsonl timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT/prof" -o run -- \
    python -u bench.py --steps 1 --warmup 1 --cpu-baseline off ${@:2} > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "rocprof failed"; tail -30 "$OUT/bench.err"; exit 1; }
python tools/cycle_breakdown.py "$OUT/prof" "$OUT/trace.jsonl"
