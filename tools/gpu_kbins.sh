#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-kb}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT/prof" -o run -- \
    python -u bench.py --steps 3 --warmup 1 --cpu-baseline off ${@:2} > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "rocprof failed"; tail -30 "$OUT/bench.err"; exit 1; }
python tools/kbins.py "$OUT/prof"
