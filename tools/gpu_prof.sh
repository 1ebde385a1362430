#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run.
set -o pipefail
OUT=gpurun_out/${1:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
    python -u bench.py --steps 2 --warmup 1 --cpu-baseline off ${@:2} > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
    || { echo "rocprof failed"; tail -30 "$OUT/bench_prof.err"; exit 1; }
python tools/prof_summary.py "$OUT/prof" > "$OUT/kernel_stats.csv" && cat "$OUT/kernel_stats.csv"
