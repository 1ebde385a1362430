#!/bin/bash
# Round-5 study of one config-3 solve: the cycle log, and a kernel trace of the
# bench (per-launch durations, Bellman-Ford rounds per update, per-cycle time).
set -o pipefail
TAG=${1:-study5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/cyclelog.py > "$OUT/cyclelog.out" 2> "$OUT/cyclelog.err" || { echo cyclelog failed; tail "$OUT/cyclelog.err"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d "$OUT/kt" -o run -- python -u bench.py --steps 2 --warmup 1 --cpu-baseline off > "$OUT/kt.json" 2> "$OUT/kt.err" || { echo trace failed; tail "$OUT/kt.err"; exit 1; }
python tools/kernel_trace.py "$OUT/kt" --seq --cycles > "$OUT/kt.txt"
head -30 "$OUT/kt.txt"
echo ok
