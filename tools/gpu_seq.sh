#!/bin/bash
# Kernel trace of config 3 with each update's Bellman-Ford round sequence.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/seq
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/kt -o run -- python -u bench.py --steps 2 --warmup 1 --cpu-baseline off > $OUT/kt.json 2> $OUT/kt.err || exit 1
python tools/kernel_trace.py $OUT/kt --seq > $OUT/kt.txt
python tools/kernel_trace.py $OUT/kt --cycles > $OUT/cycles.txt || true
head -30 $OUT/kt.txt
