#!/bin/bash
# Dump the residual state at the first final-phase tail cycle of a config-3 solve
# (-DKS_DUMP library variant) and analyse it on the box's CPU (tools/proto/tail_dump.c).
set -e -o pipefail
OUT=gpurun_out/dump
mkdir -p $OUT
gcc -O2 -o /tmp/tail_dump tools/proto/tail_dump.c
KS_LIB_VARIANT=dump KS_DUMP=/tmp/tail.dump timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 \
    --cpu-baseline off > $OUT/bench.json 2> $OUT/bench.err
for v in "HUBS=1 SLACK=1" "HUBS=0 SLACK=1" "HUBS=1 SLACK=4" "HUBS=0 SLACK=4"; do
    echo "== $v" >> $OUT/analysis.txt
    env $v timeout -k 10 300 /tmp/tail_dump /tmp/tail.dump >> $OUT/analysis.txt 2>&1
done
