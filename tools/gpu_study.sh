#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/study
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/kt -o run -- python -u bench.py --steps 2 --warmup 1 --cpu-baseline off > $OUT/kt.json 2> $OUT/kt.err || exit 1
python tools/kernel_trace.py $OUT/kt --seq --cycles > $OUT/kt.txt
rm -rf $OUT/kt
head -24 $OUT/kt.txt
gcc -O2 -o /tmp/tail_dump tools/proto/tail_dump.c
KS_LIB_VARIANT=dump KS_DUMP=/tmp/tail.dump timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 \
    --cpu-baseline off > $OUT/dump_bench.json 2> $OUT/dump_bench.err || exit 1
gzip -1 -c /tmp/tail.dump > $OUT/tail.dump.gz
HUBS=0 SLACK=1 timeout -k 10 300 /tmp/tail_dump /tmp/tail.dump > $OUT/analysis.txt 2>&1
echo done
