#!/bin/bash
# Config 4 re-solves: cold vs warm start (with and without the price shift for
# cost rises on flow-carrying arcs). Usage: gpu_warm_ab.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-warm_ab}
mkdir -p "$OUT"
for v in "cold:--warm 0" "warm:--warm 1" "warm2:--warm 2" "warm2_noshift:--warm 2 --opt warm_shift=-1"; do
    name=${v%%:*}; flags=${v#*:}
    echo "== $name ($flags)"
    timeout -k 10 240 python -u bench.py --workload incremental --cpu-baseline off $flags \
        > "$OUT/$name.json" 2> "$OUT/$name.log" || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
    tail -1 "$OUT/$name.json" | cut -c1-300
done
