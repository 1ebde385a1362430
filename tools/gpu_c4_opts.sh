#!/bin/bash
# Config 4 rounds under named bench flag sets, one process each, in order.
# Usage: gpu_c4_opts.sh TAG 'name:flags' ['name:flags' ...]
set -o pipefail
OUT=gpurun_out/${1:-c4_opts}; shift
mkdir -p "$OUT"
for v in "$@"; do
    name=${v%%:*}; flags=${v#*:}
    timeout -k 10 240 python -u bench.py --workload incremental --cpu-baseline off $flags \
        > "$OUT/$name.json" 2> "$OUT/$name.log" || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
    python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["ms_per_step"], d["latency"]["p50_ms"], d["latency"]["max_ms"], [r["ms"] for r in d["rounds"]][1:], [r["updates"] for r in d["rounds"]][1:])
PY
done
