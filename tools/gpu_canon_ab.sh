#!/bin/bash
# Config 4: cold re-solve vs warm starts with and without canonical prices at
# each solve's end (ks_opts.warm_canon). Usage: gpu_canon_ab.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-canon_ab}
mkdir -p "$OUT"
for v in "cold:--warm 0" "warm1c:--warm 1" "warm2c:--warm 2" "warm2:--warm 2 --opt warm_canon=-1" "cold2:--warm 0" "warm2c_log:--warm 2 --opt log_cycles=1"; do
    name=${v%%:*}; flags=${v#*:}
    timeout -k 10 240 python -u bench.py --workload incremental --cpu-baseline off $flags \
        > "$OUT/$name.json" 2> "$OUT/$name.log" || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
    python - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["ms_per_step"], d["latency"]["p50_ms"], d["latency"]["max_ms"], [r["ms"] for r in d["rounds"]], [r["updates"] for r in d["rounds"]])
PY
    grep -h "warm start:\|canonical" "$OUT/$name.log" | head -24
done
