#!/bin/bash
# bench.py under ks_opts settings (runtime options), one line each.
# Usage: gpu_bench_opts.sh TAG "BENCH ARGS" "OPTS1" ["OPTS2" ...]  (OPTS: space-separated key=value, or -)
set -o pipefail
OUT=gpurun_out/${1:-bench_opts}; BARGS=$2; shift 2
mkdir -p "$OUT"
i=0
for o in "$@"; do
    i=$((i + 1))
    flags=""
    [ "$o" != "-" ] && for kv in $o; do flags="$flags --opt $kv"; done
    timeout -k 10 240 python -u bench.py --cpu-baseline off $BARGS $flags > "$OUT/$i.json" 2> "$OUT/$i.err" \
        || { echo "$o failed"; tail -5 "$OUT/$i.err"; exit 1; }
    python - "$OUT/$i.json" "$o" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["ms_per_step"], d.get("latency", {}).get("p50_ms"), d.get("latency", {}).get("max_ms"),
      {k: v["ms_per_step"] for k, v in d["roofline"]["kinds"].items()})
PY
done
