#!/bin/bash
# Interleaved A/B of a compile-time library variant (KS_LIB_VARIANT, built by
# _build.build_variant) against the default build on one workload.
# Usage: gpu_lib_ab.sh TAG VARIANT [bench args...]
set -o pipefail
OUT=gpurun_out/${1:-lib_ab}; VAR=$2; shift 2
mkdir -p "$OUT"
for rep in 1 2; do
    for v in base "$VAR"; do
        if [ "$v" = base ]; then unset KS_LIB_VARIANT; else export KS_LIB_VARIANT=$v; fi
        timeout -k 10 240 python -u bench.py --cpu-baseline off "$@" > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" \
            || { echo "$v failed"; tail -5 "$OUT/${v}_$rep.err"; exit 1; }
        python - "$OUT/${v}_$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["ms_per_step"], d.get("latency"), d["roofline"]["kernel"], d["roofline"]["frac"], d["roofline"].get("avg_launch_us"))
PY
    done
done
