#!/bin/bash
# Config-4 A/B: interleaved arms of the incremental bench,
# each "label|bench args|library variant". Usage: gpu_c4ab5.sh TAG REPS ARM...
set -o pipefail
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in $(seq 1 $REPS); do
    for arm in "$@"; do
        IFS='|' read -r label bargs var <<< "$arm"
        KS_LIB_VARIANT=$var timeout -k 10 300 python -u bench.py --workload incremental --cpu-baseline off $bargs \
            > "$OUT/${label}_$i.json" 2> "$OUT/${label}_$i.err" || { echo "arm $label $i failed"; tail -20 "$OUT/${label}_$i.err"; exit 1; }
        python - "$OUT/${label}_$i.json" "$label" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
l = d.get("latency") or {}
print(sys.argv[2], "ms", d["ms_per_step"], "p50", l.get("p50_ms"), "max", l.get("max_ms"), "max/med", l.get("max_over_median"),
      "parity", (d.get("parity") or {}).get("match"))
PY
    done
done
echo ok
