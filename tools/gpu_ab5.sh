#!/bin/bash
# Interleaved A/B of ks_opts settings on one workload (round 5).
# Usage: gpu_ab5.sh TAG WORKLOAD_ARGS REPS OPT_A OPT_B   (OPT: "" or "field=value[,field=value]")
set -o pipefail
TAG=$1; WL=$2; REPS=${3:-3}; A=$4; B=$5
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# an option spec may name a library variant: VARIANT=tag (libksmcmf_tag.so, _build.build_variant)
optargs() { local o=$1; local r=""; IFS=',' read -ra kv <<< "$o"; for x in "${kv[@]}"; do case $x in VARIANT=*) ;; "") ;; *) r="$r --opt $x";; esac; done; echo "$r"; }
variant() { local o=$1; IFS=',' read -ra kv <<< "$o"; for x in "${kv[@]}"; do case $x in VARIANT=*) echo "${x#VARIANT=}";; esac; done; }
for i in $(seq 1 $REPS); do
    for v in A B; do
        if [ $v = A ]; then o=$A; else o=$B; fi
        KS_LIB_VARIANT=$(variant "$o") timeout -k 10 300 python -u bench.py $WL --cpu-baseline off $(optargs "$o") > "$OUT/${v}_$i.json" 2> "$OUT/${v}_$i.err" \
            || { echo "bench $v $i failed"; tail -20 "$OUT/${v}_$i.err"; exit 1; }
        python - "$OUT/${v}_$i.json" "$v[$o]" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; l = d.get("latency") or {}
print(sys.argv[2], "ms", d["ms_per_step"], "p50", l.get("p50_ms"), "max", l.get("max_ms"), r.get("kernel"), "avg_us", r.get("avg_launch_us"),
      "k_ms", r.get("kernel_ms_per_step"), "parity", (d.get("parity") or {}).get("match"))
PY
    done
done
echo ok
