#!/bin/bash
# Interleaved A/B on the config-3 bench (same box, same run). Each variant is
# "default" (libksmcmf.so), a library tag (libksmcmf_<tag>.so), or environment
# settings "K=V[,K=V]" applied to the default library. AB_ARGS adds bench flags.
# Usage: ab.sh TAG ROUNDS variant...
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
    for v in "$@"; do
        name=$(echo "$v" | sed 's/[,=@:+]/_/g')
        if [[ "$v" == *@* ]]; then   # lib@K=V[,K=V]: a library variant with environment settings
            lib="KS_LIB_VARIANT=${v%%@*}"; envs=$(echo "${v#*@}" | tr ',' ' ')
        elif [[ "$v" == *=* ]]; then
            envs=$(echo "$v" | tr ',' ' '); lib=""
        elif [ "$v" = default ]; then envs=""; lib=""
        else envs=""; lib="KS_LIB_VARIANT=$v"
        fi
        timeout -k 10 120 env $envs $lib python -u bench.py --steps 10 --warmup 2 --cpu-baseline off ${AB_ARGS} \
            > "$OUT/$name.$r.json" 2> "$OUT/$name.$r.err" \
            || { echo "bench $v failed"; tail -20 "$OUT/$name.$r.err"; exit 1; }
        python - "$OUT/$name.$r.json" "$v" "$r" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); s = sorted(d["step_ms"]); r = d.get("solve", {})
print(sys.argv[2], sys.argv[3], "ms/step", d["ms_per_step"], "median", s[len(s) // 2], "min", s[0],
      "sweeps", r.get("sweeps"), "gus", r.get("global_updates"), "tail", r.get("tail_calls"), r.get("tail_sweeps"),
      "cost", d.get("parity", {}).get("gpu_costs"))
PY
    done
done
