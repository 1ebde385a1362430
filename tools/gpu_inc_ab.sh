#!/bin/bash
# Config-4 A/B: cold vs warm re-solves and tail thresholds (no CPU baseline).
# Usage: gpu_inc_ab.sh TAG [variant ...]   (variant: "cold", "warm", or KS_BENCH_OPTS specs)
set -o pipefail
TAG=${1:-incab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in "$@"; do
    warm=0; opts=""
    case "$v" in
        warm*) warm=1; opts=${v#warm};;
        cold*) opts=${v#cold};;
    esac
    opts=${opts#:}
    KS_BENCH_OPTS="$opts" timeout -k 10 300 python -u bench.py --workload incremental --steps 6 --warmup 1 --warm $warm \
        --cpu-baseline off > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "bench $v failed"; tail -20 "$OUT/$v.err"; exit 1; }
    python - "$OUT/$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "ms/round", d["ms_per_step"], d["config"]["round_ms"], "parity", d["parity"]["match"],
      "solve_ms", [r["solve_ms"] for r in d["rounds"]], "updates", [r["updates"] for r in d["rounds"]],
      "rebuilt", [r["rebuilt"] for r in d["rounds"]])
PY
done
