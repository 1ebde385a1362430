#!/bin/bash
# Round-5 measurement: one bench line per headline workload (with its CPU
# baseline legs), then the PMC + kernel-trace passes of each workload
# (tools/gpu_pmc.sh). Usage: gpu_r04_final.sh TAG [bench|pmc|trace|all]
set -o pipefail
TAG=${1:-r05}
OUT=gpurun_out/$TAG
WHAT=${2:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
bench() {   # name, bench args...
    local name=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
        || { echo "bench $name failed"; tail -20 "$OUT/bench_$name.err"; exit 1; }
    python - "$OUT/bench_$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], d["value"], d["unit"], d["ms_per_step"], d.get("latency"), r["kernel"], r["frac"],
      r.get("avg_launch_us"), (d.get("cpu_baseline") or {}).get("value"))
PY
}
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
    bench config3
    bench config2 --config config2 --steps 10
    bench config4 --workload incremental
    bench config5 --workload batch
fi
if [ "$WHAT" != bench ]; then
    PASSES=all; [ "$WHAT" = trace ] && PASSES=trace
    for wl in config3 config2 config4 config5; do
        bash tools/gpu_pmc.sh "${TAG}_pmc_$wl" "$wl" "$PASSES" > "$OUT/pmc_$wl.log" 2>&1 \
            || { echo "pmc $wl failed"; tail -20 "$OUT/pmc_$wl.log"; exit 1; }
        echo "pmc $wl ok"
    done
fi
echo ok
