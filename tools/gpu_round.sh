#!/bin/bash
# One round's measurement on the GPU box (run through gpurun; tools/collect.sh then
# copies the results into profiles/):
#   suite  the GPU test suite and smoke()
#   bench  one bench line per headline workload (configs 3, 2, 4, 5), each with its
#          CPU baseline legs
#   pmc    per workload: PMC passes (traffic, atomics, VALU) and a kernel-trace pass
#          of the same bench command (tools/gpu_pmc.sh)
# Every GPU step has its own time limit and the script stops at the first failure.
# Usage: gpu_round.sh TAG [suite|bench|pmc|all]
set -o pipefail
TAG=${1:-round}
WHAT=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$WHAT" = suite ] || [ "$WHAT" = all ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
    tail -1 "$OUT/pytest_gpu.log"
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 1; }
    tail -1 "$OUT/smoke.log"
fi
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
if [ "$WHAT" = pmc ] || [ "$WHAT" = all ]; then
    for wl in config3 config2 config4 config5; do
        bash tools/gpu_pmc.sh "${TAG}_pmc_$wl" "$wl" all > "$OUT/pmc_$wl.log" 2>&1 \
            || { echo "pmc $wl failed"; tail -20 "$OUT/pmc_$wl.log"; exit 1; }
        echo "pmc $wl ok"
    done
fi
echo ok
