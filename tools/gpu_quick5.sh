#!/bin/bash
# Round-5 quick check on the GPU box: the GPU suite, then one bench line per
# workload without the CPU legs. Usage: gpu_quick5.sh TAG [tests|bench|all]
set -o pipefail
TAG=${1:-r05}
WHAT=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$WHAT" != bench ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
    tail -2 "$OUT/pytest_gpu.log"
fi
if [ "$WHAT" != tests ]; then
    for wl in config3 config2 config4 config5; do
        case $wl in
            config3) args="--steps 10 --warmup 2";;
            config2) args="--config config2 --steps 20 --warmup 2";;
            config4) args="--workload incremental";;
            config5) args="--workload batch --steps 10 --warmup 2";;
        esac
        timeout -k 10 300 python -u bench.py $args --cpu-baseline off > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" \
            || { echo "bench $wl failed"; tail -20 "$OUT/bench_$wl.err"; exit 1; }
        python - "$OUT/bench_$wl.json" $wl <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "ms", d["ms_per_step"], "lat", d.get("latency"), r.get("kernel"), "frac", r.get("frac"),
      "avg_us", r.get("avg_launch_us"), "parity", (d.get("parity") or {}).get("match"))
PY
    done
fi
echo ok
