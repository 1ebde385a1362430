#!/bin/bash
# GPU parity tests + one bench line per workload (full / incremental / batch).
set -o pipefail
OUT=gpurun_out/${1:-wl}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for wl in full incremental batch; do
    timeout -k 10 300 python -u bench.py --workload $wl --steps ${STEPS:-5} --warmup 2 --cpu-baseline ${CPU:-off} \
        > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" \
        || { echo "bench $wl failed"; tail -30 "$OUT/bench_$wl.err"; exit 1; }
    python - "$OUT/bench_$wl.json" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
print(d["config"]["workload"][:60], "| ms/step", d["ms_per_step"], "| value", d["value"],
      "| frac", d["roofline"]["frac"], "| cpu", (d.get("cpu_baseline") or {}).get("value"))
for r in d.get("rounds", []):
    print("  round", r)
if "gather" in d: print("  gather", d["gather"])
EOF
done
