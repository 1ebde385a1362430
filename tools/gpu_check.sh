#!/bin/bash
# One GPU-box pass: parity tests, smoke, a short bench, rocprofv3 kernel stats.
# Usage (from the build container):
#   gpurun --timeout 900 -- bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
    python -u bench.py --steps 5 --warmup 2 --cpu-baseline off > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
    || { echo "rocprof failed"; tail -30 "$OUT/bench_prof.err"; exit 1; }
python tools/prof_summary.py "$OUT/prof" > "$OUT/kernel_stats.csv" && cat "$OUT/kernel_stats.csv"
