#!/bin/bash
# Round artefacts on the GPU box: GPU tests, smoke, rocprofv3 kernel stats of the
# headline command, PMC passes (traffic, atomics) + FETCH_SIZE calibration, and
# the bench lines (config 3 with CPU baseline, config 4, config 5).
# Usage: gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
    python -u bench.py --steps 5 --warmup 1 --cpu-baseline off > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
    || { echo "rocprof failed"; tail -30 "$OUT/bench_prof.err"; exit 1; }
python tools/prof_summary.py "$OUT/prof" > "$OUT/kernel_stats.csv" && head -6 "$OUT/kernel_stats.csv"
tools/gpu_pmc.sh "$TAG/pmc" || exit 1
# FETCH_SIZE calibration (tools/gpu_calib.sh) is a one-off: profiles/r02_fetch_calibration.json
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('full', d['ms_per_step'], d['value'], d['cpu_baseline']['value'], d['parity']['match'])"
for wl in incremental batch; do
    timeout -k 10 400 python -u bench.py --workload $wl --steps 5 --warmup 2 > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" \
        || { echo "bench $wl failed"; tail -30 "$OUT/bench_$wl.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_$wl.json')); print('$wl', d['ms_per_step'], d['value'], (d.get('cpu_baseline') or {}).get('value'), d.get('parity'))"
done
