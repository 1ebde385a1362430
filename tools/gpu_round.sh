#!/bin/bash
# Round artefacts on the GPU box: parity tests, smoke, bench (with CPU baseline),
# rocprofv3 kernel stats, and PMC traffic passes.  Usage: gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
    python -u bench.py --steps 5 --warmup 1 --cpu-baseline off > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
    || { echo "rocprof failed"; tail -30 "$OUT/bench_prof.err"; exit 1; }
python tools/prof_summary.py "$OUT/prof" > "$OUT/kernel_stats.csv" && head -6 "$OUT/kernel_stats.csv"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch" -o run -- \
    python -u bench.py --steps 1 --warmup 0 --cpu-baseline off > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" \
    || { echo "pmc fetch failed"; tail -20 "$OUT/pmc_fetch.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/pmc_write" -o run -- \
    python -u bench.py --steps 1 --warmup 0 --cpu-baseline off > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err" \
    || { echo "pmc write failed"; tail -20 "$OUT/pmc_write.err"; exit 1; }
python tools/pmc_summary.py "$OUT/pmc_fetch" "$OUT/pmc_write" > "$OUT/pmc_traffic.json" && cat "$OUT/pmc_traffic.json"
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
for wl in incremental batch; do
    timeout -k 10 300 python -u bench.py --workload $wl --steps 5 --warmup 2 > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" \
        || { echo "bench $wl failed"; tail -30 "$OUT/bench_$wl.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_$wl.json')); print('$wl', d['ms_per_step'], d['value'], (d.get('cpu_baseline') or {}).get('value'), d.get('parity'))"
done
