#!/bin/bash
# Correctness + headline check on the GPU box: the full -m gpu suite, smoke(),
# then the bench lines (config 3 with CPU baseline; optionally config 4 / 2 / 5).
# Usage: gpu_check.sh TAG [all]
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('config3', d['ms_per_step'], d['value'], d['parity']['match'], d['roofline']['kernel'], d['roofline']['frac'])"
[ "$2" = "all" ] || exit 0
timeout -k 10 400 python -u bench.py --workload incremental > "$OUT/bench_incremental.json" 2> "$OUT/bench_incremental.err" \
    || { echo "bench incremental failed"; tail -30 "$OUT/bench_incremental.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_incremental.json')); print('config4', d['ms_per_step'], d['config']['round_ms'], d['parity']['match'], d['cpu_baseline']['ms'], d['cpu_baseline']['cold_reference_path']['ms'])"
timeout -k 10 300 python -u bench.py --config config2 --steps 20 --warmup 3 > "$OUT/bench_config2.json" 2> "$OUT/bench_config2.err" \
    || { echo "bench config2 failed"; tail -30 "$OUT/bench_config2.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_config2.json')); print('config2', d['ms_per_step'], d['value'], d['parity']['match'])"
timeout -k 10 300 python -u bench.py --workload batch > "$OUT/bench_batch.json" 2> "$OUT/bench_batch.err" \
    || { echo "bench batch failed"; tail -30 "$OUT/bench_batch.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_batch.json')); print('config5 abi', d['ms_per_step'], d['value'], d['parity'].get('match'))"
timeout -k 10 300 python -u bench.py --workload batch --batch-mode streams --workers 8 > "$OUT/bench_batch_streams.json" 2> "$OUT/bench_batch_streams.err" \
    || { echo "bench batch streams failed"; tail -30 "$OUT/bench_batch_streams.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_batch_streams.json')); print('config5 streams', d['ms_per_step'], d['value'], d['parity'].get('match'), d['cell_latency'])"
