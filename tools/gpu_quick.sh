#!/bin/bash
# Usage: gpu_quick.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
K=${2:-parity}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print('config3 ms/step', d['ms_per_step'], 'steps', d['step_ms'], 'cost', d['parity']['gpu_costs'])"
