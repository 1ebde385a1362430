#!/bin/bash
# Concurrency regression probe + GPU tests + full bench after a coherence change.
set -o pipefail
OUT=gpurun_out/${1:-bf}
mkdir -p "$OUT"
timeout -k 10 150 python -u tools/probe_batch.py 64 4,8 > "$OUT/probe.log" 2>&1 || { tail -20 "$OUT/probe.log"; exit 1; }
grep -v amdgpu.ids "$OUT/probe.log"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > "$OUT/bench.json" 2> "$OUT/bench.err" \
    || { echo "bench failed"; tail -30 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('full ms/step', d['ms_per_step'], d['step_ms'])"
