#!/bin/bash
# Round-4 GPU check: the GPU suite, then config-5 (cell solver, one workgroup
# per cell) and config-2 bench lines. Usage: gpu_r04.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r04}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 200 python -u bench.py --workload batch --steps 5 --warmup 2 --cpu-baseline off > "$OUT/bench_batch.json" 2> "$OUT/bench_batch.err" \
    || { echo "bench batch failed"; tail -20 "$OUT/bench_batch.err"; exit 1; }
timeout -k 10 200 python -u bench.py --config config2 --steps 10 --warmup 2 --cpu-baseline off > "$OUT/bench_config2.json" 2> "$OUT/bench_config2.err" \
    || { echo "bench config2 failed"; tail -20 "$OUT/bench_config2.err"; exit 1; }
python - "$OUT" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench_batch", "bench_config2"):
    d = json.load(open(f"{o}/{f}.json"))
    print(f, d["ms_per_step"], d.get("latency"), d["roofline"]["kernel"], d["roofline"]["frac"], d["solve"]["solver"], d["solve"].get("cells"))
PY
