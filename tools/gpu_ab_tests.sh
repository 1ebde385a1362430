#!/bin/bash
# GPU parity tests, then an env A/B on the full bench (VARIANTS as in exp_env.sh).
set -o pipefail
OUT=gpurun_out/${1:-abt}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { echo "pytest failed"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash tools/exp_env.sh "${1:-abt}_env"
