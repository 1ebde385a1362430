#!/bin/bash
# PMC traffic passes only (FETCH_SIZE, WRITE_SIZE in separate runs).
set -o pipefail
OUT=gpurun_out/${1:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch" -o run -- \
    python -u bench.py --steps 1 --warmup 0 --cpu-baseline off > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" \
    || { echo "pmc fetch failed"; tail -20 "$OUT/pmc_fetch.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/pmc_write" -o run -- \
    python -u bench.py --steps 1 --warmup 0 --cpu-baseline off > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err" \
    || { echo "pmc write failed"; tail -20 "$OUT/pmc_write.err"; exit 1; }
python tools/pmc_summary.py "$OUT/pmc_fetch" "$OUT/pmc_write" > "$OUT/pmc_traffic.json" && cat "$OUT/pmc_traffic.json"
