#!/bin/bash
# FETCH_SIZE / WRITE_SIZE / atomic-counter calibration on known byte counts
# (tools/calib/calib_fetch.hip), plus the counter list of this rocprofv3.
set -o pipefail
OUT=gpurun_out/${1:-calib}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
grep -i -E "atomic|FETCH_SIZE|WRITE_SIZE|EA0_RDREQ|EA0_WRREQ" "$OUT/counters.txt" | head -60 > "$OUT/counters_atomic.txt" || true
for c in FETCH_SIZE WRITE_SIZE ${CALIB_EXTRA}; do
    timeout -s KILL 60 rocprofv3 --pmc $c -f csv -d "$OUT/pmc_$c" -o run -- tools/calib/calib_fetch \
        > "$OUT/calib_$c.json" 2> "$OUT/calib_$c.err" || { echo "pass $c failed"; tail -5 "$OUT/calib_$c.err"; exit 1; }
done
echo ok
