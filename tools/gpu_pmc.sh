#!/bin/bash
# PMC passes over one bench run of a workload, one rocprofv3 run per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass; TCC holds 4 counters, TA 2),
# then a kernel-trace pass for the per-kernel device time of the same command.
# Usage: gpu_pmc.sh TAG [config3|config2|config4|config5]
set -o pipefail
OUT=gpurun_out/${1:-pmc}
WL=${2:-config3}
case "$WL" in
    config3) ARGS="--steps 1 --warmup 0" ;;
    config2) ARGS="--config config2 --steps 3 --warmup 0" ;;
    config4) ARGS="--workload incremental --steps 3 --warmup 0" ;;
    config5) ARGS="--workload batch --steps 1 --warmup 0" ;;
    *) echo "unknown workload $WL"; exit 2 ;;
esac
mkdir -p "$OUT"
export TMPDIR=/tmp
run_pass() {   # name, rocprofv3 args...
    local name=$1; shift
    timeout -s KILL 150 rocprofv3 "$@" -f csv -d "$OUT/$name" -o run -- \
        python -u bench.py $ARGS --cpu-baseline off > "$OUT/$name.json" 2> "$OUT/$name.err" \
        || { echo "pass $name failed"; tail -20 "$OUT/$name.err"; exit 1; }
}
run_pass fetch --pmc FETCH_SIZE
run_pass write --pmc WRITE_SIZE
run_pass atom --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum
run_pass ta --pmc TA_FLAT_ATOMIC_WAVEFRONTS_sum
run_pass trace --kernel-trace --stats
python tools/pmc_per_kernel.py "$OUT/fetch" "$OUT/write" "$OUT/atom" "$OUT/ta" > "$OUT/pmc_per_kernel.json"
python tools/prof_summary.py "$OUT/trace" > "$OUT/kernel_stats.csv"
echo "$WL" > "$OUT/workload.txt"
echo ok
