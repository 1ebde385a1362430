#!/bin/bash
# PMC passes over one bench run of a workload, one rocprofv3 run per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass; TCC holds 4 counters, TA 2),
# then a kernel-trace pass for the per-kernel device time. The trace pass runs
# the bench line's own arguments (TARGS, as tools/gpu_round.sh runs them), so
# its per-kernel averages cover the same launch mix as the event-timed line.
# Usage: gpu_pmc.sh TAG [config3|config2|config4|config5] [all|trace]
set -o pipefail
OUT=gpurun_out/${1:-pmc}
WL=${2:-config3}
case "$WL" in
    config3) ARGS="--steps 1 --warmup 0"; TARGS="" ;;
    config2) ARGS="--config config2 --steps 3 --warmup 0"; TARGS="--config config2 --steps 10" ;;
    config4) ARGS="--workload incremental --steps 3 --warmup 0"; TARGS="--workload incremental" ;;
    config5) ARGS="--workload batch --steps 1 --warmup 0"; TARGS="--workload batch" ;;
    *) echo "unknown workload $WL"; exit 2 ;;
esac
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=${3:-all}
run_pass() {   # name, bench args, rocprofv3 args...
    local name=$1 bargs=$2; shift 2
    timeout -s KILL 150 rocprofv3 "$@" -f csv -d "$OUT/$name" -o run -- \
        python -u bench.py $bargs --cpu-baseline off > "$OUT/$name.json" 2> "$OUT/$name.err" \
        || { echo "pass $name failed"; tail -20 "$OUT/$name.err"; exit 1; }
}
if [ "$PASSES" = all ]; then
    run_pass fetch "$ARGS" --pmc FETCH_SIZE
    run_pass write "$ARGS" --pmc WRITE_SIZE
    run_pass atom "$ARGS" --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum
    run_pass ta "$ARGS" --pmc TA_FLAT_ATOMIC_WAVEFRONTS_sum
    run_pass valu "$ARGS" --pmc SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE
    python tools/pmc_per_kernel.py "$OUT/fetch" "$OUT/write" "$OUT/atom" "$OUT/ta" "$OUT/valu" > "$OUT/pmc_per_kernel.json"
fi
run_pass trace "$TARGS" --kernel-trace --stats
python tools/prof_summary.py "$OUT/trace" > "$OUT/kernel_stats.csv"
echo "$WL" > "$OUT/workload.txt"
echo ok
