#!/bin/bash
# L2 hit/miss and VALU activity of the cell kernel: one config-2 cell alone vs the
# 64-cell batch (config 5). One rocprofv3 pass per counter group.
# Usage: gpu_cell_l2.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-cell_l2}
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {   # name, workload args..., then the counters after --
    local name=$1; shift
    local wl=()
    while [ "$1" != "--" ]; do wl+=("$1"); shift; done
    shift
    timeout -s KILL 120 rocprofv3 --kernel-include-regex 'k_cell$|k_cell[^_]' --pmc "$@" -f csv -d "$OUT/$name" -o run -- \
        python -u "${wl[@]}" > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -20 "$OUT/$name.log"; exit 1; }
}
ONE=(tools/cell_check.py --reps 1 --graphs 1 --min-n 12000 --engine 0)
BAT=(bench.py --workload batch --steps 1 --warmup 0 --cpu-baseline off)
pass one_tcc "${ONE[@]}" -- TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum
pass bat_tcc "${BAT[@]}" -- TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum
pass one_sq "${ONE[@]}" -- SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU
pass bat_sq "${BAT[@]}" -- SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU
echo ok
