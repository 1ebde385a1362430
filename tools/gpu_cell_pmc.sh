#!/bin/bash
# PMC passes over one config-2 solve by the cell solver (k_cell), one rocprofv3
# run per pass. Usage: gpu_cell_pmc.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-cell_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
run_pass() {
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 --kernel-include-regex 'k_cell$|k_cell[^_]' "$@" -f csv -d "$OUT/$name" -o run -- \
        python -u tools/cell_check.py --reps 1 --graphs 1 --min-n 10000 --engine 0 > "$OUT/$name.log" 2>&1 \
        || { echo "pass $name failed"; tail -20 "$OUT/$name.log"; exit 1; }
}
if [ "$2" = "valu" ]; then
    run_pass valu --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES
    echo ok; exit 0
fi
run_pass sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM
run_pass sqc --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
run_pass tcp --pmc TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
run_pass lds --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_IFETCH SQ_BUSY_CYCLES
echo ok
