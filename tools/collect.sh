#!/bin/bash
# Copy a round's measurement (tools/gpu_round.sh TAG) from gpurun_out/ into
# profiles/ under PREFIX: bench lines, per-workload PMC traffic (pmc_traffic.py,
# calibration carried from profiles/r03m_pmc_traffic.json) and kernel stats, the GPU
# suite log and smoke output.
# Usage: collect.sh TAG PREFIX DATE
set -e
TAG=$1; P=$2; DATE=$3
IN=gpurun_out/$TAG
for wl in config3 config2 config4 config5; do
    [ -f "$IN/bench_$wl.json" ] && tail -1 "$IN/bench_$wl.json" > "profiles/${P}_bench_$wl.json"
    d=gpurun_out/${TAG}_pmc_$wl
    if [ -d "$d/fetch" ]; then
        python tools/pmc_traffic.py "$d" profiles/r03m_pmc_traffic.json "$DATE" > "profiles/${P}_pmc_$wl.json"
        cp "$d/kernel_stats.csv" "profiles/${P}_kernel_stats_$wl.csv"
    fi
done
[ -f gpurun_out/$TAG/pytest_gpu.log ] && cp gpurun_out/$TAG/pytest_gpu.log "profiles/${P}_pytest_gpu.log"
[ -f gpurun_out/$TAG/smoke.log ] && cp gpurun_out/$TAG/smoke.log "profiles/${P}_smoke.log"
ls -la profiles/${P}_*
