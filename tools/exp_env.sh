#!/bin/bash
# Interleaved env-variant comparison on the full bench: VARIANTS="X=1;KS_A=2 KS_B=3;..." tools/exp_env.sh out
set -o pipefail
OUT=gpurun_out/${1:-envx}
mkdir -p "$OUT"
IFS=';' read -ra VS <<< "${VARIANTS:-X=1}"
for rep in $(seq ${REPS:-2}); do
    for i in "${!VS[@]}"; do
        e=${VS[$i]}
        env $e timeout -k 10 120 python -u bench.py --steps ${NSTEPS:-20} --warmup 2 --cpu-baseline off ${ARGS} > "$OUT/v${i}_$rep.json" 2>/dev/null || { echo "fail $e"; exit 1; }
        python -c "import json; d=json.load(open('$OUT/v${i}_$rep.json')); s=sorted(d['step_ms']); x=d['solve']; print('%-40s mean %7.2f med %7.2f min %7.2f | sw %5d gus %4d bfr %5d bfl %5d' % ('$e', d['ms_per_step'], s[len(s)//2], s[0], x['sweeps'], x['global_updates'], x['gu_iterations'], x['gu_launches']))"
    done
done
