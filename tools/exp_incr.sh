#!/bin/bash
# Incremental (config 4) variants: VARIANTS="X=1;KS_WARM_K=1 KS_WARM_D=8" tools/exp_incr.sh out
set -o pipefail
OUT=gpurun_out/${1:-incrx}
mkdir -p "$OUT"
IFS=';' read -ra VS <<< "${VARIANTS:-X=1}"
for i in "${!VS[@]}"; do
    e=${VS[$i]}
    env $e timeout -k 10 200 python -u bench.py --workload incremental --steps ${STEPS:-5} --warmup 2 --cpu-baseline off ${ARGS} > "$OUT/v$i.json" 2>/dev/null || { echo "fail $e"; exit 1; }
    python -c "
import json; d=json.load(open('$OUT/v$i.json'))
r=d['rounds'][2:]
print('%-36s ms/step %7.2f | solve %s | phases %s sweeps %s' % ('$e', d['ms_per_step'], [x['solve_ms'] for x in r], [x['phases'] for x in r], [x['sweeps'] for x in r]))"
done
