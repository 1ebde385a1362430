#!/bin/bash
# A/B of an env switch on the full bench, interleaved runs on one box: A="ENV=.." B="ENV=.." tools/exp_ab.sh out
set -o pipefail
OUT=gpurun_out/${1:-ab}
mkdir -p "$OUT"
for rep in 1 2 3; do
    for v in A B; do
        e=${!v}
        env $e timeout -k 10 120 python -u bench.py --steps 8 --warmup 1 --cpu-baseline off ${ARGS} > "$OUT/${v}_$rep.json" 2>/dev/null || exit 1
        python -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); s=sorted(d['step_ms']); print('$v', '$e', 'mean', d['ms_per_step'], 'median', s[len(s)//2], 'min', s[0])"
    done
done
