#!/bin/bash
# config-4 parameter probe: ms per round for alpha / gu-interval settings
set -o pipefail
mkdir -p gpurun_out/inc
for a in "--alpha 8" "--alpha 4" "--alpha 16" "--gu-interval 16" "--gu-interval 32"; do
  timeout -k 10 200 python -u bench.py --workload incremental --steps 5 --warmup 1 --cpu-baseline off $a > gpurun_out/inc/x.json 2>/dev/null \
    && python -c "import json; d=json.load(open('gpurun_out/inc/x.json')); print('$a', d['ms_per_step'], [(r['round'], round(r['solve_ms']), r['phases'], r['sweeps'], r['updates']) for r in d['rounds']])" || exit 1
done
