#!/bin/bash
# Solver parameter sweep on the GPU box: bench lines for each (workload, alpha, gu_interval, warm).
# Usage: param_sweep.sh TAG "workload:alpha:gu:warm" ...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for cfg in "$@"; do
  IFS=: read wl a gi w <<< "$cfg"
  timeout -k 10 150 python -u bench.py --workload $wl --alpha $a --gu-interval $gi --warm $w --steps 6 --warmup 1 \
      --cpu-baseline off > $O/$wl-$a-$gi-$w.json 2> $O/$wl-$a-$gi-$w.err || { echo "fail $cfg"; tail -5 $O/$wl-$a-$gi-$w.err; exit 1; }
  python - "$O/$wl-$a-$gi-$w.json" "$cfg" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
rs = d.get("rounds")
extra = [(r["solve_ms"], r["phases"], r["sweeps"], r["rebuilt"]) for r in rs[1:]] if rs else d.get("step_ms")
print(sys.argv[2], d["ms_per_step"], extra, flush=True)
PY
done
