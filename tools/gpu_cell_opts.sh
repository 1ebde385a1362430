#!/bin/bash
# Cell-solver ks_opts settings on the config-2-size goldens (runtime options, one
# process per setting). Usage: gpu_cell_opts.sh TAG 'JSON' ['JSON' ...]
set -o pipefail
OUT=gpurun_out/${1:-cell_opts}; shift
mkdir -p "$OUT"
i=0
for o in "$@"; do
    i=$((i + 1))
    timeout -k 10 150 python -u tools/cell_check.py --reps 3 --min-n 12000 --graphs 3 --engine 0 --opts "$o" \
        > "$OUT/$i.json" 2> "$OUT/$i.log" || { echo "$o failed"; tail -5 "$OUT/$i.log"; exit 1; }
    python - "$OUT/$i.json" "$o" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
print(sys.argv[2], [(r["cell"]["ok"], r["cell"]["ms"], r["cell"]["updates"], r["cell"]["sweeps"]) for r in rows])
PY
done
