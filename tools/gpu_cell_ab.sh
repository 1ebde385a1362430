#!/bin/bash
# Cell-solver variants (KS_LIB_VARIANT) on the config-2-size goldens, interleaved.
# Usage: gpu_cell_ab.sh TAG VARIANT... (base = the default build)
set -o pipefail
OUT=gpurun_out/${1:-cell_ab}; shift
mkdir -p "$OUT"
for v in "$@"; do
    if [ "$v" = base ]; then unset KS_LIB_VARIANT; else export KS_LIB_VARIANT=$v; fi
    timeout -k 10 150 python -u tools/cell_check.py --reps 3 --min-n 12000 --graphs 3 --engine 0 --log 1 \
        > "$OUT/$v.json" 2> "$OUT/$v.log" || { echo "$v failed"; tail -5 "$OUT/$v.log"; exit 1; }
    python - "$OUT/$v.json" "$v" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
print(sys.argv[2], [(r["cell"]["ok"], r["cell"]["ms"], r["cell"]["bf_rounds"], r["cell"]["sweeps"]) for r in rows])
PY
done
