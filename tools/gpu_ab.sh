#!/bin/bash
# Quick GPU check of a change: the parity tests, then an interleaved options A/B.
# Usage: gpu_ab.sh TAG "A opts" "B opts" [pytest -k expr]
set -o pipefail
TAG=${1:-ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
K=${4:-parity}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" \
    > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python -u tools/ab_opts.py --a "$2" --b "$3" ${AB_ARGS} > $OUT/ab.txt 2> $OUT/ab.err \
    || { echo "ab failed"; tail -20 $OUT/ab.err; cat $OUT/ab.txt; exit 1; }
grep -v '^{' $OUT/ab.txt
