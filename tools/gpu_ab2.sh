#!/bin/bash
# Options A/B over configs 2, 3 and 4 after the parity tests. Usage: gpu_ab2.sh TAG "A opts" "B opts"
set -o pipefail
TAG=${1:-ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${K:-parity}" \
    > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/ab_opts.py --config config2 --a "$2" --b "$3" --solves ${SOLVES:-20} --rounds 0 | grep -v '^{' || exit 1
timeout -k 10 300 python tools/ab_opts.py --config config3 --a "$2" --b "$3" --solves ${SOLVES:-20} --rounds ${ROUNDS:-10} | grep -v '^{' || exit 1
