#!/bin/bash
# Options sweep: each variant against the defaults on config 3 (and config 4 rounds).
set -o pipefail
export TMPDIR=/tmp
for v in "$@"; do
  echo "== $v"
  timeout -k 10 300 python tools/ab_opts.py --config config3 --a "" --b "$v" --solves ${SOLVES:-16} --rounds ${ROUNDS:-6} | grep -v '^{' || exit 1
done
