#!/bin/bash
# Library-variant A/B: default library (a) vs KS_LIB_VARIANT=$1 (b), same options, configs 2, 3, 4.
set -o pipefail
export TMPDIR=/tmp
V=$1; shift
for cfg in config2 config3; do
  timeout -k 10 300 python tools/ab_variant.py --variant "$V" --config $cfg --solves ${SOLVES:-16} "$@" || exit 1
done
timeout -k 10 300 python tools/ab_variant.py --variant "$V" --solves 0 --rounds ${ROUNDS:-10} "$@" || exit 1
