#!/bin/bash
# Build the library of git revision REV as ksched_amd/libksmcmf_<TAG>.so (A/B baselines).
# Usage: tools/build_rev.sh REV TAG
set -euo pipefail
REV=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p "$T/ksched_amd/csrc" "$T/include"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" ksched_amd/csrc/); do
    git -C "$ROOT" show "$REV:$f" > "$T/$f"
done
git -C "$ROOT" show "$REV:include/ksmcmf.h" > "$T/include/ksmcmf.h"
cd "$T/ksched_amd/csrc"
SRCS=""
for f in ks_engine.hip ks_cell.hip ks_store.hip ks_sched.hip ks_batch.hip ks_host.cpp; do
    [ -f "$f" ] && SRCS="$SRCS $f"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-function -I"$T/include" \
    $SRCS -ldl -o "$ROOT/ksched_amd/libksmcmf_$TAG.so"
rm -rf "$T"
