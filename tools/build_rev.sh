#!/bin/bash
# Build the HIP engine of an earlier git revision as quadrupedwholebodycontroller_amd/libwbc_hip_<name>.so
# (A/B timing against the working tree with tools/variants.py).  Usage: tools/build_rev.sh <rev> <name>
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" quadrupedwholebodycontroller_amd/csrc include | tar -x -C "$T"
make -C "$T/quadrupedwholebodycontroller_amd/csrc" -j8 OUT="$ROOT/quadrupedwholebodycontroller_amd/libwbc_hip_$NAME.so" \
    "$ROOT/quadrupedwholebodycontroller_amd/libwbc_hip_$NAME.so" ROOT="$T" > /dev/null
rm -rf "$T"
echo "built libwbc_hip_$NAME.so from $REV"
