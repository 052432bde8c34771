#!/bin/bash
# Build the product device library of a git revision as an A/B variant:
#   tools/build_rev_variant.sh REV NAME     -> pnraytracing_amd/variants/libpnrt_NAME.so
# (the revision's own csrc/ and include/ are checked out into a temporary tree; same flags as build.py)
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2
T=$(mktemp -d)
git archive "$REV" pnraytracing_amd/csrc include | tar -x -C "$T"
mkdir -p pnraytracing_amd/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -fno-gpu-rdc \
  -fno-slp-vectorize -DPNRT_SRC_HASH="\"rev-$REV\"" -I "$T/include" "$T/pnraytracing_amd/csrc/pnrt_device.hip" \
  -o pnraytracing_amd/variants/libpnrt_$NAME.so
rm -rf "$T"
echo "built $NAME from $REV"
