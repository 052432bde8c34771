#!/bin/bash
# Build libpnrt variants (compile-time switches) for GPU A/B runs:
#   tools/build_variants.sh name:"-DFOO=1 -DBAR=2" ...
cd "$(dirname "$0")/.."
mkdir -p pnraytracing_amd/variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -fno-slp-vectorize -DPNRT_DIAG_BUILD \
    -fno-gpu-rdc -I include $flags pnraytracing_amd/csrc/pnrt_device.hip -o pnraytracing_amd/variants/libpnrt_$name.so \
    || exit 1
  echo "built $name ($flags)"
done
