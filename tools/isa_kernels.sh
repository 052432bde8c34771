#!/bin/bash
# Static instruction census of every pt_wf_* kernel (device assembly):
#   tools/isa_kernels.sh [extra hipcc flags]
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fno-gpu-rdc -I include "$@" \
  --cuda-device-only -S pnraytracing_amd/csrc/pnrt_device.hip -o /tmp/isa_all.s 2>/dev/null || exit 1
for k in $(grep -o '^_Z[0-9]*pt_wf_[a-z_]*[^:]*:' /tmp/isa_all.s | tr -d ':'); do
  awk -v k="$k" 'index($0, k":") == 1 {p=1} p && /^\.Lfunc_end/ {p=0} p' /tmp/isa_all.s > /tmp/isa_k.s
  printf "%-60s VALU %4d SALU %4d VMEM %3d  " "$(echo $k | cut -c1-60)" "$(grep -c '^\s*v_' /tmp/isa_k.s)" \
    "$(grep -c '^\s*s_' /tmp/isa_k.s)" "$(grep -c '^\s*\(global\|buffer\|scratch\)_' /tmp/isa_k.s)"
  grep -A30 "\.name:\s*$k\$" /tmp/isa_all.s | grep -E "^\s*\.(vgpr_count|vgpr_spill_count):" | tr -s ' \n' ' '; echo
done
