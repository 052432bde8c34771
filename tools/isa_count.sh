#!/bin/bash
# Static instruction census of the trace kernel (device assembly), for A/B of code shape:
#   tools/isa_count.sh [extra hipcc flags]
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize -fno-gpu-rdc -I include "$@" \
  --cuda-device-only -S pnraytracing_amd/csrc/pnrt_device.hip -o /tmp/isa_count.s 2>/dev/null || exit 1
# the instantiation C2 runs (no table leaves)
K=$(grep -o '^_Z11pt_wf_traceILi8ELb0ELb0EE[A-Za-z0-9_]*:' /tmp/isa_count.s | head -1)
awk -v k="$K" 'index($0, k) == 1, /^\.Lfunc_end/' /tmp/isa_count.s > /tmp/isa_trace.s
echo "trace kernel: VALU $(grep -c '^\s*v_' /tmp/isa_trace.s)  SALU $(grep -c '^\s*s_' /tmp/isa_trace.s)  branches $(grep -c 's_cbranch' /tmp/isa_trace.s)  VMEM $(grep -c '^\s*\(global\|buffer\|scratch\)_' /tmp/isa_trace.s)"
grep -A25 "\.name:.*${K%:}" /tmp/isa_count.s | grep -E "vgpr_count|vgpr_spill" | tr '\n' ' '; echo
# the identity-permutation step loop (the last depth-2 loop of the kernel) to the kernel's end
L=$(grep -n "This Loop Header: Depth=2" /tmp/isa_trace.s | tail -1 | cut -d: -f1)
tail -n +$L /tmp/isa_trace.s > /tmp/isa_loop.s
echo "ident step loop: VALU $(grep -c '^\s*v_' /tmp/isa_loop.s)  SALU $(grep -c '^\s*s_' /tmp/isa_loop.s)  v_cndmask $(grep -c 'v_cndmask' /tmp/isa_loop.s)"
