#!/bin/bash
# drain-tail census of the lone 512x512 frame (WF_TIMING build), D2 and C2 share-size
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03s6; mkdir -p $O
export TMPDIR=/tmp
PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_timing.so timeout -k 10 120 python bench.py --config D2 --sync-per-frame --steps 8 --warmup 2 --no-cpu-baseline --no-pmc --serial-steps 0 > $O/D2_timing.json 2> $O/D2_timing.err
echo "timing rc=$?"; grep "trace timing" $O/D2_timing.err | tail -8
exit 0
