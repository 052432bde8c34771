#!/bin/bash
# Shard simulations (N = 8, 4) with 8 hardware queues, as the multi-rank bench runs:
#   VARIANTS="a b" tools/gpu_pipes_n8.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
V=$PWD/pnraytracing_amd/variants
for rep in 1 2; do for p in ${VARIANTS:-p3 p4}; do for n in 8 4; do
  GPU_MAX_HW_QUEUES=8 PNRT_DEVICE_LIB=$V/libpnrt_$p.so timeout -k 10 100 python tools/shard_sim_one.py $n 30 > gpurun_out/hwq.log 2>&1 || exit 1
  echo "q=8 $p $(tail -1 gpurun_out/hwq.log | cut -c1-60)"
done; done; done
