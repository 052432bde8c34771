#!/bin/bash
# Shard-simulation A/B of prebuilt variants (per-rank rates at N = 1/2/4/8):
#   VARIANTS="base ppb1k" REPS=2 tools/gpu_shard_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/shab; mkdir -p $O
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
for rep in $(seq ${REPS:-1}); do
  for v in ${VARIANTS}; do
    PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 200 python tools/shard_sim.py ${STEPS:-30} ${FPC:-4} \
      > $O/$v.txt 2>&1
    rc=$?; printf "%-10s rc=%d " $v $rc; grep -o "N=[0-9]: .*per rank" $O/$v.txt | sed 's/rank-0 rows [0-9]*, //' | tr '\n' ' '; echo
    [ $rc -eq 0 ] || exit $rc
  done
done
