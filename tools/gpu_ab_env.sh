#!/bin/bash
# Bench A/B of prebuilt variants under given environments:
#   RUNS="base:GPU_MAX_HW_QUEUES=4 p4:GPU_MAX_HW_QUEUES=8" BENCH_ARGS="--steps 20" tools/gpu_ab_env.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for rep in $(seq ${REPS:-1}); do
for r in ${RUNS}; do
  v=${r%%:*}; e=${r#*:}; [ "$e" = "$r" ] && e=""
  env $e PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline \
    ${BENCH_ARGS} > gpurun_out/ab/$v.log 2>&1
  rc=$?; printf "%-8s %-22s rc=%d " $v "$e" $rc; grep -o '"value": [0-9.]*' gpurun_out/ab/$v.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
done
