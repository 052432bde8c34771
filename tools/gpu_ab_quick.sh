#!/bin/bash
# Bench-only A/B of prebuilt variants (pnraytracing_amd/variants/libpnrt_<name>.so):
#   VARIANTS="base koenv" BENCH_ARGS="--steps 20" tools/gpu_ab_quick.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for rep in $(seq ${REPS:-1}); do
for v in ${VARIANTS}; do
  PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline \
    ${BENCH_ARGS} > gpurun_out/ab/$v.log 2>&1
  rc=$?; printf "%-10s rc=%d " $v $rc; grep -o '"value": [0-9.]*\|"ms_per_launch": [0-9.]*' gpurun_out/ab/$v.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || exit $rc
done
done
