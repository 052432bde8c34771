#!/bin/bash
# A/B of variants on the N=8 shard simulation and the C2 bench: VARIANTS="a b" tools/gpu_grid.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
V=$PWD/pnraytracing_amd/variants
for p in $VARIANTS; do
  for n in 8 4 2; do
    PNRT_DEVICE_LIB=$V/libpnrt_$p.so timeout -k 10 100 python tools/shard_sim_one.py $n 30 > gpurun_out/grid.log 2>&1 || exit 1
    echo "$p $(tail -1 gpurun_out/grid.log | cut -c1-60)"
  done
  PNRT_DEVICE_LIB=$V/libpnrt_$p.so timeout -k 10 100 python bench.py --steps 30 --no-cpu-baseline > gpurun_out/grid.log 2>&1 || exit 1
  echo "$p C2: $(grep -o '"value": [0-9.]*' gpurun_out/grid.log)"
done
