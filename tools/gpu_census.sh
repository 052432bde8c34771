#!/bin/bash
# Serialised per-kernel timing (one call in flight) and the trace census:
#   libs built by: tools/build_variants.sh serial:"-DWF_PIPES=1" stats:"-DWF_PIPES=1 -DWF_STATS=1"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/census
export TMPDIR=/tmp
V=pnraytracing_amd/variants
PNRT_DEVICE_LIB=$PWD/$V/libpnrt_stats.so timeout -k 10 200 python bench.py --steps 2 --warmup 0 --no-cpu-baseline ${BENCH_ARGS} \
  > gpurun_out/census/stats.log 2>&1
rc=$?; echo "stats rc=$rc"; grep "trace stats" gpurun_out/census/stats.log | head -8; [ $rc -eq 0 ] || exit $rc
PNRT_DEVICE_LIB=$PWD/$V/libpnrt_serial.so timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/census/prof -o run \
  --output-format csv -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/census/serial.log 2>&1
rc=$?; echo "serial rc=$rc"; tail -1 gpurun_out/census/serial.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
