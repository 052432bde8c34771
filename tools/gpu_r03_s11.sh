#!/bin/bash
# Round-3 session 11: tiled shade with LDS-DMA prefetch of the next tile's state
# records (WF_SHADE_TILES 2 / 4): parity of each variant on the parity + full-size
# GPU tests, then an alternating C2 A/B against the default build (base).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s11
export TMPDIR=/tmp
for v in ${PARITY:-sh2 sh4}; do
  PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 400 python -u -m pytest \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/s11/parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc"; tail -2 gpurun_out/s11/parity_$v.log; [ $rc -eq 0 ] || exit $rc
done
SKIP_TESTS=1 VARIANTS="${VARIANTS:-base sh2 sh4}" REPS=${REPS:-3} D2=1 bash tools/gpu_r03_s7.sh
