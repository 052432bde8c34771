#!/bin/bash
# Round-3 session 7: GPU parity suite on the default build, then an alternating
# A/B of two prebuilt variants on C2 (and D2 synchronised per frame).
#   VARIANTS="wr0 wr1" REPS=3 tools/gpu_r03_s7.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq ${REPS:-3}); do
for v in ${VARIANTS}; do
  PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 150 python bench.py --no-cpu-baseline \
    --no-pmc ${BENCH_ARGS} > gpurun_out/ab/${v}_$rep.log 2>&1
  rc=$?; printf "C2 %-8s rc=%d " $v $rc; grep -o '"value": [0-9.]*' gpurun_out/ab/${v}_$rep.log | head -1 | tr '\n' ' '
  python - gpurun_out/ab/${v}_$rep.log <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith('{'):
        d = json.loads(line); k = d.get('kernels_exclusive') or {}
        print(' '.join(f"{n}={v['ms_per_launch']}" for n, v in k.items()))
PY
  [ $rc -eq 0 ] || exit $rc
  if [ -n "$D2" ]; then
    PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 150 python bench.py --no-cpu-baseline \
      --no-pmc --config D2 --sync-per-frame > gpurun_out/ab/${v}_d2_$rep.log 2>&1
    rc=$?; printf "D2 %-8s rc=%d " $v $rc; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/${v}_d2_$rep.log | head -1; echo
    [ $rc -eq 0 ] || exit $rc
  fi
done
done
