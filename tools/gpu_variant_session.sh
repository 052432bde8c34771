#!/bin/bash
# One GPU session for kernel variants (pnraytracing_amd/variants/libpnrt_<name>.so):
#   1. parity: the full-size + parity GPU tests against every variant in CHECK
#      (variants that can change results: layout / control-flow changes)
#   2. A/B: bench.py (no CPU baseline, no PMC) for every variant in VARIANTS, REPS rounds
#   3. optional census (CENSUS=1) with the stats variant
# Every GPU step has its own time limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/vs; mkdir -p $O
export TMPDIR=/tmp
for v in ${CHECK}; do
  PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 300 python -u -m pytest -x -q \
    --timeout ${CHECK_TIMEOUT:-200} --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py \
    ${PYTEST_K} > $O/check_$v.log 2>&1
  rc=$?; echo "check $v rc=$rc $(tail -1 $O/check_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -rs --timeout 300 --timeout-method thread $TESTS > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || exit $rc
fi
for rep in $(seq ${REPS:-1}); do
  for v in ${VARIANTS}; do
    PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 150 python bench.py --no-cpu-baseline \
      --no-pmc ${BENCH_ARGS} > $O/ab_$v.log 2>&1
    rc=$?; printf "%-10s rc=%d " $v $rc
    python -c "import json,sys;d=json.loads(open('$O/ab_$v.log').read().strip().splitlines()[-1]);k=d.get('kernels_exclusive',{});print(d['value'],d['ms_per_step'],' '.join(f'{n}={e[\"ms_per_launch\"]}' for n,e in k.items()))" 2>/dev/null || echo
    [ $rc -eq 0 ] || exit $rc
  done
done
if [ -n "$CENSUS" ]; then
  timeout -k 10 600 python tools/census.py ${CENSUS_CONFIGS:-C2} > $O/census.log 2>&1; rc=$?; echo "census rc=$rc"; cat $O/census.log
  cp profiles/census.json $O/census.json
fi
exit 0
