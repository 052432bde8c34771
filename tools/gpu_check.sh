#!/bin/bash
# One GPU-box session: smoke -> gpu parity tests -> bench -> rocprofv3 kernel
# stats -> PMC passes (one counter group per rocprofv3 run, kernel-trace only).
# Every GPU step has its own time limit; a crash/timeout/abort ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }   # 1 = test failures, not a crash
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; ok $rc || exit $rc
  timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log; ok $rc || exit $rc
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_PMC" ] && exit 0
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc/p${i}_default -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/p${i}.log 2>&1
  rc=$?; echo "pmc pass $i [$grp] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
