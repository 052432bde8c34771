#!/bin/bash
# Round-end style refresh on one GPU box: smoke, GPU tests, bench lines C2-C5,
# rocprofv3 kernel stats (C2), PMC traffic passes (C2).  Every GPU step has its
# own time limit; a crash / timeout / abort ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/refresh; mkdir -p $O/pmc
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -1 $O/gpu_tests.log; ok $rc || exit $rc
timeout -k 10 300 python bench.py > $O/bench_C2.log 2>&1; rc=$?; echo "bench C2 rc=$rc"; ok $rc || exit $rc
for c in C3 C4; do
  timeout -k 10 300 python bench.py --config $c --cpu-seconds 6 > $O/bench_$c.log 2>&1; rc=$?; echo "bench $c rc=$rc"; ok $rc || exit $rc
done
timeout -k 10 300 python bench.py --config C5 --steps 10 --no-cpu-baseline > $O/bench_C5.log 2>&1; rc=$?; echo "bench C5 rc=$rc"; ok $rc || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; ok $rc || exit $rc
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $O/pmc/p${i}_default -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc/p${i}.log 2>&1
  rc=$?; echo "pmc pass $i [$grp] rc=$rc"; ok $rc || exit $rc
done
exit 0
