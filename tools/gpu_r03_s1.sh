#!/bin/bash
# Round-3 session 1: smoke, the whole GPU suite (incl. the trace-fault test), then
# same-box A/B of the current library against the round-2 build (REPS rounds, C2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03s1; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$SECONDS; "$@"; local rc=$?; echo "$name rc=$rc ($((SECONDS - t0)) s)"; [ $rc -eq 0 ] || exit $rc; }
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step gpu-tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -4 $O/gpu_tests.log
cp pnraytracing_amd/libpnrt.so pnraytracing_amd/variants/libpnrt_cur.so
for rep in $(seq ${REPS:-3}); do
  for v in ${VARIANTS:-cur r02}; do
    PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 150 python bench.py --no-cpu-baseline \
      --no-pmc ${BENCH_ARGS} > $O/ab_$v.log 2>&1
    rc=$?; printf "%-8s rc=%d " $v $rc
    python -c "import json;d=json.loads(open('$O/ab_$v.log').read().strip().splitlines()[-1]);k=d.get('kernels_exclusive') or {};print(d['value'],d['ms_per_step'],' '.join(f'{n}={e[\"ms_per_launch\"]}' for n,e in k.items()))" 2>/dev/null || tail -3 $O/ab_$v.log
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
