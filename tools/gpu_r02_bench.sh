#!/bin/bash
# Round-2 measurement on one GPU box: default bench lines (live PMC passes +
# exclusive kernel times inside bench.py) for C2-C5, then the trace census.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02; mkdir -p $O
export TMPDIR=/tmp
for c in ${CONFIGS:-C2 C3 C4 C5}; do
  extra=""; [ $c = C5 ] && extra="--steps 10"; [ $c != C2 ] && extra="$extra --cpu-seconds 6"
  timeout -k 10 600 python bench.py --config $c $extra > $O/bench_$c.json 2> $O/bench_$c.err
  rc=$?; echo "bench $c rc=$rc"; tail -c 600 $O/bench_$c.json; [ $rc -eq 0 ] || exit $rc
done
if [ -z "$NO_CENSUS" ]; then
  timeout -k 10 600 python tools/census.py ${CONFIGS:-C2 C3 C4 C5} > $O/census.log 2>&1; rc=$?; echo "census rc=$rc"; cat $O/census.log; [ $rc -eq 0 ] || exit $rc
  cp profiles/census.json $O/census.json
fi
exit 0
