#!/bin/bash
# End-of-session measurement on one GPU box, in dependency order:
#   smoke -> GPU tests -> trace census of these sources (profiles/census.json, read
#   by bench.py) -> bench lines C2-C5 (live PMC passes, exclusive kernel times) ->
#   rocprofv3 kernel stats (pipelined + serial) and timeline of the C2 command.
# Needs pnraytracing_amd/variants/libpnrt_stats.so built from the same sources:
#   tools/build_variants.sh stats:"-DWF_PIPES=1 -DWF_STATS=1"
# Every GPU step has its own time limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/final}; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$SECONDS; "$@"; local rc=$?; echo "$name rc=$rc ($((SECONDS - t0)) s)" >&2; [ $rc -eq 0 ] || exit $rc; }
if [ -z "$SKIP_TESTS" ]; then
  step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  step gpu-tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -3 $O/gpu_tests.log
fi
if [ -n "$FUZZ" ]; then   # widened fuzz campaign: FUZZ random scenes x 3 kernel modes vs the oracle
  step fuzz env PNRT_FUZZ_SEEDS=$FUZZ timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1
  tail -1 $O/fuzz.log
fi
step census timeout -k 10 600 python tools/census.py ${CONFIGS:-C2 C3 C4 C5} > $O/census.log 2>&1
cp profiles/census.json $O/census.json
for c in ${CONFIGS:-C2 C3 C4 C5}; do
  extra=""; [ $c = C5 ] && extra="--steps 10"; [ $c != C2 ] && extra="$extra --cpu-seconds 6"
  step bench-$c timeout -k 10 600 python bench.py --config $c $extra > $O/bench_$c.json 2> $O/bench_$c.err
  python -c "import json;d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]);r=d['roofline'];print('  $c', d['value'], d['ms_per_step'], 'frac', r['frac'], 'requested', (r.get('requested') or {}).get('frac_of_l2'))"
done
[ -n "$SKIP_PROF" ] && exit 0
OUT=$O/prof step prof bash tools/gpu_prof.sh > $O/prof.log 2>&1
tail -20 $O/prof.log
exit 0
