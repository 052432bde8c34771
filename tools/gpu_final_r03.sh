#!/bin/bash
# Round-3 end-of-round measurement on one GPU box, in dependency order:
#   smoke -> GPU tests -> trace census of these sources (profiles/census.json, read by
#   bench.py) -> bench lines C2..C5 (live PMC, calibrated traffic, exclusive times) ->
#   profiles/pmc.json from the N = 1 lines (read by N > 1 lines) -> the reference's
#   dispatch shape D2 / D3 -> rocprofv3 stats of the --serial and default C2 commands.
# Needs pnraytracing_amd/variants/libpnrt_stats.so built from the same sources:
#   tools/build_variants.sh stats:"-DWF_PIPES=1 -DWF_STATS=1"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/final3}; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$SECONDS; "$@"; local rc=$?; echo "$name rc=$rc ($((SECONDS - t0)) s)"; [ $rc -eq 0 ] || exit $rc; }
if [ -z "$SKIP_TESTS" ]; then
  step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  step gpu-tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -3 $O/gpu_tests.log
fi
step census timeout -k 10 600 python tools/census.py C2 C3 C4 C5 > $O/census.log 2>&1
cp profiles/census.json $O/census.json
for c in ${CONFIGS:-C2 C3 C4 C5}; do
  extra=""; [ $c = C5 ] && extra="--steps 10"; [ $c != C2 ] && extra="$extra --cpu-seconds 6"
  step bench-$c timeout -k 10 600 python bench.py --config $c $extra > $O/bench_$c.json 2> $O/bench_$c.err
  python - $O/bench_$c.json <<'PY'
import json, sys
d = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")][-1]; r = d["roofline"]
print(" ", d["config"]["workload"][:20], d["value"], d["ms_per_step"], r["bound"], r["frac"], r["traffic"], r["kernel_ms"])
PY
done
step record timeout -k 10 60 python tools/record_pmc.py $O/bench_C2.json $O/bench_C3.json $O/bench_C4.json $O/bench_C5.json
cp profiles/pmc.json $O/pmc.json
for c in D2 D3; do
  for sync in "" "--sync-per-frame"; do
    step $c$sync timeout -k 10 200 python bench.py --config $c $sync --steps 240 --warmup 16 --no-cpu-baseline --no-pmc --serial-steps 0 --kernel-times > $O/${c}${sync}.json 2> $O/${c}${sync}.err
  done
done
step prof-serial timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_serial -o run --output-format csv -- \
  python bench.py --steps 8 --warmup 4 --no-cpu-baseline --no-pmc --serial > $O/prof_serial.json 2> $O/prof_serial.err
step prof-pipe timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_pipe -o run --output-format csv -- \
  python bench.py --steps 8 --warmup 4 --no-cpu-baseline --no-pmc > $O/prof_pipe.json 2> $O/prof_pipe.err
exit 0
