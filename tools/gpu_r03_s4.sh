#!/bin/bash
# Round-3 session 4: trace census of the current sources, the default C2 line
# (live PMC + calibrated traffic), its record in profiles/pmc.json, and bench.py's
# multi-rank path rehearsed with gloo ranks sharing the box's GPU (2 and 4 ranks).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03s4; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$SECONDS; "$@"; local rc=$?; echo "$name rc=$rc ($((SECONDS - t0)) s)"; [ $rc -eq 0 ] || exit $rc; }
step census timeout -k 10 600 python tools/census.py ${CONFIGS:-C2 C3 C4 C5} > $O/census.log 2>&1
cp profiles/census.json $O/census.json
step bench-C2 timeout -k 10 600 python bench.py > $O/bench_C2.json 2> $O/bench_C2.err
step record timeout -k 10 60 python tools/record_pmc.py $O/bench_C2.json
cp profiles/pmc.json $O/pmc.json
for np in 2 4; do
  step rehearsal-$np env NPROC=$np ARGS="--steps 8 --warmup 4 --no-cpu-baseline --no-pmc --config C2" timeout -k 10 700 bash tools/dist_rehearsal.sh > $O/rehearsal_$np.log 2>&1
  cat $O/rehearsal_$np.log
  cp gpurun_out/dist_n2.log $O/dist_n${np}_line.log
done
step D2-times timeout -k 10 120 python bench.py --config D2 --sync-per-frame --kernel-times --steps 240 --warmup 16 --no-cpu-baseline --no-pmc --serial-steps 0 > $O/D2_times.json 2> $O/D2_times.err
exit 0
