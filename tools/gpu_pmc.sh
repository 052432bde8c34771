#!/bin/bash
# PMC passes on the default library: one counter group per rocprofv3 run
# (kernel-trace only, never combined with sys/runtime traces).
#   tools/gpu_pmc.sh <groups-file> [out-dir]     (one group per line)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=${2:-gpurun_out/pmcdiag}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p${i}_default -o run --output-format csv -- \
    python bench.py $ARGS > $OUT/p${i}.log 2>&1
  rc=$?; echo "pass $i [$grp] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done < "$1"
exit 0
