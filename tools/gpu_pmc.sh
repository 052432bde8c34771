#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only, no sys/runtime trace).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline"}
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  for v in ${VARIANTS:-v2 v1}; do
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc/p${i}_$v -o run --output-format csv -- \
      python bench.py $ARGS --kernel $v > gpurun_out/pmc/p${i}_$v.log 2>&1
    rc=$?; echo "pass $i [$grp] $v rc=$rc"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  done
done <<GROUPS
${PMC_GROUPS}
GROUPS
