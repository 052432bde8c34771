#!/bin/bash
# PMC passes on one kernel (KREGEX, default the trace kernel) (one counter group per rocprofv3 run, kernel-trace only):
#   PMC_GROUPS=$'SQ_WAVE_CYCLES SQ_BUSY_CYCLES\nTA_BUSY_avr' tools/gpu_pmc_trace.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmct
export TMPDIR=/tmp
if [ -n "$LIST" ]; then timeout -k 5 60 rocprofv3 --list-avail > gpurun_out/pmct/avail.txt 2>&1; echo "list rc=$?"; fi
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "${KREGEX:-pt_wf_trace}" -d gpurun_out/pmct/p${i} -o run \
    --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/pmct/p${i}.log 2>&1
  rc=$?; echo "pmc pass $i [$grp] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<GROUPS
${PMC_GROUPS}
GROUPS
exit 0
