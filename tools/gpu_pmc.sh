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
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
GROUPS
