#!/bin/bash
# A/B of frames per call / batch size / hardware queues on the bench (C2, N = 1):
#   run <variant lib> <iters per call> <GPU_MAX_HW_QUEUES or "-">
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ipc; mkdir -p $O; export TMPDIR=/tmp
run() {
  local q=""; [ "$3" != "-" ] && q="GPU_MAX_HW_QUEUES=$3"
  env $q PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$1.so timeout -k 10 150 python bench.py --no-cpu-baseline \
    --no-pmc --iters-per-call $2 --steps 24 ${BENCH_ARGS} > $O/ab_$1_$2_$3.log 2>&1
  local rc=$?; printf "%-6s ipc=%s hwq=%s rc=%d " $1 $2 $3 $rc
  python -c "import json;d=json.loads([l for l in open('$O/ab_$1_$2_$3.log') if l.startswith('{')][-1]);k=d.get('kernels_exclusive',{});print(d['value'],d['ms_per_step'],' '.join(f'{n}={e[\"ms_per_launch\"]}' for n,e in k.items()))" 2>/dev/null || tail -3 $O/ab_$1_$2_$3.log
  return $rc
}
for rep in $(seq ${REPS:-2}); do
  for spec in ${RUNS:-"base:2:-" "mc16:4:-" "mc16:4:8" "base:2:8"}; do
    IFS=: read -r v i q <<< "$spec"; run $v $i $q || exit 1
  done
done
