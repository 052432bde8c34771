#!/bin/bash
# Round-3 session 10: non-temporal ray-prefetch A/B, then gloo rehearsals of the
# multi-rank bench (2 and 4 ranks on the box's one GPU) on the final build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s10
export TMPDIR=/tmp
SKIP_TESTS=1 VARIANTS="${VARIANTS:-base pf64nt pf16nt}" REPS=${REPS:-3} bash tools/gpu_r03_s7.sh || exit $?
for np in 2 4; do
  NPROC=$np bash tools/dist_rehearsal.sh > gpurun_out/s10/rehearsal_n$np.txt 2>&1
  rc=$?; echo "rehearsal N=$np rc=$rc"; cat gpurun_out/s10/rehearsal_n$np.txt; [ $rc -eq 0 ] || exit $rc
  cp gpurun_out/dist_n2.log gpurun_out/s10/dist_n${np}.json
done
