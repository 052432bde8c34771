#!/bin/bash
# Round-3 session 16: shard simulation (per-rank rates at N = 1/2/4/8) and the
# 2-rank gloo rehearsal of the multi-rank bench, on the final build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s16
export TMPDIR=/tmp
timeout -k 10 300 python tools/shard_sim.py 20 16 > gpurun_out/s16/shard_sim.txt 2>&1
rc=$?; echo "shard sim rc=$rc"; grep "^N=" gpurun_out/s16/shard_sim.txt; [ $rc -eq 0 ] || exit $rc
NPROC=2 bash tools/dist_rehearsal.sh > gpurun_out/s16/rehearsal_n2.txt 2>&1
rc=$?; echo "rehearsal N=2 rc=$rc"; cat gpurun_out/s16/rehearsal_n2.txt; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/dist_n2.log gpurun_out/s16/dist_n2.json
