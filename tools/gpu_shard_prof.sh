#!/bin/bash
# Shard simulation (per-rank rates at N = 1/2/4/8) + a kernel trace of rank 0's
# N=8 share with its per-class timeline.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/shard}; mkdir -p $O
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
timeout -k 10 300 python tools/shard_sim.py 30 > $O/shard_sim.txt 2>&1; rc=$?; cat $O/shard_sim.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/n8 -o run --output-format csv -- python tools/shard_sim_one.py 8 30 > $O/n8.log 2>&1
rc=$?; echo "n8 prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(ls $O/n8/*kernel_trace.csv $O/n8/*/*kernel_trace.csv 2>/dev/null | head -1)
python tools/timeline2.py $f 60 | tee $O/n8_timeline.txt
