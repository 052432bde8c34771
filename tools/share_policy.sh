#!/bin/bash
# rank 0's share at bench.py's own call sizes (N = 8 / 4 / 2 / 1: 16 / 16 / 8 / 4 iterations), 2 rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-sharep}; mkdir -p $O
for r in 1 2; do
  for spec in "8 16" "4 16" "2 8" "1 4"; do
    set -- $spec
    timeout -k 10 120 python tools/share_bench.py $1 $2 20 5 >> $O/share.txt 2>> $O/share.err || exit 1
  done
done
cat $O/share.txt
