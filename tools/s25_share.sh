#!/bin/bash
# share_bench.py over call sizes for N = 8 / 4 (session 25)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05s25; mkdir -p $O
for r in 1 2; do
  for spec in "8 10" "8 16" "8 20" "8 12" "4 10" "4 16" "4 20"; do
    set -- $spec
    timeout -k 10 120 python tools/share_bench.py $1 $2 20 5 >> $O/share.txt 2>> $O/share.err || exit 1
  done
done
cat $O/share.txt
