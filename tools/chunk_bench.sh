#!/bin/bash
# share_bench.py over call sizes, on a library given by LIB (default: the product one)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/chunkb; mkdir -p $O
for n in ${NS:-8 4 2 1}; do
  for ipc in ${IPCS:-4 8 16}; do
    PNRT_DEVICE_LIB=${LIB:-} timeout -k 10 120 python tools/share_bench.py $n $ipc ${STEPS:-20} ${WARM:-5} >> $O/${TAG:-x}.txt 2>> $O/${TAG:-x}.err || exit 1
  done
done
cat $O/${TAG:-x}.txt
