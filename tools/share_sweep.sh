#!/bin/bash
# rank 0's share timed as bench.py times it (tools/share_bench.py) over "N ipc" pairs, ROUNDS rounds, in
# each of MODES (plain: the calls alone; collective: bench.py's gather path through a one-rank RCCL group):
#   SPECS="8 20;4 20;2 20;1 20" MODES="plain collective" ROUNDS=2 [LIB=variants/libpnrt_x.so] TAG=name \
#     bash tools/share_sweep.sh
# (the default SPECS are bench.py's own call sizes for --steps 20; profiles/r06/h/)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-share}; mkdir -p $O
IFS=';' read -ra specs <<< "${SPECS:-8 20;4 20;2 20;1 20}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in "${specs[@]}"; do
    for mode in ${MODES:-plain collective}; do
      set -- $spec
      flag=""; [ $mode = collective ] && flag="--collective"
      PNRT_DEVICE_LIB=${LIB:-} timeout -k 10 120 python tools/share_bench.py $1 $2 ${STEPS:-20} ${WARM:-5} $flag \
        >> $O/share.txt 2>> $O/share.err || exit 1
    done
  done
done
cat $O/share.txt
