#!/bin/bash
# A/B of bench.py's iterations per call on one GPU (IPCS, CONFIGS, ROUNDS), no PMC / parity / serial steps:
#   IPCS="4 8" CONFIGS="C2 C3" ROUNDS=3 [LIB=variants/libpnrt_x.so] TAG=name bash tools/ab_ipc.sh   (GPU box)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-ab_ipc}; mkdir -p $O
for r in $(seq 1 ${ROUNDS:-3}); do
  for c in ${CONFIGS:-C2}; do
    for ipc in ${IPCS:-4 8}; do
      f=$O/ab_${c}_ipc${ipc}_$r
      PNRT_DEVICE_LIB=${LIB:-} timeout -k 10 200 python bench.py --config $c --no-pmc --no-parity --serial-steps 0 --no-cpu-baseline \
        --iters-per-call $ipc ${AB_ARGS:-} > $f.json 2> $f.err || exit 1
      python3 -c "import json; d=[json.loads(l) for l in open('$f.json') if l.startswith('{')][-1]; print('$c ipc $ipc round $r', d['value'], d['ms_per_step'])" | tee -a $O/ab_ipc.txt
    done
  done
done
