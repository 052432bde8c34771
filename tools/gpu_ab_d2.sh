#!/bin/bash
# A/B of library variants on the reference dispatch shape (D2 / D3, synchronised per frame)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/abd2; mkdir -p $O
export TMPDIR=/tmp
for rep in $(seq ${REPS:-2}); do
  for v in ${VARIANTS}; do
    for c in ${CONFIGS:-D2 D3}; do
      PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 120 python bench.py --config $c --sync-per-frame \
        --steps 240 --warmup 16 --no-cpu-baseline --no-pmc --serial-steps 0 ${BENCH_ARGS} > $O/${c}_$v.json 2> $O/${c}_$v.err
      rc=$?; printf "%-4s %-8s rc=%d " $c $v $rc
      python -c "import json;d=[json.loads(x) for x in open('$O/${c}_$v.json') if x.startswith('{')][-1];print(d['value'],d['ms_per_step'],d['kernels'].get('trace',{}).get('ms_per_launch'))"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
exit 0
