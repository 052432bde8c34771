cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r04s11}; mkdir -p $O
for r in 1 2; do
  for v in ${VARIANTS:-base}; do
    lib=""; [ $v != base ] && lib=pnraytracing_amd/variants/libpnrt_$v.so
    env PNRT_DEVICE_LIB=$lib GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/shard_sim.py 30 16 > $O/shard_${v}_$r.txt 2>&1 || exit 1
    echo "== $v $r"; grep "^N=" $O/shard_${v}_$r.txt
    [ -n "$NO_C2I2" ] && continue
    env PNRT_DEVICE_LIB=$lib timeout -k 10 300 python bench.py --config C2 --iters-per-call 2 --no-pmc --no-parity --serial-steps 0 \
      > $O/${v}_C2i2_$r.json 2> $O/${v}_C2i2_$r.err || exit 1
    python3 -c "import json; d=[json.loads(x) for x in open('$O/${v}_C2i2_$r.json') if x.startswith('{')][-1]; print('$v C2i2', d['value'])"
  done
done
exit 0
