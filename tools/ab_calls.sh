cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-r04s9}; mkdir -p $O
run() {  # name lib config extra...
  local v=$1 lib=$2 c=$3 tag=$4; shift 4
  env PNRT_DEVICE_LIB=$lib timeout -k 10 300 python bench.py --config $c "$@" --no-pmc --no-parity --serial-steps 0 \
    > $O/${v}_${tag}.json 2> $O/${v}_${tag}.err || exit 1
  python3 -c "import json; d=[json.loads(x) for x in open('$O/${v}_${tag}.json') if x.startswith('{')][-1]; print('$v $tag', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  for v in ${VARIANTS:-base}; do
    lib=""; [ $v != base ] && lib=pnraytracing_amd/variants/libpnrt_$v.so
    run $v "$lib" C2 C2_$r || exit 1
    run $v "$lib" C4 C4_$r || exit 1
    run $v "$lib" C5 C5_$r --steps 10 || exit 1
    run $v "$lib" C3 C3_$r || exit 1
    [ -z "$NO_C2I2" ] && { run $v "$lib" C2 C2i2_$r --iters-per-call 2 || exit 1; }
  done
done
exit 0
