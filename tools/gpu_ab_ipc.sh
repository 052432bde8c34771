cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ipc; mkdir -p $O; export TMPDIR=/tmp
run() { PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$1.so timeout -k 10 150 python bench.py --no-cpu-baseline --no-pmc --iters-per-call $2 --steps 24 > $O/ab_$1_$2.log 2>&1; rc=$?; printf "%-6s ipc=%s rc=%d " $1 $2 $rc; python -c "import json;d=json.loads(open('$O/ab_$1_$2.log').read().strip().splitlines()[-1]);k=d.get('kernels_exclusive',{});print(d['value'],d['ms_per_step'],' '.join(f'{n}={e[\"ms_per_launch\"]}' for n,e in k.items()))" 2>/dev/null || tail -3 $O/ab_$1_$2.log; return $rc; }
for rep in 1 2; do
  run base 2 || exit 1; run mc16 4 || exit 1; run mc16h 4 || exit 1; run base 4 || exit 1
done
