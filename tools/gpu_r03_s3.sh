#!/bin/bash
# Round-3 session 3: the whole GPU suite, the idle-call trace grid sweep on the
# reference dispatch shape (D2 / D3, synchronised per frame and pipelined), the
# default C2 bench line, and the rocprofv3 stats of the --serial command.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03s3; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$SECONDS; "$@"; local rc=$?; echo "$name rc=$rc ($((SECONDS - t0)) s)"; [ $rc -eq 0 ] || exit $rc; }
val() { python - "$1" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); k = d.get("kernels") or {}
        print(d["value"], d["ms_per_step"], " ".join(f"{n}={e['ms_per_launch']}x{e['launches_per_step']}" for n, e in k.items()))
PY
}
step gpu-tests timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
for rep in 1 2; do
  for v in cur alone128 alone512 alone1024 r02; do
    for c in D2 D3; do
      step $c-$v env PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 120 python bench.py --config $c --sync-per-frame --steps 240 --warmup 16 --no-cpu-baseline --no-pmc --serial-steps 0 > $O/${c}_$v.json 2> $O/${c}_$v.err
      echo "  $c sync $v $(val $O/${c}_$v.json)"
    done
  done
done
for v in cur r02; do
  step D2p-$v env PNRT_DEVICE_LIB=$PWD/pnraytracing_amd/variants/libpnrt_$v.so timeout -k 10 120 python bench.py --config D2 --steps 240 --warmup 16 --no-cpu-baseline --no-pmc --serial-steps 0 > $O/D2p_$v.json 2> $O/D2p_$v.err
  echo "  D2 pipelined $v $(val $O/D2p_$v.json)"
done
step bench-C2 timeout -k 10 600 python bench.py > $O/bench_C2.json 2> $O/bench_C2.err
echo "  C2 $(val $O/bench_C2.json)"
step prof-serial timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/serial -o run --output-format csv -- \
  python bench.py --steps 8 --warmup 4 --no-cpu-baseline --no-pmc --serial > $O/serial.json 2> $O/serial.err
exit 0
