#!/bin/bash
# A/B of prebuilt libpnrt variants: quick parity diag + bench per variant, then
# optional PMC passes (one counter group per rocprofv3 run) on the default lib.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
for lib in ${LIBS:-default}; do
  if [ "$lib" = default ]; then unset PNRT_DEVICE_LIB; else export PNRT_DEVICE_LIB=$PWD/$lib; fi
  timeout -k 10 300 python tools/diag.py > gpurun_out/diag_$(basename $lib).log 2>&1
  rc=$?; echo "diag [$lib] rc=$rc"; cat gpurun_out/diag_$(basename $lib).log | tail -8; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 240 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$(basename $lib).log 2>&1
  rc=$?; echo "bench [$lib] rc=$rc"; tail -1 gpurun_out/ab_$(basename $lib).log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
unset PNRT_DEVICE_LIB
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc/p${i}_default -o run --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc/p${i}.log 2>&1
  rc=$?; echo "pmc pass $i [$grp] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<GROUPS
${PMC_GROUPS}
GROUPS
exit 0
