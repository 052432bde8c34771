#!/bin/bash
# Round-3 session 5: working-set probe of the trace kernel (bunny resolutions),
# and its L2 hit rate with one call in flight vs pipelined.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03s5; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; local t0=$SECONDS; "$@"; local rc=$?; echo "$name rc=$rc ($((SECONDS - t0)) s)"; [ $rc -eq 0 ] || exit $rc; }
step ws-probe timeout -k 10 600 python tools/ws_probe.py 264x132 186x93 132x66 66x33 528x264 > $O/ws_probe.log 2>&1
cat $O/ws_probe.log
for m in serial pipe; do
  extra=""; [ $m = serial ] && extra="--serial"
  step pmc-$m timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $O/pmc_$m -o run --output-format csv -- \
    python bench.py --steps 8 --warmup 4 --no-cpu-baseline --no-pmc --serial-steps 0 $extra > $O/pmc_$m.json 2> $O/pmc_$m.err
done
python - <<'PY'
import csv, glob
for m in ("serial", "pipe"):
    acc = {}
    for f in glob.glob(f"gpurun_out/r03s5/pmc_{m}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
            acc.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        if not k.startswith("pt_"): continue
        h, mi = sum(cs.get("TCC_HIT_sum", [0])), sum(cs.get("TCC_MISS_sum", [0]))
        print(m, k, "L2 hit %.3f" % (h / max(h + mi, 1)), "RDREQ/launch %.3g" % (sum(cs.get("TCC_EA0_RDREQ_sum", [0])) / max(len(cs.get("TCC_EA0_RDREQ_sum", [1])), 1)))
PY
exit 0
