"""Per-kernel averages of the counters in gpurun_out/pmcdiag (tools/gpu_pmc.sh output)."""
import collections, csv, glob, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcdiag"
kernels = sys.argv[2:] or ["pt_wf_trace", "pt_wf_setup", "pt_wf_shade"]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/p*_default/run_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
        per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, d), cs in per.items():
        for c, v in cs.items():
            res[k][c].append(v)
for k in kernels:
    a = {c: sum(v) / len(v) for c, v in res[k].items()}
    print("==", k)
    for c, v in sorted(a.items()):
        print(f"   {c:40s} {v:16.4g}")
    if "TCC_HIT_sum" in a:
        print(f"   L2 hit rate {a['TCC_HIT_sum'] / max(1, a['TCC_HIT_sum'] + a['TCC_MISS_sum']):.3f}")
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in a:
        print(f"   L1 miss ratio (TCC reqs / accesses) {a['TCP_TCC_READ_REQ_sum'] / max(1, a['TCP_TOTAL_CACHE_ACCESSES_sum']):.3f}")
    if "TA_BUSY_avr" in a:
        print(f"   TA busy {a['TA_BUSY_avr'] / max(1, a['GRBM_GUI_ACTIVE'] / 8):.3f}")
