"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (avg per dispatch)."""
import csv, glob, os, sys, collections
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*_*/run_counter_collection.csv"))):
    var = os.path.basename(os.path.dirname(f)).split("_", 1)[1]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, d), cs in per.items():
        for c, v in cs.items():
            res[(var, k)][c].append(v)
for (var, k), cs in sorted(res.items()):
    if "pack" in k or "rocclr" in k or "math" in k: continue
    print(f"== {var} {k}")
    for c, vs in sorted(cs.items()):
        print(f"   {c:32s} {sum(vs)/len(vs):16.4g}  (n={len(vs)})")
