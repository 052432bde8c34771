"""Fold rocprofv3 --pmc passes (gpurun_out/pmc/p*_default) into profiles/pmc.json.

HBM bytes per launch of each kernel = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md
"HBM": on gfx950 FETCH_SIZE reports half of the bytes read; WRITE_SIZE is exact).
FETCH_SIZE/WRITE_SIZE are reported in KiB; the raw TCC_EA0 request counts are
kept beside them as a cross-check.  Usage: python tools/pmc_to_json.py CFG_NAME [ROWS]
"""
import collections, csv, glob, json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1]
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1080
root = os.environ.get("PMC_ROOT") or os.path.join(REPO, "gpurun_out", "pmc")
SHORT = {"pt_wf_trace": "trace", "pt_wf_setup": "setup", "pt_wf_shade": "shade", "pt_wf_gen": "gen",
         "pt_wf_gen_setup": "gen", "pt_wf_shade_setup": "shade",
         "pt_primary_kernel": "primary", "pt_primary_wf": "primary", "pt_blend_kernel": "blend", "pt_render_kernel": "v1"}
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*_default", "run_counter_collection.csv"))):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
        per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, d), cs in per.items():
        for c, v in cs.items():
            acc[k][c].append(v)
out_path = os.path.join(REPO, "profiles", "pmc.json")
res = json.load(open(out_path)) if os.path.exists(out_path) else {}
for k, cs in acc.items():
    if k not in SHORT:
        continue
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    e = {"kernel": k, "rows": rows, "dispatches": max(len(v) for v in cs.values()), "counters_avg": avg}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        e["hbm_bytes_per_launch"] = 2 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        e["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"], 1)
    res[f"{cfg}/{SHORT[k]}"] = e
    print(f"{cfg}/{SHORT[k]}", {kk: (round(v) if isinstance(v, float) else v) for kk, v in e.items() if kk != "counters_avg"})
json.dump(res, open(out_path, "w"), indent=1, sort_keys=True)
