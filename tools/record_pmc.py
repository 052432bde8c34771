#!/usr/bin/env python3
"""Record an N = 1 bench line's live-PMC roofline traffic in profiles/pmc.json,
keyed by config / kernel and the device-source hash, so that a multi-GPU bench
run whose rank-0 PMC passes fail (or run with --no-pmc) can still report its
rank's traffic per launch as a labelled derivation (bench.py: the figure x the rank's share of the
rows x its frames per launch / the recorded launch's).

    python tools/record_pmc.py BENCH_LINE.json [...]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "profiles", "pmc.json")


def main(paths):
    db = {}
    if os.path.exists(OUT):
        old = json.load(open(OUT))
        db = {k: v for k, v in old.items() if "source_hash" in v}      # drop entries without a source hash
    for p in paths:
        line = [json.loads(x) for x in open(p) if x.startswith("{")][-1]
        r, c = line["roofline"], line["config"]
        if line["n_gpus"] != 1 or not r.get("traffic"):
            print(f"{p}: not an N = 1 line with live traffic; skipped")
            continue
        src = line["device"]["library"].rsplit(" ", 1)[-1]
        name = c["workload"].split(":")[0]
        kshort = {"pt_wf_trace": "trace", "pt_render_kernel": "v1"}[r["kernel"]]
        db[f"{name}/{kshort}"] = {
            "bytes_per_launch": r["traffic"], "traffic_source": r["traffic_source"],
            "l2_hit_rate": r.get("l2_hit_rate"), "rows": c["height"],
            "frames_per_launch": c["spp_per_step"] * c["iters_per_call"], "source_hash": src,
            "from": os.path.basename(p)}
        print(f"{name}/{kshort}: {r['traffic']:.4g} B per launch (src {src})")
    json.dump(db, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:])
