#!/usr/bin/env python3
"""Per-kernel launch durations from a rocprofv3 --kernel-trace CSV, checked
against the bench line of the same command (the roofline's
kernel_ms must be reproducible from the committed rocprof record).

bench.py issues one untimed sizing call before its warm-up (cold caches and
first-touch pages make its launches slower); the summary therefore reports
every launch AND the launches after that first call.  With `--serial --warmup 20
--steps 20` (tools/gpu_session.sh prof) every call is a whole one-batch call of the
bench's size (20 iterations, 80 frames of 1080p; 16 frames until late round 6) in
flight alone, so the trace kernel's average over the later launches is the line's
exclusive kernel_ms.

    python tools/prof_summary.py KERNEL_TRACE.csv BENCH_LINE.json [OUT.json] [--serial]

The line's config.calls ("serial" / "pipelined", round 4) picks the comparison;
--serial marks a line written before that field existed.
"""
import csv
import json
import statistics
import sys

SHORT = {"pt_wf_trace": "trace", "pt_wf_gen_setup": "gen", "pt_wf_shade_setup": "shade",
         "pt_primary_kernel": "primary", "pt_primary_wf": "primary", "pt_blend_kernel": "blend", "pt_render_kernel": "v1"}


def main():
    pos = [a for a in sys.argv[1:] if not a.startswith("--")]
    trace, line_path = pos[0], pos[1]
    line = [json.loads(x) for x in open(line_path) if x.startswith("{")][-1]
    ipc = line["config"]["iters_per_call"]
    rows = []
    for r in csv.DictReader(open(trace)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
        if name in SHORT:
            rows.append((int(r["Start_Timestamp"]), SHORT[name], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    rows.sort()
    # the sizing call ends where the second call's ray generation starts (one gen
    # launch per call at these sizes; the primary pass runs only when a pipe's
    # cached primary records are stale, round 4)
    gen = [i for i, (_, k, _) in enumerate(rows) if k == "gen"]
    cut = gen[1] if len(gen) > 1 else 0
    out = {"trace_csv": trace, "bench_line": line_path, "sizing_call_launches": cut, "kernels": {}}
    for k in sorted(set(k for _, k, _ in rows)):
        allv = [d for _, kk, d in rows if kk == k]
        later = [d for i, (_, kk, d) in enumerate(rows) if kk == k and i >= cut]
        out["kernels"][k] = {"launches": len(allv), "mean_ms_all": round(statistics.mean(allv), 4),
                             "launches_after_sizing_call": len(later),
                             "mean_ms_after_sizing_call": round(statistics.mean(later), 4) if later else None,
                             "min_ms": round(min(allv), 4), "max_ms": round(max(allv), 4)}
    kname = {"pt_wf_trace": "trace", "pt_render_kernel": "v1"}[line["roofline"]["kernel"]]
    kms, kpipe = line["roofline"]["kernel_ms"], line["roofline"].get("kernel_ms_pipelined")
    got = out["kernels"].get(kname, {}).get("mean_ms_after_sizing_call")
    # a --serial command's launches are exclusive (compare with kernel_ms); a default
    # command's overlap the other calls' kernels (compare with kernel_ms_pipelined,
    # the HIP-event average over its timed launches)
    calls = line["config"].get("calls")
    serial = calls == "serial" if calls else "--serial" in sys.argv[1:]
    ref = kms if serial else kpipe
    out["check"] = {"kernel": kname, "line_kernel_ms": kms, "line_kernel_ms_pipelined": kpipe,
                    "compared_with": "kernel_ms" if serial else "kernel_ms_pipelined", "rocprof_mean_ms": got,
                    "rel_diff": round(got / ref - 1.0, 4) if (got and ref) else None, "iters_per_call": ipc}
    print(json.dumps(out, indent=1))
    if len(pos) > 2:
        json.dump(out, open(pos[2], "w"), indent=1)


if __name__ == "__main__":
    main()
