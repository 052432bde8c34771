#!/usr/bin/env python3
"""Where a synchronised one-frame-per-call loop (bench.py --config D2 --sync-per-frame)
spends its frame, from a rocprofv3 kernel trace: per frame (gen -> {trace -> shade} x depth
-> blend) the kernels' own durations by class, the GPU-side gaps between consecutive
kernels of the frame, and the gap from one frame's blend to the next frame's first kernel
(the host's synchronise + the next call's launch latency).  Medians over the frames.

    python tools/frame_gaps.py run_kernel_trace.csv [skip_frames]
"""
import csv
import statistics as st
import sys

KS = {"pt_wf_gen_setup": "gen", "pt_wf_trace": "trace", "pt_wf_shade_setup": "shade", "pt_blend_kernel": "blend",
      "pt_primary_wf": "primary"}


def cls(name):
    n = name.replace("void ", "").split("(")[0].split("<")[0].strip()
    return KS.get(n)


def main(path, skip=4):
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), cls(r["Kernel_Name"])) for r in csv.DictReader(open(path))]
    rows = sorted(r for r in rows if r[2])
    frames, cur = [], []
    for r in rows:
        cur.append(r)
        if r[2] == "blend":
            frames.append(cur)
            cur = []
    frames = frames[skip:]
    if len(frames) < 3:
        print("too few frames")
        return
    per = {}
    inner, between, span = [], [], []
    for i, f in enumerate(frames):
        for s, e, k in f:
            per.setdefault(k, []).append((e - s) / 1e3)
        inner.append(sum(max(0, f[j + 1][0] - f[j][1]) for j in range(len(f) - 1)) / 1e3)
        span.append((f[-1][1] - f[0][0]) / 1e3)
        if i + 1 < len(frames):
            between.append((frames[i + 1][0][0] - f[-1][1]) / 1e3)
    print(f"{len(frames)} frames; medians in us")
    for k, v in sorted(per.items()):
        n = len(v) / len(frames)
        print(f"  {k:8s} {st.median(v):8.1f} per launch x {n:.1f} = {st.median(v) * n:8.1f}")
    busy = sum(st.median(v) * len(v) / len(frames) for v in per.values())
    print(f"  kernels  {busy:8.1f}")
    print(f"  gaps inside the frame (GPU-side, between dependent kernels) {st.median(inner):8.1f}")
    print(f"  frame span (first kernel start -> blend end)                {st.median(span):8.1f}")
    print(f"  blend end -> next frame's first kernel (sync + launch)       {st.median(between):8.1f}")
    print(f"  frame period                                                  {st.median(span) + st.median(between):8.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
