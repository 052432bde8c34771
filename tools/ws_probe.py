#!/usr/bin/env python3
"""Does the trace kernel's lane-step rate depend on the scene's working set?

C2 with the bunny stand-in at several resolutions (same camera, env, depth):
for each, the exclusive trace time per 16-frame launch (PNRT_SERIAL: one call in
flight, full grid) with the product library, and the lane steps per launch from
the WF_STATS census build (variants/libpnrt_stats.so), in child processes.
Geometry bytes = nodes (64 B) + triangle records (48 B) -- against the 4 MB L2
of one XCD.

    python tools/ws_probe.py [nu x nv ...]      (on the GPU box)
"""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
STATS = os.path.join(REPO, "pnraytracing_amd", "variants", "libpnrt_stats.so")
PAT = re.compile(r"\[trace stats\] bounce (\d+) n=(\d+) iters=(\d+) active/iter=[\d.]+ tri=(\d+) node=(\d+) "
                 r"uniform-fetch iters=(\d+) refills=(\d+) rays=(\d+)")


def child(mode, nu, nv):
    from pnraytracing_amd import scenes as S
    from pnraytracing_amd.tracer import SERIAL, TRAVERSE_ZCULL, PathTracer
    cfg = S.bunny_c2(nu=nu, nv=nv)
    pt = PathTracer(0)
    if mode == "time":
        pt.load(cfg, TRAVERSE_ZCULL | SERIAL)
        pt.render(0, 16)
        pt.synchronize()
        pt.profile_select(["trace"])
        pt.profile_enable(True)
        for k in range(4):
            pt.render(16 * (k + 1), 16)
        prof = pt.profile_read()
        ms, n = prof["trace"]
        info = pt.device_info()
        print(json.dumps({"trace_ms": ms / n, "launches": n, "nodes": info["n_interior"], "tris": cfg.n_triangles}))
    else:
        pt.load(cfg)
        pt.render(0, 16)
        pt.synchronize()
    pt.close()


def main(specs):
    out = []
    for sp in specs:
        nu, nv = map(int, sp.split("x"))
        t = subprocess.run([sys.executable, __file__, "--child", "time", str(nu), str(nv)], capture_output=True,
                           text=True, timeout=300)
        if t.returncode:
            raise SystemExit(t.stdout + t.stderr)
        r = json.loads([x for x in t.stdout.splitlines() if x.startswith("{")][-1])
        s = subprocess.run([sys.executable, __file__, "--child", "stats", str(nu), str(nv)], capture_output=True,
                           text=True, timeout=300, env=dict(os.environ, PNRT_DEVICE_LIB=STATS))
        if s.returncode:
            raise SystemExit(s.stdout + s.stderr)
        b = [tuple(map(int, m.groups())) for m in PAT.finditer(s.stderr)]
        steps = sum(x[3] + x[4] for x in b) / len(b)         # lane steps per launch (16 frames, one bounce)
        rays = sum(x[7] for x in b) / len(b)
        geo = r["nodes"] * 64 + r["tris"] * 48
        r.update({"nu": nu, "nv": nv, "geometry_MB": round(geo / 1e6, 2), "lane_steps_per_launch": steps,
                  "rays_per_launch": rays, "G_lane_steps_per_s": round(steps / (r["trace_ms"] * 1e-3) / 1e9, 1),
                  "G_rays_per_s": round(rays / (r["trace_ms"] * 1e-3) / 1e9, 2)})
        print(json.dumps(r), flush=True)
        out.append(r)
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    else:
        main(sys.argv[1:] or ["264x132", "186x93", "132x66", "66x33", "528x264"])
