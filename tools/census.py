"""Trace-kernel request census -> profiles/census.json (read by bench.py).

Runs one 4-spp call of a config with the WF_STATS build of the CURRENT sources
(pnraytracing_amd/variants/libpnrt_stats.so, made by
`tools/build_variants.sh stats:"-DWF_PIPES=1 -DWF_STATS=1"`), whose trace
kernel counts per launch its lane-steps (node visits, triangle tests) and rays.
Requested bytes of one trace launch, in the device layout:
  node visit      64 B  (both child boxes + refs/axis: four 16-B loads)
  triangle test   48 B  (the record; the fourth 16-B load of a triangle lane
                         reads one shared address)
  ray             32 B  (origin + direction) + 4 B result
(rays = every ray the launch took, the moot light rays included: each takes one
lane step, its root box test; moot_light / moot_env count the shadow rays the
setup found moot, pt_wf.h WF_SKIP_MOOT -- the env ones are not queued at all --
and moot_cont the last bounce's continuation rays, NaN rays like the light ones)
The entry carries the source hash of the sources it was measured on; bench.py
uses it only while they are unchanged.

    python tools/census.py C2 C3 C4 C5        (on the GPU box)
"""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
LIB = os.path.join(REPO, "pnraytracing_amd", "variants", "libpnrt_stats.so")
PAT = re.compile(r"\[trace stats\] bounce (\d+) n=(\d+) iters=(\d+) active/iter=[\d.]+ tri=(\d+) node=(\d+) "
                 r"uniform-fetch iters=(\d+) refills=(\d+) rays=(\d+)")
MOOT = re.compile(r"\[trace moot\] bounce (\d+) light=(\d+) env=(\d+) cont=(\d+)")


def child(name):
    from pnraytracing_amd import scenes as S
    from pnraytracing_amd.tracer import PathTracer
    cfg = S.CONFIGS[name]()
    pt = PathTracer(0)
    pt.load(cfg)
    pt.render(0, cfg.spp)
    pt.synchronize()
    pt.close()
    print("rows", cfg.height, "name", cfg.name, flush=True)


def main(names):
    from pnraytracing_amd import build
    out_path = os.path.join(REPO, "profiles", "census.json")
    res = json.load(open(out_path)) if os.path.exists(out_path) else {}
    for name in names:
        env = dict(os.environ, PNRT_DEVICE_LIB=LIB)
        r = subprocess.run([sys.executable, __file__, "--child", name], env=env, capture_output=True, text=True,
                           timeout=600)
        if r.returncode != 0:
            print(r.stdout[-2000:], r.stderr[-2000:])
            raise SystemExit(f"{name}: census run failed ({r.returncode})")
        b = [tuple(map(int, m.groups())) for m in PAT.finditer(r.stderr)]
        moot = {int(m.group(1)): (int(m.group(2)), int(m.group(3)), int(m.group(4))) for m in MOOT.finditer(r.stderr)}
        rows = int(re.search(r"rows (\d+) name (\S+)", r.stdout).group(1))
        cname = re.search(r"rows (\d+) name (\S+)", r.stdout).group(2)
        launches = len(b)
        tri = sum(x[3] for x in b)
        node = sum(x[4] for x in b)
        rays = sum(x[7] for x in b)
        req = 64 * node + 48 * tri + 36 * rays
        res[cname] = {"source_hash": build.device_source_hash(), "rows": rows, "frames": 4, "trace_launches": launches,
                      "per_bounce": [{"bounce": x[0], "paths": x[1], "iters": x[2], "tri_steps": x[3],
                                      "node_steps": x[4], "rays": x[7],
                                      "moot_light": moot.get(x[0], (0, 0, 0))[0], "moot_env": moot.get(x[0], (0, 0, 0))[1],
                                      "moot_cont": moot.get(x[0], (0, 0, 0))[2]}
                                     for x in b],
                      "lane_steps_per_ray": round((tri + node) / max(rays, 1), 3),
                      "requested_bytes_per_launch": round(req / max(launches, 1))}
        print(cname, {k: v for k, v in res[cname].items() if k != "per_bounce"}, flush=True)
    json.dump(res, open(out_path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2])
    else:
        main(sys.argv[1:])
