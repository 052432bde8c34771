"""Algorithmic bytes per sample per bench config, from the
CPU oracle's counters on a row sample; writes profiles/algorithmic_bytes.json
(used by bench.py when it runs without its CPU-baseline leg).

    python tools/algorithmic_bytes.py [C2 C4 C5]
"""
import json, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np
import pyoracle
from pnraytracing_amd import scenes as S

STEP = {"C2": 9, "C3": 9, "C4": 9, "C5": 45}      # every k-th row (oracle cost bound)
out_path = os.path.join(REPO, "profiles", "algorithmic_bytes.json")
res = json.load(open(out_path)) if os.path.exists(out_path) else {}
for name in sys.argv[1:] or ["C2", "C4"]:
    cfg = S.CONFIGS[name]()
    o = pyoracle.Oracle(cfg)
    acc = np.zeros((cfg.height, cfg.width, 4), np.float32)
    t = time.perf_counter()
    _, st = o.render(0, cfg.spp, rows=(0, cfg.height), y_step=STEP[name], accum=acc)
    n = st["samples"]
    res[cfg.name] = {"bytes_per_sample": pyoracle.algorithmic_bytes(st) / n,
                     "trace_bytes_per_sample": pyoracle.bounce_traversal_bytes(st) / n,
                     "samples": n, "rows": f"every {STEP[name]}th row, frames 0..{cfg.spp - 1}",
                     "counters": st}
    print(name, cfg.name, f"{time.perf_counter() - t:.1f}s", res[cfg.name]["bytes_per_sample"],
          res[cfg.name]["trace_bytes_per_sample"], flush=True)
json.dump(res, open(out_path, "w"), indent=1, sort_keys=True)
