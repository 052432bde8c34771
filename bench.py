#!/usr/bin/env python3
"""bench.py -- Msamples/s of the MI355X path tracer on the BASELINE workload.

Workload (BASELINE.json metric / configs[1]; SURVEY 8d "C2"): Cornell box +
~70k-triangle bunny stand-in + vignaioli_night_1k HDR environment,
1920x1080, one step = one 4-spp iteration (frames 4k..4k+3 blended in order),
MAX_BOUNCE_DEPTH 4.  Synthetic scene data (procedural mesh stand-ins; the
reference's OBJ assets do not exist), the reference's real 1k HDR.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

N > 1: one process per GPU; the image rows are dealt in 8-row bands
(rank r owns bands b with b % N == r), each rank renders its rows, and the
accumulated rows are gathered to rank 0 over RCCL every step (strong
scaling: the frame is fixed, its rows are split).

Prints ONE JSON line (rank 0) with roofline and cpu_baseline objects; see
DESIGN.md "Measurement" for every field's derivation.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BAND = 8
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=["C2", "C4", "C5"])
    ap.add_argument("--mode", default="zcull", choices=["exact", "zcull"])
    ap.add_argument("--kernel", default="v3", choices=["v1", "v3"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--save-image", default="")
    return ap.parse_args()


def cpu_baseline(cfg, target_s: float):
    """CPU oracle (the C restatement of ray_tracing.comp, OpenMP over rows) on a
    bounded row sample of the same workload; returns (dict, bytes_per_sample)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    o = pyoracle.Oracle(cfg)
    H = cfg.height
    # whole-frame 4-spp iterations of the same workload until ~target_s (max 8)
    acc = np.zeros((H, cfg.width, 4), np.float32)
    tot = None
    it = 0
    t = time.perf_counter()
    while it < 8:
        _, st = o.render(it * cfg.spp, cfg.spp, accum=acc, threads=threads)
        tot = st if tot is None else {k: tot[k] + st[k] for k in st}
        it += 1
        if time.perf_counter() - t >= target_s:
            break
    dt = time.perf_counter() - t
    n = tot["samples"]
    bps = pyoracle.algorithmic_bytes(tot) / n
    return ({"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
             "sample": f"{cfg.name}: {it} full {cfg.width}x{H} iterations x {cfg.spp} spp = {n} samples "
                       f"in {dt:.1f}s, oracle/pn_oracle.c OpenMP {threads} threads"},
            bps, tot)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from pnraytracing_amd import scenes
    from pnraytracing_amd.tracer import KERNEL_V1, TRAVERSE_EXACT, TRAVERSE_ZCULL, PathTracer, shard_rows

    builders = {"C2": scenes.bunny_c2, "C4": scenes.teapot_c4, "C5": scenes.synthetic_c5}
    cfg = builders[args.config]()
    W, H, spp = cfg.width, cfg.height, cfg.spp

    pt = PathTracer(local)
    stream = torch.cuda.Stream()               # a real stream handle (the default one is NULL)
    torch.cuda.set_stream(stream)
    pt.set_stream(stream.cuda_stream)
    opts = (TRAVERSE_ZCULL if args.mode == "zcull" else TRAVERSE_EXACT) | {"v1": KERNEL_V1, "v3": 0}[args.kernel]
    pt.load(cfg, opts)
    info = pt.device_info()

    rows = [torch.as_tensor(shard_rows(H, BAND, world, r), device="cuda") for r in range(world)]
    maxrows = max(len(r) for r in rows)
    if world > 1:
        sendbuf = torch.zeros((maxrows, W, 4), dtype=torch.float32, device="cuda")
        recv = [torch.zeros_like(sendbuf) for _ in range(world)] if rank == 0 else None
        image = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda") if rank == 0 else None

    def step(k, ev=None):
        if ev is not None:
            ev[0].record(stream)
        pt.render(spp * k, spp, BAND, world, rank)
        if ev is not None:
            ev[1].record(stream)
        if world > 1:
            pt.pack_rows(sendbuf.data_ptr(), BAND, world, rank)
            dist.gather(sendbuf, recv, dst=0)
            if rank == 0:
                for r in range(world):
                    image.index_copy_(0, rows[r], recv[r][: len(rows[r])])

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k, events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    if args.save_image and rank == 0:
        img = (image.cpu().numpy() if world > 1 else pt.read_accum())
        np.save(args.save_image, img)

    samples = W * H * spp * args.steps
    value = samples / elapsed / 1e6
    line = None
    if rank == 0:
        cpu = None
        bps = None
        if world == 1 and not args.no_cpu_baseline:
            cpu, bps, _ = cpu_baseline(cfg, args.cpu_seconds)
        if bps is None:
            bps = float(json.load(open(os.path.join(REPO, "profiles", "algorithmic_bytes.json")))[cfg.name]) \
                if os.path.exists(os.path.join(REPO, "profiles", "algorithmic_bytes.json")) else None
        rows0 = len(rows[0])
        samples_per_launch = rows0 * W * spp
        achieved = (bps * samples_per_launch / (kern_ms * 1e-3) / 1e9) if bps else None
        traffic = None
        pmc = os.path.join(REPO, "profiles", f"pmc_{cfg.name}.json")
        if os.path.exists(pmc):
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch_full_frame")
            if traffic is not None:
                traffic = traffic * rows0 / H
        line = {
            "metric": "Msamples/sec (whole node) at 1920x1080, 4spp/iter; fraction of HBM roofline",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (procedural bunny stand-in, reference 1k HDR)",
            "config": {"workload": f"{cfg.name}: {cfg.description}", "width": W, "height": H,
                       "spp_per_step": spp, "max_bounce_depth": cfg.max_depth, "triangles": cfg.n_triangles,
                       "traverse": args.mode, "kernel_version": args.kernel, "parallelism": f"row-bands{BAND}x{world}",
                       "kernel": {"v1": "pt_render_kernel", "v3": "pt_wf_trace"}[args.kernel]},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "traffic": traffic,
                         "bytes_per_sample": round(bps, 1) if bps else None,
                         "kernel_ms": round(kern_ms, 4)},
            "cpu_baseline": cpu,
            "device": {"bvh_interior_nodes": info["n_interior"], "max_depth": info["max_depth"],
                       "scene_bytes": info["device_bytes"]},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    pt.close()


if __name__ == "__main__":
    main()
