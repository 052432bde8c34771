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
    ap.add_argument("--config", default="C2", choices=["C2", "C3", "C4", "C5"])
    ap.add_argument("--mode", default="zcull", choices=["exact", "zcull"])
    ap.add_argument("--kernel", default="v3", choices=["v1", "v3"])
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--save-image", default="")
    ap.add_argument("--spp", type=int, default=0, help="experiment: samples per step other than the config's 4")
    ap.add_argument("--kernel-times", action="store_true",
                    help="time every kernel class with HIP events (default: only the dominant kernel)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N>1 (nccl = RCCL over xGMI; gloo = host-staged rehearsal)")
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
    bps = {"bytes_per_sample": pyoracle.algorithmic_bytes(tot) / n,
           "trace_bytes_per_sample": pyoracle.bounce_traversal_bytes(tot) / n}
    return ({"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
             "sample": f"{cfg.name}: {it} full {cfg.width}x{H} iterations x {cfg.spp} spp = {n} samples "
                       f"in {dt:.1f}s, oracle/pn_oracle.c OpenMP {threads} threads"},
            bps, tot)


def stored(path, cfg_name):
    path = os.path.join(REPO, "profiles", path)
    if not os.path.exists(path):
        return None
    return json.load(open(path)).get(cfg_name)


def main():
    args = parse()
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # multi-rank: RCCL adds a stream of its own beside the library's four (own +
        # three workers); 8 hardware queues keep it off theirs (set before HIP starts)
        os.environ["GPU_MAX_HW_QUEUES"] = "8"
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    ndev = torch.cuda.device_count()
    if ndev and local >= ndev:          # rehearsal of N ranks on fewer GPUs (gloo only)
        if args.backend == "nccl":
            raise SystemExit(f"LOCAL_RANK {local} but only {ndev} GPU(s): RCCL needs one GPU per rank")
        local = local % ndev
    torch.cuda.set_device(local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    from pnraytracing_amd import scenes
    from pnraytracing_amd.dist import ShardedFrame
    from pnraytracing_amd.tracer import KERNEL_V1, TRAVERSE_EXACT, TRAVERSE_ZCULL, PathTracer

    builders = {"C2": scenes.bunny_c2, "C3": scenes.marry_c3, "C4": scenes.teapot_c4, "C5": scenes.synthetic_c5}
    cfg = builders[args.config]()
    if args.spp:
        cfg.spp = args.spp
    W, H, spp = cfg.width, cfg.height, cfg.spp

    pt = PathTracer(local)
    # torch works on the library's own stream (created with the context, before its
    # three worker streams): a fifth stream of torch's own would share one of the
    # process's 4 hardware queues with a busy stream (measured -4 %)
    stream = torch.cuda.ExternalStream(pt.stream_handle())
    torch.cuda.set_stream(stream)
    pt.set_stream(stream.cuda_stream)
    opts = (TRAVERSE_ZCULL if args.mode == "zcull" else TRAVERSE_EXACT) | {"v1": KERNEL_V1, "v3": 0}[args.kernel]
    pt.load(cfg, opts)
    info = pt.device_info()

    sf = ShardedFrame(pt, band=BAND, device=torch.device("cuda", local))   # pnraytracing_amd/dist.py
    image = None

    def step(k):
        sf.render(spp * k, spp)
        if world > 1:
            sf.gather_async()                  # one RCCL gather of the row bands to rank 0, overlapped
                                               # with the next step's rendering

    for k in range(args.warmup):
        step(k)
    if world > 1:
        sf.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # live per-kernel timing: the library brackets every launch with HIP events
    # recorded on the stream it launches on (pnrt_profile_enable)
    # only the dominant kernel is bracketed unless --kernel-times: every event record
    # is a queue packet between launches of the overlapped calls
    pt.profile_select(None if args.kernel_times else [{"v1": "v1", "v3": "trace"}[args.kernel]])
    pt.profile_enable(True)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    if world > 1:
        image = sf.finish()                    # every gather completes inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    prof = pt.profile_read()
    pt.profile_enable(False)
    kname = {"v1": "v1", "v3": "trace"}[args.kernel]
    k_ms_total, k_launches = prof[kname]
    kern_ms = k_ms_total / max(k_launches, 1)                  # average launch duration
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cuda" if args.backend == "nccl" else "cpu")
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
            bps = stored("algorithmic_bytes.json", cfg.name)
        rows0 = sf.my_rows
        samples_per_step = rows0 * W * spp
        launches_per_step = k_launches / args.steps
        achieved = path = None
        if bps:
            # dominant kernel: algorithmic bytes of one launch / its average duration
            per_sample = bps["trace_bytes_per_sample"] if args.kernel == "v3" else bps["bytes_per_sample"]
            bytes_per_launch = per_sample * samples_per_step / launches_per_step
            achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
            # SURVEY 8d whole-path figure: all algorithmic bytes / wall time per step
            path_gbs = bps["bytes_per_sample"] * samples_per_step * args.steps / elapsed / 1e9
            path = {"bytes_per_sample": round(bps["bytes_per_sample"], 1), "achieved": round(path_gbs, 2),
                    "frac": round(path_gbs / HBM_PEAK_GBS, 4)}
        traffic = None
        pmc = stored("pmc.json", f"{cfg.name}/{kname}")
        if pmc and pmc.get("hbm_bytes_per_launch"):
            traffic = round(pmc["hbm_bytes_per_launch"] * rows0 / pmc.get("rows", H))
        kernels = {k: {"ms_per_launch": round(ms / n, 4), "launches_per_step": n / args.steps}
                   for k, (ms, n) in prof.items() if n}
        line = {
            "metric": "Msamples/sec (whole node) at 1920x1080, 4spp/iter; fraction of HBM roofline",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: procedural stand-in meshes (reference OBJs absent), reference HDR/texture assets",
            "config": {"workload": f"{cfg.name}: {cfg.description}", "width": W, "height": H,
                       "spp_per_step": spp, "max_bounce_depth": cfg.max_depth, "triangles": cfg.n_triangles,
                       "traverse": args.mode, "kernel_version": args.kernel, "parallelism": f"row-bands{BAND}x{world}",
                       "kernel": {"v1": "pt_render_kernel", "v3": "pt_wf_trace"}[args.kernel]},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2) if achieved else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                         "traffic": traffic,
                         "kernel": {"v1": "pt_render_kernel", "v3": "pt_wf_trace"}[args.kernel],
                         "kernel_ms": round(kern_ms, 4),
                         "algorithmic_bytes_per_launch": round(bytes_per_launch) if bps else None,
                         "path": path},
            "kernels": kernels,
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
