"""Rank 0's share of an N-GPU C2 bench run, timed the way bench.py times it:
one untimed sizing call, a reset, the warm-up calls, a synchronise, then the K
timed steps as calls of `ipc` 4-spp iterations (the last one cut) and a
synchronise.  Measures what the calls' size does to a rank's rate inside the
driver's 20-step region (iters_per_call).

Two columns (VERDICT r5 "Next" 6):
  plain       the share's calls alone, no gather;
  collective  the same calls through bench.py's own gather path: a ONE-rank RCCL
              process group and ShardedFrame(collective=True, shard=(N, 0)) --
              after every call pack_rows + an asynchronous dist.gather on the
              double-buffered slots, the last one completed (and the image
              assembled) inside the timed region, exactly as bench.py's ranks do.
              What one GPU cannot show is the other N - 1 ranks' rows arriving
              over xGMI (rank 0 receives (N - 1) / N of the frame per call); the
              caller reports that transfer's time at the link rate beside it.

    python tools/share_bench.py N ipc [steps] [warmup] [--collective]     (on the GPU box)
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pnraytracing_amd import scenes  # noqa: E402
from pnraytracing_amd.tracer import PathTracer, shard_rows  # noqa: E402

argv = [a for a in sys.argv[1:] if not a.startswith("--")]
collective = "--collective" in sys.argv
n, ipc = int(argv[0]), int(argv[1])
steps = int(argv[2]) if len(argv) > 2 else 20
warm = int(argv[3]) if len(argv) > 3 else 5
SPP = 4
if n > 1:
    # as bench.py's ranks (world > 1): 8 hardware queues, so RCCL's stream gets one beside the
    # library's four (set before anything initialises HIP)
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
cfg = scenes.bunny_c2()
rows = len(shard_rows(cfg.height, 8, n, 0))


def groups(lo, hi):
    return [(k, min(ipc, hi - k)) for k in range(lo, hi, ipc)]


# untimed sizing calls, as bench.py issues them (bench.sizing_calls): one per distinct call size
SIZES = [ipc] + sorted({m for _, m in groups(0, warm) + groups(warm, warm + steps)} - {ipc}, reverse=True)
if os.environ.get("SHARE_ONE_SIZING"):       # (the round-5 plan: the timed calls' size only)
    SIZES = [ipc]


# diagnostic (SHARE_PROBE): the plain calls, but in a process that first initialises torch's HIP context
# ("torch"), also puts torch on the library's stream ("stream"), or also joins a one-rank RCCL group ("dist")
probe = os.environ.get("SHARE_PROBE", "")
if probe and not collective:
    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    if probe == "indexcopy":          # one torch index_copy_ (small tensors)
        torch.zeros((64, 4), device="cuda").index_copy_(0, torch.arange(8, device="cuda"), torch.ones((8, 4), device="cuda"))
    if probe == "stridedcopy":        # one strided torch copy_ (small tensors)
        torch.zeros((16, 4), device="cuda")[::2].copy_(torch.ones((8, 4), device="cuda"))
    if probe == "sort":               # an unrelated torch kernel family
        torch.sort(torch.rand(1024, device="cuda"))
    torch.cuda.synchronize()
    if probe in ("dist", "gather", "allgather", "gatherbig", "gatherasync"):
        import socket
        import torch.distributed as dist
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(so.getsockname()[1]), RANK="0", WORLD_SIZE="1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        x = torch.zeros(1024, device="cuda")
        big = torch.zeros((136, 1920, 4), device="cuda")
        if probe == "gather":         # one RCCL gather (send / recv to itself) before the calls
            dist.gather(x, [torch.zeros_like(x)], dst=0)
        if probe == "gatherbig":      # ... of a rank's 4.2 MB share
            dist.gather(big, [torch.zeros_like(big)], dst=0)
        if probe == "gatherasync":    # ... asynchronous, then waited for (ShardedFrame.gather_async / finish)
            dist.gather(big, [torch.zeros_like(big)], dst=0, async_op=True).wait()
        if probe == "allgather":      # one RCCL ring collective instead
            dist.all_gather_into_tensor(torch.zeros_like(x), x)
        torch.cuda.synchronize()
if not collective:
    with PathTracer(0) as pt:
        if probe in ("stream", "dist", "gather", "allgather", "gatherbig", "gatherasync"):
            stream = torch.cuda.ExternalStream(pt.stream_handle())
            torch.cuda.set_stream(stream)
            pt.set_stream(stream.cuda_stream)
        pt.load(cfg)
        for m in SIZES:                          # sizing calls
            pt.render(0, SPP * m, 8, n, 0)
        pt.synchronize()
        pt.reset_accum()
        for k, m in groups(0, warm):
            pt.render(SPP * k, SPP * m, 8, n, 0)
        pt.synchronize()
        t = time.perf_counter()
        for k, m in groups(warm, warm + steps):
            pt.render(SPP * k, SPP * m, 8, n, 0)
        pt.synchronize()
        dt = (time.perf_counter() - t) / steps
else:
    import socket

    import torch
    import torch.distributed as dist
    from pnraytracing_amd.dist import ShardedFrame
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    pt = PathTracer(0)
    stream = torch.cuda.ExternalStream(pt.stream_handle())      # as bench.py: torch on the library's stream
    torch.cuda.set_stream(stream)
    pt.set_stream(stream.cuda_stream)
    pt.load(cfg)
    sf = ShardedFrame(pt, band=8, device=torch.device("cuda", 0), collective=True, shard=(n, 0))
    for m in SIZES:                              # sizing calls
        sf.render(0, SPP * m)
    torch.cuda.synchronize()
    pt.reset_accum()
    wg_mode = os.environ.get("SHARE_WARMGATHER", "1")                # (diagnostic switches)
    warm_gather = wg_mode == "1"
    barrier = os.environ.get("SHARE_BARRIER", "1") == "1"
    sync_first = os.environ.get("SHARE_SYNCFIRST") == "1"
    for k, m in groups(0, warm):
        sf.render(SPP * k, SPP * m)
        if sync_first:
            torch.cuda.synchronize()
        if warm_gather:
            sf.gather_async()
        elif wg_mode == "pack":
            pt.pack_rows(sf.sendb[0].data_ptr(), 8, n, 0)
        elif wg_mode == "gatheronly":
            dist.gather(sf.sendb[0], sf.recvb[0], dst=0, async_op=True).wait()
        elif wg_mode == "assemble":
            sf._assemble(sf.recvb[0])
        elif wg_mode == "fillimg":        # a torch kernel on the library's stream, on the image
            sf.image.fill_(0.0)
        elif wg_mode == "fillsmall":      # a torch kernel on the library's stream, small
            torch.zeros(64, device="cuda").fill_(1.0)
        elif wg_mode == "assembledef":    # the assembly on torch's default stream
            torch.cuda.synchronize()
            with torch.cuda.stream(torch.cuda.default_stream()):
                sf.image.index_copy_(0, sf.rows[0], sf.recvb[0][0][:len(sf.rows[0])])
            torch.cuda.synchronize()
    if warm_gather:
        sf.finish()
    torch.cuda.synchronize()
    if os.environ.get("SHARE_SLEEP"):
        time.sleep(float(os.environ["SHARE_SLEEP"]))
    if barrier:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    marks = []
    what = os.environ.get("SHARE_COLL", "gather")    # diagnostic: "render" (no gather), "pack" (pack only)
    for k, m in groups(warm, warm + steps):
        sf.render(SPP * k, SPP * m)
        marks.append(time.perf_counter() - t)
        if what == "gather":
            sf.gather_async()
        elif what == "pack":
            pt.pack_rows(sf.sendb[0].data_ptr(), 8, n, 0)
        marks.append(time.perf_counter() - t)
    if what == "gather":
        sf.finish()                              # every gather completes inside the timed region
    marks.append(time.perf_counter() - t)
    torch.cuda.synchronize()
    if barrier:
        dist.barrier()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    if os.environ.get("SHARE_MARKS"):           # host-side time after each render / gather_async / finish
        print("marks ms:", " ".join(f"{x * 1e3:.2f}" for x in marks), f"end {dt * steps * 1e3:.2f}", flush=True)
    pt.close()
    dist.destroy_process_group()
per_rank = rows * cfg.width * SPP / dt / 1e6
print(f"N={n} ipc={ipc} {'collective' if collective else 'plain'}: rank-0 rows {rows}, {dt * 1e3:.3f} ms/step, "
      f"{per_rank:.1f} Msamples/s per rank", flush=True)
