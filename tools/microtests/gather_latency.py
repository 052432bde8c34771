"""Latency of the one-rank RCCL collectives bench.py's gather path uses, against
a plain device copy of the same bytes (N = 8 share of a 1080p RGBA32F frame:
136 rows x 1920 x 16 B = 4.2 MB).  Host-timed, each op followed by
torch.cuda.synchronize(), median of 50 after 10 warm-up.  On the GPU box.

    python tools/microtests/gather_latency.py
"""
import os
import socket
import statistics
import time

import torch
import torch.distributed as dist

with socket.socket() as so:
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                  GPU_MAX_HW_QUEUES="8")
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
rows, W = 136, 1920
send = torch.rand((rows, W, 4), device="cuda")
recv = [torch.zeros_like(send)]
flat = torch.zeros((rows, W, 4), device="cuda")
dst = torch.zeros_like(send)


def t(fn, n=50, warm=10):
    for _ in range(warm):
        fn()
        torch.cuda.synchronize()
    xs = []
    for _ in range(n):
        a = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        xs.append(time.perf_counter() - a)
    return statistics.median(xs) * 1e6


print(f"sync only               {t(lambda: None):8.1f} us")
print(f"device copy 4.2 MB      {t(lambda: dst.copy_(send)):8.1f} us")
print(f"dist.gather             {t(lambda: dist.gather(send, recv, dst=0)):8.1f} us")
print(f"dist.gather async+wait  {t(lambda: dist.gather(send, recv, dst=0, async_op=True).wait()):8.1f} us")
print(f"all_gather_into_tensor  {t(lambda: dist.all_gather_into_tensor(flat, send)):8.1f} us")
print(f"all_reduce 4.2 MB       {t(lambda: dist.all_reduce(send)):8.1f} us")
print(f"broadcast 4.2 MB        {t(lambda: dist.broadcast(send, 0)):8.1f} us")
dist.destroy_process_group()
