"""Worker for tests/test_gpu_dist.py::test_rccl_gather_*: renders C4 (small) row
bands through ShardedFrame with the nccl (= RCCL) backend and gathers them to
rank 0 with the asynchronous double-buffered gather bench.py uses; rank 0
saves the image.  All ranks use GPU 0 (a one-GPU box): RCCL may refuse two
ranks on one device, which the test reports as a skip.

    python -m torch.distributed.run --nproc-per-node N tests/rccl_worker.py OUT.npy
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main(out):
    from pnraytracing_amd import scenes
    from pnraytracing_amd.dist import ShardedFrame
    from pnraytracing_amd.tracer import PathTracer

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    cfg = scenes.teapot_c4(320, 176)
    pt = PathTracer(0)
    pt.load(cfg)
    sf = ShardedFrame(pt, device=torch.device("cuda", 0), collective=True)
    for k in range(3):                        # three steps: both gather slots are reused
        sf.render(4 * k, 4)
        sf.gather_async()
    img = sf.finish()
    torch.cuda.synchronize()
    if dist.get_rank() == 0:
        np.save(out, img.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()
    pt.close()


if __name__ == "__main__":
    main(sys.argv[1])
