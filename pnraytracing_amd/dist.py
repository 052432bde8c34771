"""Multi-GPU row-band sharding of one frame.

Every pixel of ``ray_tracing.comp`` is independent -- the seed (``:977-979``)
and the Cranley-Patterson shift (``:540-543``) depend only on (x, y, frame) --
so any row partition reproduces the single-GPU image bit for bit.  Rank r of
N renders the rows ``{y : (y // band) % N == r}`` (interleaved 8-row bands
balance the expensive middle of the frame), packs them into a contiguous
buffer and one ``gather`` (RCCL over xGMI for CUDA tensors, gloo on CPU)
brings them to rank 0, which scatters them back into image order.  There is
no other collective: the ranks never exchange data while rendering.

One process per GPU (``torch.distributed.run``); the tracer of each rank
must launch on the stream torch uses for the collective, which
:class:`ShardedFrame` arranges for CUDA devices.

The tracer protocol is the one of :class:`pnraytracing_amd.tracer.PathTracer`:
``width``, ``height``, ``render(first, n, band, n_shards, shard)`` and
``pack_rows(dst_ptr, band, n_shards, shard)``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .tracer import shard_rows

BAND = 8


class ShardedFrame:
    """Render the rows of this rank and gather the frame to rank 0."""

    def __init__(self, tracer, band: int = BAND, device: str | torch.device = "cuda", group=None,
                 collective: bool = False, shard: tuple[int, int] | None = None):
        self.tracer, self.band, self.group = tracer, band, group
        # collective=True: gather through the process group even with one rank (the
        # RCCL path exercised on a one-GPU box; the image is the same either way)
        self.collective = collective and dist.is_initialized()
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.gworld = self.world          # ranks of the collective (the split's ranks but below)
        if shard is not None:
            # (world, rank) of a split rendered WITHOUT a process group: one rank's share
            # alone (bench.py's PMC pass of rank 0's share); no gather, render() and
            # pack_rows() use the given split.  With a ONE-rank group and collective=True:
            # rank 0's share of the split gathered through that group (its side of the
            # gather, every call's pack + dist.gather + assembly; tools/share_bench.py)
            if dist.is_initialized() and not (self.collective and self.world == 1 and int(shard[1]) == 0):
                raise ValueError("ShardedFrame: shard= is for a process without a process group "
                                 "(or rank 0 of a split over a one-rank group with collective=True)")
            self.world, self.rank = int(shard[0]), int(shard[1])
            if not (self.world >= 1 and 0 <= self.rank < self.world):
                raise ValueError(f"ShardedFrame: bad shard {shard}")
        self.device = torch.device(device)
        H, W = tracer.height, tracer.width
        if H <= 0 or W <= 0:
            raise ValueError("ShardedFrame: set_frame() the tracer first")
        # gloo cannot gather device tensors: stage through host memory (rehearsal
        # of the multi-GPU path on one GPU / CPU-only hosts); RCCL gathers in HBM
        self.stage = (dist.is_initialized() and self.device.type == "cuda"
                      and dist.get_backend(group) == "gloo")
        # the tracer and this object's torch work (pack buffers, collectives, image
        # assembly) share one stream: the caller's current stream, or -- when that is
        # the NULL stream, which does not order against the tracer's non-blocking
        # streams -- the tracer's own stream, wrapped for torch
        self.stream = None
        if self.device.type == "cuda" and hasattr(tracer, "set_stream"):
            cur = torch.cuda.current_stream(self.device)
            if cur.cuda_stream == 0 and hasattr(tracer, "stream_handle"):
                self.stream = torch.cuda.ExternalStream(tracer.stream_handle(), device=self.device)
                tracer.set_stream(None)
            else:
                tracer.set_stream(cur.cuda_stream)
        self._on_stream(lambda: self._alloc(H, W))

    def _alloc(self, H: int, W: int):
        band = self.band
        rows = [shard_rows(H, band, self.world, r) for r in range(self.world)]
        self.rows = [torch.as_tensor(r, device=self.device) for r in rows]
        self.my_rows = len(rows[self.rank])
        self.max_rows = max(len(r) for r in rows)           # rank 0 owns the most (first bands)
        # equal-sized buffers for the collective; the tail of a short shard is padding.
        # Two slots, so the gather of step k runs on the RCCL stream while step k+1
        # renders (gather_async / finish)
        cdev = torch.device("cpu") if self.stage else self.device
        self.sendb = [torch.zeros((self.max_rows, W, 4), dtype=torch.float32, device=self.device) for _ in range(2)]
        self.recvb = [[torch.zeros((self.max_rows, W, 4), dtype=torch.float32, device=cdev) for _ in range(self.gworld)]
                      if self.rank == 0 else None for _ in range(2)]
        self.send, self.recv = self.sendb[0], self.recvb[0]
        self._slot = 0
        self._work = [None, None]
        self._last = None
        self._newest = 0
        self.image = torch.zeros((H, W, 4), dtype=torch.float32, device=self.device) if self.rank == 0 else None

    def render(self, first_frame: int, n_frames: int):
        """Asynchronously render frames first..first+n-1 of this rank's rows."""
        self.tracer.render(first_frame, n_frames, self.band, self.world, self.rank)

    def _gather(self) -> torch.Tensor | None:
        """Pack this rank's rows, gather on rank 0; returns the H x W x 4 image
        (row 0 = bottom) on rank 0 and None elsewhere."""
        if self.my_rows:
            self.tracer.pack_rows(self.send.data_ptr(), self.band, self.world, self.rank)
        if self.world == 1 and not self.collective:
            self.image.copy_(self.send)
            return self.image
        if not dist.is_initialized():
            raise RuntimeError("ShardedFrame: a shard= split without a process group cannot gather")
        send = self.send.cpu() if self.stage else self.send
        dist.gather(send, self.recv if self.rank == 0 else None, dst=0, group=self.group)
        if self.rank != 0:
            return None
        return self._assemble(self.recv)

    def _on_stream(self, fn):
        if self.stream is None:
            return fn()
        with torch.cuda.stream(self.stream):
            return fn()

    def gather(self) -> torch.Tensor | None:
        """Pack this rank's rows, gather on rank 0; returns the H x W x 4 image
        (row 0 = bottom) on rank 0 and None elsewhere."""
        return self._on_stream(self._gather)

    def gather_async(self) -> None:
        """Start the gather of the current frame (see _gather_async)."""
        return self._on_stream(self._gather_async)

    def finish(self) -> torch.Tensor | None:
        """Complete the outstanding gathers; rank 0 gets the newest frame's image."""
        return self._on_stream(self._finish)

    def _assemble(self, recv) -> torch.Tensor:
        # device images from a tracer that can unpack: the library's own kernel on its stream
        # (torch's index_copy_ there left the library's later kernels 5-10 % slower on the
        # one-GPU box, tools/share_bench.py -- DESIGN.md section 17)
        lib = (self.device.type == "cuda" and hasattr(self.tracer, "unpack_rows") and
               all(t.device == self.device for t in recv))
        for r in range(len(recv)):
            n = len(self.rows[r])
            if not n:
                continue
            if lib:
                self.tracer.unpack_rows(recv[r].data_ptr(), self.image.data_ptr(), self.band, self.world, r)
            else:
                self.image.index_copy_(0, self.rows[r], recv[r][:n].to(self.device, non_blocking=False))
        return self.image

    def _gather_async(self) -> None:
        """Pack this rank's rows and START the gather (RCCL) without making the
        render stream wait for it: the next frames render while the rows travel
        over xGMI.  Double-buffered; :meth:`finish` completes the last gather and
        assembles the image on rank 0.  (Synchronous for one rank / gloo staging.)"""
        if (self.world == 1 and not self.collective) or self.stage:
            self._last = self._gather()
            return
        slot = self._slot
        self._slot ^= 1
        if self._work[slot] is not None:       # this slot's previous gather must be done before
            self._work[slot].wait()            # its send buffer is repacked (stream-ordered wait)
            self._work[slot] = None
        if self.my_rows:
            self.tracer.pack_rows(self.sendb[slot].data_ptr(), self.band, self.world, self.rank)
        self._work[slot] = dist.gather(self.sendb[slot], self.recvb[slot] if self.rank == 0 else None, dst=0,
                                       group=self.group, async_op=True)
        self._newest = slot

    def _finish(self) -> torch.Tensor | None:
        """Complete the outstanding gathers; rank 0 gets the newest frame's image."""
        if (self.world == 1 and not self.collective) or self.stage:
            return self._last
        for slot in (self._newest ^ 1, self._newest):
            if self._work[slot] is not None:
                self._work[slot].wait()
                self._work[slot] = None
        return self._assemble(self.recvb[self._newest]) if self.rank == 0 else None


def row_owner(height: int, band: int, world: int) -> np.ndarray:
    """Rank that owns each row (for tests and tools)."""
    return (np.arange(height) // band) % world
