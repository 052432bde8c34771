"""Test-only stand-in for PathTracer on hosts without a GPU: the tracer
protocol of pnraytracing_amd.dist (render with a row-band shard selector,
pack_rows into a host pointer) implemented on the CPU oracle.  Used by the
gloo multi-process tests; never by the product path."""
import ctypes

import numpy as np

import pyoracle
from pnraytracing_amd.tracer import shard_rows


class OracleTracer:
    def __init__(self, cfg, threads=2):
        self.cfg, self.threads = cfg, threads
        self.width, self.height = cfg.width, cfg.height
        self.oracle = pyoracle.Oracle(cfg)
        self.accum = np.zeros((cfg.height, cfg.width, 4), np.float32)

    def render(self, first, n, band=1, n_shards=1, shard=0):
        for y0 in range(shard * band, self.height, band * n_shards):
            self.oracle.render(first, n, rows=(y0, min(y0 + band, self.height)), accum=self.accum,
                               threads=self.threads)

    def pack_rows(self, dst_ptr, band, n_shards, shard):
        rows = np.ascontiguousarray(self.accum[shard_rows(self.height, band, n_shards, shard)])
        ctypes.memmove(dst_ptr, rows.ctypes.data, rows.nbytes)
