"""Multi-process row-band sharding + gather on CPU: gloo,
world size 2 (and 3), the oracle standing in for each rank's GPU.  The
gathered image must equal a single-process render bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, w, h, band, frames, out_path, overlap=False):
    sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle")); sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_tracer import OracleTracer
    from pnraytracing_amd import scenes as S
    from pnraytracing_amd.dist import ShardedFrame
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        tr = OracleTracer(S.cornell_c1(w, h))
        sf = ShardedFrame(tr, band=band, device="cpu")
        if overlap:                 # bench.py's per-step pattern: render, start the gather, ...
            for f0, n in frames:
                sf.render(f0, n)
                sf.gather_async()
            img = sf.finish()
        else:
            for f0, n in frames:
                sf.render(f0, n)
            img = sf.gather()
        # ranks render only their own rows
        from pnraytracing_amd.dist import row_owner
        mine = row_owner(h, band, world) == rank
        assert not tr.accum[~mine].any()
        if rank == 0:
            np.save(out_path, img.numpy())
        else:
            assert img is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h,band,overlap", [(2, 40, 44, 8, False), (3, 24, 20, 4, False), (2, 40, 44, 8, True),
                                                   (3, 24, 20, 4, True)])
def test_gather_equals_single_process(tmp_path, world, w, h, band, overlap):
    import pyoracle
    from pnraytracing_amd import scenes as S
    frames = [(0, 1), (1, 2), (3, 1)]
    out = str(tmp_path / "img.npy")
    mp.start_processes(_worker, args=(world, _free_port(), w, h, band, frames, out, overlap), nprocs=world,
                       join=True, start_method="spawn")
    got = np.load(out)
    o = pyoracle.Oracle(S.cornell_c1(w, h))
    ref = np.zeros((h, w, 4), np.float32)
    for f0, n in frames:
        o.render(f0, n, accum=ref)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def _plan_worker(rank, world, port, w, h, band, slots, spp, warm, steps, out_path):
    """bench.py's own call planning and call loop on a frame whose largest share
    crosses the batch threshold while the smaller one does not."""
    sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle")); sys.path.insert(0, os.path.join(REPO, "tests"))
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from oracle_tracer import OracleTracer
    from pnraytracing_amd import scenes as S
    from pnraytracing_amd.dist import ShardedFrame
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        tr = OracleTracer(S.cornell_c1(w, h))
        sf = ShardedFrame(tr, band=band, device="cpu")
        ns = type("A", (), {"iters_per_call": 0, "steps": steps})()
        own = [None] * world                      # what each rank would plan from its OWN share
        dist.all_gather_object(own, bench.iters_per_call(ns, sf.my_rows * w, batch_slots=slots, shards=world))
        assert len(set(own)) > 1, own             # the hazard is present in this frame
        ipc = bench.iters_per_call(ns, sf.max_rows * w, batch_slots=slots, shards=world)   # as bench.py
        bench.same_on_all_ranks([ipc, len(bench.call_groups(0, warm, ipc)),
                                 len(bench.call_groups(warm, warm + steps, ipc))], "cpu")
        n = bench.issue_calls(sf, spp, 0, warm, ipc, world)
        sf.finish()
        n += bench.issue_calls(sf, spp, warm, warm + steps, ipc, world)
        img = sf.finish()
        counts = [None] * world
        dist.all_gather_object(counts, n)
        assert len(set(counts)) == 1, counts      # every rank issued the same gathers
        if rank == 0:
            np.save(out_path, img.numpy())
    finally:
        dist.destroy_process_group()


def test_bench_gather_count_same_on_every_rank(tmp_path):
    """bench.py plans its pnrt_render calls -- and so its gathers -- from the
    largest share: ranks whose own shares fall on either side of the batch
    threshold still issue the same number of gathers (a mismatch hangs RCCL), and
    the gathered image equals one process's render."""
    import pyoracle
    from pnraytracing_amd import scenes as S
    w, h, band, spp, warm, steps = 40, 44, 8, 2, 1, 3
    slots = 20 * w * 8            # rank 1's 20 rows fit 8 frames (calls of 2 iterations), rank 0's 24 only 6 (1)
    out = str(tmp_path / "img.npy")
    mp.start_processes(_plan_worker, args=(2, _free_port(), w, h, band, slots, spp, warm, steps, out), nprocs=2,
                       join=True, start_method="spawn")
    got = np.load(out)
    o = pyoracle.Oracle(S.cornell_c1(w, h))
    ref = np.zeros((h, w, 4), np.float32)
    o.render(0, spp * (warm + steps), accum=ref)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_single_rank_without_process_group():
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_tracer import OracleTracer
    from pnraytracing_amd import scenes as S
    from pnraytracing_amd.dist import ShardedFrame
    tr = OracleTracer(S.cornell_c1(16, 12))
    sf = ShardedFrame(tr, device="cpu")
    sf.render(0, 1)
    img = sf.gather()
    assert img.shape == (12, 16, 4) and np.array_equal(img.numpy(), tr.accum)


def _share_worker(rank, world, port, w, h, band, split, frames, out_path):
    """Rank 0's share of a `split`-way frame gathered through a ONE-rank group
    (tools/share_bench.py --collective): bench.py's render / gather_async / finish."""
    sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle")); sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_tracer import OracleTracer
    from pnraytracing_amd import scenes as S
    from pnraytracing_amd.dist import ShardedFrame
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        tr = OracleTracer(S.cornell_c1(w, h))
        with pytest.raises(ValueError):        # a split's share needs collective=True over a one-rank group
            ShardedFrame(tr, band=band, device="cpu", shard=(split, 0))
        sf = ShardedFrame(tr, band=band, device="cpu", collective=True, shard=(split, 0))
        assert sf.world == split and sf.rank == 0 and sf.gworld == 1
        for f0, n in frames:
            sf.render(f0, n)
            sf.gather_async()
        np.save(out_path, sf.finish().numpy())
    finally:
        dist.destroy_process_group()


def test_share_gathered_through_one_rank_group(tmp_path):
    """VERDICT r5 "Next" 6: rank 0's share of a 3-way split, gathered through a
    one-rank group, assembles exactly rank 0's rows of the full render (the other
    rows stay zero) -- the path tools/share_bench.py --collective times."""
    import pyoracle
    from pnraytracing_amd import scenes as S
    from pnraytracing_amd.dist import row_owner
    w, h, band, split = 24, 20, 4, 3
    frames = [(0, 1), (1, 2)]
    out = str(tmp_path / "img.npy")
    mp.start_processes(_share_worker, args=(1, _free_port(), w, h, band, split, frames, out), nprocs=1, join=True,
                       start_method="spawn")
    got = np.load(out)
    o = pyoracle.Oracle(S.cornell_c1(w, h))
    ref = np.zeros((h, w, 4), np.float32)
    for f0, n in frames:
        o.render(f0, n, accum=ref)
    mine = row_owner(h, band, split) == 0
    assert np.array_equal(got[mine].view(np.uint32), ref[mine].view(np.uint32))
    assert not got[~mine].any()
