"""Multi-GPU sharding (rt_amd/shard.py, bench.py): the stripe partition covers every pixel once,
and the frame-end gather + assembly rebuilds the frame — run with world_size 2 on the gloo
backend (CPU; on MI355X the same calls run over RCCL)."""
import os
import socket

import numpy as np
import pytest


@pytest.mark.parametrize("w,h", [(1200, 600), (4096, 4096), (64, 37), (10, 3)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_stripes_partition_the_frame(w, h, world):
    from rt_amd import shard

    cover = np.zeros((h, w), np.int32)
    for r in range(world):
        tiles = shard.rank_tiles(w, h, r, world)
        for (x0, y0, tw, th) in tiles:
            assert x0 == 0 and tw == w and th > 0
            cover[y0:y0 + th, x0:x0 + tw] += 1
        assert shard.tile_pixels(tiles) <= shard.max_rank_pixels(w, h, world)
    assert (cover == 1).all()
    # balance: ranks differ by at most one stripe
    sizes = [shard.tile_pixels(shard.rank_tiles(w, h, r, world)) for r in range(world)]
    stripe = shard.stripe_rows(h, world)
    assert max(sizes) - min(sizes) <= stripe * w
    if h % (stripe * world) == 0:
        assert max(sizes) == min(sizes)


def test_stripe_rows():
    from rt_amd import shard

    assert [shard.stripe_rows(600, n) for n in (1, 2, 4, 8)] == [8, 6, 6, 5]
    assert [shard.stripe_rows(4096, n) for n in (1, 2, 4, 8)] == [8, 8, 8, 8]
    assert shard.stripe_rows(37, 8) == 1


def _pattern(w, h, tiles, n):
    """What a rank 'renders': pixel (x, y) -> (y*w + x, y, x, 1) for its tiles, in tile order."""
    buf = np.zeros((n, 4), np.float32)
    off = 0
    for (x0, y0, tw, th) in tiles:
        ys, xs = np.mgrid[y0:y0 + th, x0:x0 + tw]
        buf[off:off + tw * th] = np.stack([ys * w + xs, ys, xs, np.ones_like(xs)], -1).reshape(-1, 4)
        off += tw * th
    return buf


def _worker(rank, world, port, w, h, result_path):
    import torch
    import torch.distributed as dist

    from rt_amd import shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        n = shard.max_rank_pixels(w, h, world)
        buf = torch.from_numpy(_pattern(w, h, shard.rank_tiles(w, h, rank, world), n))
        frame = shard.gather_frame(buf, w, h, rank, world, dist)
        if rank == 0:
            ys, xs = np.mgrid[0:h, 0:w]
            want = np.stack([ys * w + xs, ys, xs, np.ones_like(xs)], -1).astype(np.float32)
            np.save(result_path, np.array([np.array_equal(frame.numpy(), want)]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("w,h", [(64, 37), (120, 60)])
def test_gloo_world2_gather_assembles_the_frame(tmp_path, w, h):
    import torch.multiprocessing as mp

    res = str(tmp_path / "ok.npy")
    mp.spawn(_worker, args=(2, _free_port(), w, h, res), nprocs=2, join=True)
    assert bool(np.load(res)[0])


def test_assemble_single_rank_is_identity():
    from rt_amd import shard

    w, h = 33, 10
    buf = _pattern(w, h, shard.rank_tiles(w, h, 0, 1), w * h)
    frame = shard.assemble([buf], w, h, 1)
    assert np.array_equal(frame.reshape(-1, 4), buf)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_step_sample_accounting(world):
    """bench.py's accounting (rt_amd.shard.step_samples): strong keeps the job at W*H*spp per step
    whatever N, each rank spp per pixel of its 1/N of the frame; weak gives every rank the 1-GPU
    step's work, W*H/N pixels at N*spp, so the job is N times the 1-GPU step."""
    from rt_amd import shard

    w, h, spp = 1200, 600, 1000
    s_rank, s_job = shard.step_samples(w, h, spp, world, strong=True)
    assert (s_rank, s_job) == (spp, w * h * spp)
    w_rank, w_job = shard.step_samples(w, h, spp, world, strong=False)
    assert (w_rank, w_job) == (spp * world, w * h * spp * world)
    # every rank's share of one step, summed over ranks, is the job
    stripe = shard.stripe_rows(h, world)
    for spp_rank, job in ((s_rank, s_job), (w_rank, w_job)):
        assert sum(shard.tile_pixels(shard.rank_tiles(w, h, r, world, stripe)) * spp_rank
                   for r in range(world)) == job
        # and with equal stripe counts each rank's share is job / N (balanced)
        assert {shard.tile_pixels(shard.rank_tiles(w, h, r, world, stripe)) * spp_rank
                for r in range(world)} == {job // world}
