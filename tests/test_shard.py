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


@pytest.mark.parametrize("steps", [1, 3, 7])
def test_gather_steps_pin_which_steps_gather(steps):
    """"frame" (north_star's single gather at frame end): only the last step gathers; "step"
    (the reference's per-batch read-back): every step does."""
    from rt_amd import shard

    assert shard.gather_steps(steps, "frame") == [False] * (steps - 1) + [True]
    assert shard.gather_steps(steps, "step") == [True] * steps
    with pytest.raises(ValueError):
        shard.gather_steps(steps, "never")


class _PatternCtx:
    """Stand-in for render.Context on the CPU: writes, into the rank's host buffer, the value
    every pixel of its tiles would hold after `sample_end` samples (pixel index, sample_end)."""

    def __init__(self, w):
        self.w, self.calls = w, []

    def render_device_async(self, ptr, tiles, s0, n, stream=0):
        import ctypes as C

        from rt_amd import shard

        npx = shard.tile_pixels(tiles)
        buf = np.ctypeslib.as_array((C.c_float * (4 * npx)).from_address(ptr)).reshape(npx, 4)
        off = 0
        for (x0, y0, tw, th) in tiles:
            ys, xs = np.mgrid[y0:y0 + th, x0:x0 + tw]
            buf[off:off + tw * th, 0] = (ys * self.w + xs).ravel()
            buf[off:off + tw * th, 1] = s0 + n
            buf[off:off + tw * th, 3] = 1.0
            off += tw * th
        self.calls.append((s0, n))

    def synchronize(self):
        pass

    def launch_stats(self):
        return {"render_ms": 0.0, "trace_ms": 0.0, "n_trace_launches": len(self.calls), "n_timed_launches": 0}


def _frame_steps_worker(rank, world, port, mode, res_path):
    import torch.distributed as dist

    from rt_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, h, spp, steps = 40, 24, 3, 4
        stripe = shard.stripe_rows(h, world)
        tiles = shard.rank_tiles(w, h, rank, world, stripe)
        fs = shard.FrameSteps(_PatternCtx(w), tiles, w, h, rank, world, stripe, spp, None, dist=dist,
                              backend="gloo", gather=mode)
        r = fs.run(steps, 2)
        if rank == 0:
            f = fs.frame()
            ok = bool((f[..., 3] == 1).all() and (f[..., 1] == (2 + steps) * spp).all()
                      and (f[..., 0] == np.arange(w * h).reshape(h, w)).all())
            np.save(res_path, np.array([ok, r["gathers"], len(fs.ctx.calls)]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,gathers", [("frame", 1), ("step", 4)])
def test_frame_steps_gathers_world2(tmp_path, mode, gathers):
    """FrameSteps over gloo with two ranks (a CPU stand-in context): 4 timed steps after 2 warmup
    ones; "frame" gathers once, after the last step, "step" after each; either way rank 0's frame
    is every pixel after all 6 steps' samples."""
    import torch.multiprocessing as mp

    res = str(tmp_path / "r.npy")
    mp.spawn(_frame_steps_worker, args=(2, _free_port(), mode, res), nprocs=2, join=True)
    ok, n_gathers, calls = np.load(res)
    assert ok and n_gathers == gathers and calls == 6


def test_frame_after_more_steps_is_not_stale():
    """run() keeps a host copy of the frame; a step() after run() must drop it, so
    frame() then reassembles the current buffer (one rank, no collective) instead of returning
    the frame from before that step."""
    from rt_amd import shard

    w, h, spp = 16, 8, 2
    tiles = [(0, 0, w, h)]
    fs = shard.FrameSteps(_PatternCtx(w), tiles, w, h, 0, 1, 8, spp, None)
    fs.run(2, 1)
    assert (fs.frame()[..., 1] == 3 * spp).all()
    fs.step()
    assert (fs.frame()[..., 1] == 4 * spp).all()
