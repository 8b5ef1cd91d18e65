"""Multi-rank rendering with real renderer output: 2 processes share device 0,
each renders its 1-row stripes (rt_amd/shard.py) with rt_render_device, the frames are gathered
to rank 0 over gloo from host copies (on an 8-GPU node the same gather runs over RCCL, bench.py),
and the assembled frame must equal the 1-rank frame bit for bit — the RNG and the running mean
are keyed on the global pixel and the absolute sample."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scene, spp, batch, result_path):
    import sys

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "gpu-ray_trace-rust_amd"), os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from conftest import load_scene
    from rt_amd import render, shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        sc = load_scene(scene)
        w, h = int(sc.info.width), int(sc.info.height)
        tiles = shard.rank_tiles(w, h, rank, world)
        n = shard.max_rank_pixels(w, h, world)
        torch.cuda.set_device(0)
        buf = torch.zeros((n, 4), dtype=torch.float32, device="cuda:0")
        with render.Context(sc, device=0) as ctx:
            for s0 in range(0, spp, batch):
                torch.cuda.current_stream().synchronize()
                ctx.render_device(buf.data_ptr(), tiles, s0, batch)
        torch.cuda.synchronize()
        frame = shard.gather_frame(buf.cpu(), w, h, rank, world, dist)
        if rank == 0:
            np.save(result_path, frame.numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("scene,spp,batch", [("walled", 6, 3), ("biplane", 2, 1)])
def test_two_ranks_equal_one(gpu_available, tmp_path, scene, spp, batch):
    import torch.multiprocessing as mp

    from conftest import load_scene
    from rt_amd import render

    res = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(WORLD, _free_port(), scene, spp, batch, res), nprocs=WORLD, join=True)
    got = np.load(res)
    sc = load_scene(scene)
    w, h = int(sc.info.width), int(sc.info.height)
    with render.Context(sc) as ctx:
        for s0 in range(0, spp, batch):
            one = ctx.render(None, s0, batch, want_output=(s0 + batch >= spp))
    one = one.reshape(h, w, 4)
    assert (got[..., 3] == 1.0).all()  # every pixel rendered by some rank
    assert np.array_equal(got, one)
