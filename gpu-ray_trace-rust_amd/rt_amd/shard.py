"""Multi-GPU sharding of one frame: pixels are dealt to ranks as stripes of a few
rows, round-robin, so sky-only and geometry-heavy rows spread over every rank.  Each rank
renders its stripes for the whole sample range (rt_render_device into one buffer, its tiles
concatenated in order); one collective per frame — a gather to rank 0 (RCCL over xGMI on
MI355X, gloo in the CPU tests) — and rank 0 reassembles the frame.  A pixel's value does not
depend on which rank renders it (RNG and running mean are keyed on the global pixel and the
absolute sample), so the assembled frame equals the 1-GPU frame bit for bit."""
from __future__ import annotations

STRIPE_MAX = 8  # rows: the queue hands out a launch's pixels in 8 x 8 blocks (RT_PIX_BLOCK)


def stripe_rows(height: int, world: int) -> int:
    """Rows per stripe: the tallest S <= STRIPE_MAX that deals every rank the same number of
    stripes (height % (S * world) == 0), else 1.  Taller stripes let the queue order's 8 x 8
    blocks, and with them the camera-ray packets of the mesh kernel, form inside a rank's share
    (1-row stripes leave 64 x 1 strips); equal counts keep the ranks balanced.  600 rows: 5 / 6
    rows over 8 / 2 ranks; 4096 rows: 8."""
    for s in range(STRIPE_MAX, 0, -1):
        if height % (s * world) == 0:
            return s
    return 1


def rank_tiles(width: int, height: int, rank: int, world: int, stripe: int | None = None):
    """rank's stripes as (x0, y0, w, h) tiles; consecutive stripes of one rank merge."""
    stripe = stripe or stripe_rows(height, world)
    tiles = []
    for i, y0 in enumerate(range(0, height, stripe)):
        if i % world == rank:
            hh = min(stripe, height - y0)
            if tiles and tiles[-1][1] + tiles[-1][3] == y0:
                x, yy, ww, h0 = tiles[-1]
                tiles[-1] = (x, yy, ww, h0 + hh)
            else:
                tiles.append((0, y0, width, hh))
    return tiles


def tile_pixels(tiles) -> int:
    return int(sum(t[2] * t[3] for t in tiles))


def max_rank_pixels(width: int, height: int, world: int, stripe: int | None = None) -> int:
    """Size of the per-rank buffer: every rank gathers a buffer of this many pixels."""
    return max(tile_pixels(rank_tiles(width, height, r, world, stripe)) for r in range(world))


def assemble(parts, width: int, height: int, world: int, stripe: int | None = None):
    """Frame (height, width, C) from every rank's gathered buffer (rank r's tiles concatenated
    at the start of parts[r]).  Works on numpy arrays and torch tensors alike."""
    import numpy as np

    first = parts[0]
    frame = (first.new_zeros((height, width, first.shape[-1])) if hasattr(first, "new_zeros")
             else np.zeros((height, width, first.shape[-1]), first.dtype))
    for r in range(world):
        off = 0
        for (x0, y0, w, h) in rank_tiles(width, height, r, world, stripe):
            frame[y0:y0 + h, x0:x0 + w] = parts[r][off:off + w * h].reshape(h, w, -1)
            off += w * h
    return frame


def gather_frame(buf, width: int, height: int, rank: int, world: int, dist, gather_list=None):
    """The frame-end collective: every rank's buffer to rank 0, which returns the assembled
    frame (other ranks return None).  `gather_list` may be preallocated on rank 0."""
    if world == 1:
        return assemble([buf], width, height, 1)
    if rank == 0 and gather_list is None:
        gather_list = [buf.new_empty(buf.shape) for _ in range(world)]
    dist.gather(buf, gather_list=gather_list if rank == 0 else None, dst=0)
    return assemble(gather_list, width, height, world) if rank == 0 else None


def step_samples(width: int, height: int, spp: int, world: int, strong: bool) -> tuple:
    """Sample accounting of one multi-rank step (bench.py): (spp every rank renders for each of
    its pixels, samples all ranks render together).  Strong scaling keeps the frame fixed: the
    ranks split W*H pixels at spp, so the job is W*H*spp whatever N.  Weak scaling keeps each
    rank's work at the 1-GPU step's: W*H/N pixels at N*spp, so the job grows to W*H*N*spp."""
    spp_rank = spp if strong else spp * world
    return spp_rank, width * height * spp_rank


GATHER_MODES = ("frame", "step")


def gather_steps(steps: int, mode: str) -> list:
    """Which of a run's `steps` steps end in the gather: "frame" (north_star's single gather of
    tile radiance at frame end) only the last one; "step" (the reference's per-batch read-back,
    draw_scene.rs:34-42) every one."""
    if mode not in GATHER_MODES:
        raise ValueError(f"gather mode {mode!r}: one of {GATHER_MODES}")
    return [mode == "step" or i == steps - 1 for i in range(steps)]


class FrameSteps:
    """The step loop of a sharded frame, as bench.py times it and the multi-rank
    tests run it: each step renders `spp_rank` more samples of this rank's stripes into one device
    buffer (rt_render_device_async on torch's current stream, or the synchronous rt_render_device);
    the gather of every rank's buffer to rank 0 — the one collective — runs after the last step of
    the frame (gather="frame") or after every step (gather="step").  backend "nccl" (RCCL over
    xGMI) gathers the device buffers on torch's stream behind the step's fold; "gloo" gathers host
    copies (several ranks sharing one GPU, where RCCL refuses)."""

    def __init__(self, ctx, tiles, width: int, height: int, rank: int, world: int, stripe: int,
                 spp_rank: int, device: int, dist=None, backend: str = "nccl", sync: bool = False,
                 gather: str = "frame"):
        import torch

        self.torch = torch
        self.ctx, self.tiles = ctx, tiles
        self.width, self.height, self.rank, self.world, self.stripe = width, height, rank, world, stripe
        self.spp_rank, self.dist, self.backend, self.sync = spp_rank, dist, backend, sync
        gather_steps(1, gather)  # validates the mode
        self.gather_mode = gather
        self.n_gathers = 0
        self.npix = tile_pixels(tiles)
        n = max(max_rank_pixels(width, height, world, stripe), self.npix)
        # device None: host buffers and no HIP at all (the CPU tests' stand-in context)
        self.on_cpu = device is None
        self.out = torch.zeros((n, 4), dtype=torch.float32, device="cpu" if self.on_cpu else f"cuda:{device}")
        self.device = device
        on_host = backend == "gloo" or self.on_cpu
        self.gather = None
        if dist is not None and rank == 0:
            self.gather = [torch.empty((n, 4), dtype=torch.float32, device="cpu" if on_host else f"cuda:{device}")
                           for _ in range(world)]
        self.stream = 0 if self.on_cpu else torch.cuda.current_stream().cuda_stream
        self.sample = 0
        self.gather_ev = []
        self.gather_s = []
        self.sync_stats = []

    def step(self, gather: bool = True):
        torch = self.torch
        self.host_frame_parts = None  # run()'s host copy is stale once another step runs
        if self.sync:
            self.ctx.render_device(self.out.data_ptr(), self.tiles, self.sample, self.spp_rank)
            self.sync_stats.append(self.ctx.launch_stats())  # each synchronous call is its own window
        else:
            self.ctx.render_device_async(self.out.data_ptr(), self.tiles, self.sample, self.spp_rank,
                                         stream=self.stream)
        self.sample += self.spp_rank
        if self.dist is None or not gather:
            return
        self.n_gathers += 1
        if self.backend == "gloo":
            import time

            t0 = time.perf_counter()
            host = self.out.cpu()  # ordered after the step's fold on torch's stream
            self.dist.gather(host, gather_list=self.gather, dst=0)
            self.gather_s.append(time.perf_counter() - t0)
        else:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            self.dist.gather(self.out, gather_list=self.gather, dst=0)
            e1.record()
            self.gather_ev.append((e0, e1))

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()
        if not self.on_cpu:
            self.torch.cuda.synchronize()

    def run(self, steps: int, warmup: int) -> dict:
        """W untimed steps, then exactly `steps` steps between barrier + synchronize on both
        sides; the elapsed time is the maximum over ranks.  Returns {elapsed_s, launch stats of
        the timed steps, gather_ms_per_step}."""
        import time

        for g in gather_steps(warmup, self.gather_mode) if warmup else []:
            self.step(gather=g)
        self.ctx.synchronize()
        self.barrier()
        self.gather_ev.clear()
        self.gather_s.clear()
        self.sync_stats.clear()
        self.n_gathers = 0
        t0 = time.perf_counter()
        for g in gather_steps(steps, self.gather_mode):
            self.step(gather=g)
        self.ctx.synchronize()
        self.barrier()
        elapsed = time.perf_counter() - t0
        # the final result on the host: one D2H copy of the frame after the timed
        # steps, timed on its own (rank 0: the gathered buffers; every rank waits for it)
        t1 = time.perf_counter()
        if self.rank == 0:
            parts = self.gather if self.dist is not None else [self.out]
            self.host_frame_parts = [p.cpu() for p in parts]
        self.barrier()
        host_copy = time.perf_counter() - t1
        if self.sync:
            ls = {k: sum(s[k] for s in self.sync_stats)
                  for k in ("render_ms", "trace_ms", "n_trace_launches", "n_timed_launches")}
        else:
            ls = self.ctx.launch_stats()
        if self.dist is not None:
            t = self.torch.tensor([elapsed], device="cpu" if self.backend == "gloo" or self.on_cpu else f"cuda:{self.device}")
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            elapsed = float(t.item())
        if self.dist is not None:
            t = self.torch.tensor([host_copy], device="cpu" if self.backend == "gloo" or self.on_cpu else f"cuda:{self.device}")
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
            host_copy = float(t.item())
        res = {"elapsed_s": elapsed, "launch": ls, "host_copy_s": host_copy, "gathers": self.n_gathers,
               "gather_mode": self.gather_mode}
        # gather time: per gather, and spread over the run's steps (one gather per frame: / steps)
        if self.gather_ev:
            tot = sum(a.elapsed_time(b) for a, b in self.gather_ev)
        elif self.gather_s:
            tot = 1e3 * sum(self.gather_s)
        else:
            tot = None
        if tot is not None:
            n = len(self.gather_ev) or len(self.gather_s)
            res.update(gather_ms_per_gather=tot / n, gather_ms_per_step=tot / steps)
        return res

    def frame(self):
        """Rank 0: the last step's frame assembled from every rank's gathered buffer (H, W, 4) as
        a host array (the single-rank frame for world 1); None elsewhere."""
        if self.rank != 0:
            return None
        parts = getattr(self, "host_frame_parts", None) or (self.gather if self.dist is not None else [self.out])
        f = assemble(parts, self.width, self.height, self.world, self.stripe)
        return f.cpu().numpy() if hasattr(f, "cpu") else f
