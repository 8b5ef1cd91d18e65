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
