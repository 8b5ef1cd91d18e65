"""A/B, in one process: the 1-GPU step (whole frame, spp) against rank 0's share of an N-rank
step (its stripes, N x spp), alternating, on one context.  Prints Msamples/s per round.
Usage: python tools/tiling_ab.py [--scene walled] [--spp 1000] [--ranks 2 8] [--stripe 1]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="walled")
    ap.add_argument("--spp", type=int, default=1000)
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 8])
    ap.add_argument("--stripes", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    from rt_amd import render, scheme, shard

    sch = scheme.load_json(os.path.join(ROOT, "tests", "golden", "scenes", a.scene + ".json"))
    loaded = scheme.load(sch, assets_root=os.path.join(ROOT, "assets_pack"))
    w, h = int(loaded.info.width), int(loaded.info.height)
    ctx = render.Context(loaded)
    out = torch.zeros((w * h, 4), dtype=torch.float32, device="cuda:0")
    cases = [("n1", [(0, 0, w, h)], a.spp)]
    for n in a.ranks:
        for s in a.stripes:
            cases.append((f"rank0of{n}_stripe{s}", shard.rank_tiles(w, h, 0, n, s), a.spp * n))
    res = {c[0]: [] for c in cases}
    sample = 0
    for r in range(a.rounds + 1):
        for name, tiles, spp in cases:
            npix = sum(t[2] * t[3] for t in tiles)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.render_device(out.data_ptr(), tiles, sample, spp)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            sample += spp
            if r:
                res[name].append(round(npix * spp / dt / 1e6, 1))
    for k, v in res.items():
        print(json.dumps({"case": k, "Msamples_s": v, "best": max(v)}))


if __name__ == "__main__":
    main()
