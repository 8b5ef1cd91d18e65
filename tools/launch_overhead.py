"""Fixed cost of one queue launch (start-up + drain tail): walled.yml rendered in ONE launch at
several spp (RT_DEBUG_LAUNCH radiance_gib raised so that 2000 spp still fit one launch), kernel time from
the launch's HIP events; a least-squares line ms = a + b * spp gives the per-launch intercept a.
Usage: python tools/launch_overhead.py [--scene walled] [--spp 250 500 1000 2000]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="walled")
    ap.add_argument("--spp", type=int, nargs="+", default=[250, 500, 1000, 2000])
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    os.environ.setdefault("RT_DEBUG_LAUNCH", "radiance_gib=32")
    import numpy as np
    import torch  # noqa: F401  (owns the HIP runtime)
    from rt_amd import render, scheme

    sch = scheme.load_json(os.path.join(ROOT, "tests", "golden", "scenes", a.scene + ".json"))
    loaded = scheme.load(sch, assets_root=os.path.join(ROOT, "assets_pack"))
    ctx = render.Context(loaded)
    ctx.render(None, 0, min(a.spp), want_output=False)  # warm-up
    best = {}
    for _ in range(a.rounds):
        for spp in a.spp:
            ctx.render(None, 0, spp, want_output=False)
            ms = ctx.last_kernel_ms()
            best[spp] = min(best.get(spp, ms), ms)
    x = np.array(sorted(best), dtype=float)
    y = np.array([best[s] for s in sorted(best)])
    b, c = np.polyfit(x, y, 1)
    print(json.dumps({"scene": a.scene, "kernel_ms": {str(int(s)): round(best[s], 3) for s in sorted(best)},
                      "ms_per_spp": round(b, 5), "intercept_ms_per_launch": round(c, 3)}))


if __name__ == "__main__":
    main()
