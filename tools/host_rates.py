"""Host-buffer (PCIe-inclusive) rates of the drop-in boundary, beside bench.py's device-resident
value: rt_render into a host buffer per call (the frame copied back after every call), and
rt_render_to_target, the reference's whole render_to_target_gpu (draw_scene.rs:17-47: scene upload
and KD build, every batch, the RGBA8 frame back to the host after each batch).
Usage: python tools/host_rates.py   (on the GPU box)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402,F401  (owns the HIP runtime, as in bench.py)
from conftest import load_scene  # noqa: E402
from rt_amd import render  # noqa: E402


def rt_render_rate(name, spp, calls, **kw):
    sc = load_scene(name, **kw)
    w, h = int(sc.info.width), int(sc.info.height)
    with render.Context(sc) as ctx:
        ctx.render(None, 0, spp)  # warm-up
        t0 = time.perf_counter()
        for i in range(calls):
            ctx.render(None, (i + 1) * spp, spp)
        dt = time.perf_counter() - t0
    return {"call": "rt_render (host buffer)", "scene": name, "pixels": w * h, "spp_per_call": spp,
            "calls": calls, "Msamples_s": round(w * h * spp * calls / dt / 1e6, 1),
            "ms_per_call": round(dt / calls * 1e3, 2)}


def to_target_rate(name, spp, batch, **kw):
    sc = load_scene(name, **kw)
    w, h = int(sc.info.width), int(sc.info.height)
    render.render_to_target(sc, 0, batch)  # first-touch costs of the process, untimed
    t0 = time.perf_counter()
    render.render_to_target(sc, 0, batch)  # zero batches: rt_create (KD build, uploads) + rt_destroy
    setup = time.perf_counter() - t0
    t0 = time.perf_counter()
    with render.Context(sc):
        pass
    create = time.perf_counter() - t0
    t0 = time.perf_counter()
    img = render.render_to_target(sc, spp, batch)
    dt = time.perf_counter() - t0
    assert img.shape == (h, w, 4)
    return {"call": "rt_render_to_target (scene upload + KD build + every batch + RGBA8 readbacks)",
            "scene": name, "pixels": w * h, "spp": spp, "batch": batch, "seconds": round(dt, 3),
            "Msamples_s": round(w * h * spp / dt / 1e6, 1), "setup_s": round(setup, 3),
            "rt_create_s": round(create, 3)}


for r in (rt_render_rate("walled", 1000, 5),
          to_target_rate("walled", 20000, 1000),
          to_target_rate("biplane", 200, 10),
          to_target_rate("a380", 10, 1),
          to_target_rate("spaceship_r1", 100, 25, width=4096, height=4096)):
    print(json.dumps(r), flush=True)
