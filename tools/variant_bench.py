"""A/B timing of kernel variants in ONE process, interleaved rounds (cdna guide §5.4 rule 24).
Usage: python tools/variant_bench.py [--scene walled] [--spp 32] [--rounds 3] name1[:VAR=VAL,...] ...
("main" is lib/librt_amd.so; other names lib/variants/librt_<name>.so)"""
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
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("names", nargs="+")
    a = ap.parse_args()
    import torch  # noqa: F401  (owns the HIP runtime)
    from rt_amd import abi, render, scheme

    sch = scheme.load_json(os.path.join(ROOT, "tests", "golden", "scenes", a.scene + ".json"))
    ctxs = {}
    for n in a.names:
        # name[:VAR=VAL,...]: a library variant, with environment knobs read at its rt_create
        lname, _, envs = n.partition(":")
        saved = {}
        for kv in filter(None, envs.split(",")):
            k, v = kv.split("=", 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        path = (os.path.join(ROOT, "gpu-ray_trace-rust_amd", "lib", "librt_amd.so") if lname == "main" else
                os.path.join(ROOT, "gpu-ray_trace-rust_amd", "lib", "variants", f"librt_{lname}.so"))
        lib = abi.load_library(path)
        loaded = scheme.load(sch, assets_root=os.path.join(ROOT, "assets_pack"), lib=lib, width=a.width,
                             height=a.height)
        ctxs[n] = (render.Context(loaded, lib=lib), loaded)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    res = {n: [] for n in a.names}
    ref = prev = None
    for r in range(a.rounds + 1):
        for n, (ctx, loaded) in ctxs.items():
            w, h = int(loaded.info.width), int(loaded.info.height)
            t0 = time.perf_counter()
            img = ctx.render(None, 0, a.spp, want_output=(r == 0))
            dt = time.perf_counter() - t0
            if r == 0:
                if ref is None:
                    ref = img
                same = bool((img == ref).all())
                same_prev = bool((img == prev).all()) if prev is not None else True
                prev = img
                print(f"{n}: identical to {a.names[0]}: {same} (to the previous variant: {same_prev})", flush=True)
                continue
            res[n].append(w * h * a.spp / (ctx.last_kernel_ms() * 1e-3) / 1e6)
    for n, v in res.items():
        print(json.dumps({"variant": n, "Msamples_s_kernel": [round(x, 1) for x in v], "best": round(max(v), 1)}))


if __name__ == "__main__":
    main()
