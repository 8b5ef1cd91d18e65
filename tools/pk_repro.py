"""Tiny triangle + light scene (tests/test_gpu_edges.py) against the oracle, per library variant.
Usage: python tools/pk_repro.py main sb0 ..."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("gpu-ray_trace-rust_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import torch  # noqa: F401
from test_gpu_edges import _scheme, TRI, LIGHT
import oracle_py
from rt_amd import abi, render, scheme
tiles = [(0, 0, 48, 32)]
for name in sys.argv[1:]:
    path = (os.path.join(ROOT, "gpu-ray_trace-rust_amd", "lib", "librt_amd.so") if name == "main" else
            os.path.join(ROOT, "gpu-ray_trace-rust_amd", "lib", "variants", f"librt_{name}.so"))
    lib = abi.load_library(path)
    sc = _scheme([TRI, LIGHT])
    o = oracle_py.render(sc, tiles, 0, 6, accum=oracle_py.ACCUM_FORWARD)
    for spp in (1, 6):
        o = oracle_py.render(sc, tiles, 0, spp, accum=oracle_py.ACCUM_FORWARD)
        with render.Context(sc, lib=lib) as c:
            g = c.render(tiles, 0, spp)
        d = np.abs(g - o).max(axis=1)
        idx = np.nonzero(d > 0)[0]
        print(name, "spp", spp, "bad", len(idx), [(int(i % 48), int(i // 48)) for i in idx[:6]],
              g[idx[0]] if len(idx) else "", o[idx[0]] if len(idx) else "", flush=True)
