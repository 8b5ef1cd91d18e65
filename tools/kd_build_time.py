"""rt_kd_build wall time per scene for library variants (host C++ KD build; best of 5).
Usage: python tools/kd_build_time.py main kdold ..."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_scene  # noqa: E402
from rt_amd import abi  # noqa: E402

scenes = {n: load_scene(n) for n in ("walled", "biplane", "spaceship_r1", "a380")}
for name in sys.argv[1:]:
    lib = abi.load_library(os.path.join(ROOT, "gpu-ray_trace-rust_amd", "lib",
                                        "librt_amd.so" if name == "main" else f"variants/librt_{name}.so"))
    row = []
    for sn, sc in scenes.items():
        best = 1e9
        for _ in range(5):
            ptr = C.POINTER(abi.rt_kd_tree)()
            t0 = time.perf_counter()
            abi.check(lib, lib.rt_kd_build(C.byref(sc.desc), int(sc.info.kd_tree_depth), C.byref(ptr)))
            best = min(best, time.perf_counter() - t0)
            lib.rt_kd_free(ptr)
        row.append(f"{sn} {best * 1e3:.1f} ms")
    print(name, "|", ", ".join(row), flush=True)
