"""Wave-clock breakdown of the general (mesh) queue kernel from a -DRT_TIMING=1 variant build
(tools/build_variants.sh tim="-DRT_TIMING=1").  Usage: python tools/timing_breakdown.py [scene] [spp]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "biplane"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import torch  # noqa: F401
    from rt_amd import abi, render, scheme

    path = os.path.join(ROOT, "gpu-ray_trace-rust_amd", "lib", "variants", "librt_tim.so")
    lib = abi.load_library(path)
    raw = C.CDLL(path)
    raw.rt_debug_timing.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    sch = scheme.load_json(os.path.join(ROOT, "tests", "golden", "scenes", scene + ".json"))
    loaded = scheme.load(sch, assets_root=os.path.join(ROOT, "assets_pack"), lib=lib)
    ctx = render.Context(loaded, lib=lib)
    buf = (C.c_ulonglong * 8)()
    ctx.render(None, 0, spp, want_output=False)  # warm
    raw.rt_debug_timing(buf, 1)
    ctx.render(None, spp, spp, want_output=False)
    raw.rt_debug_timing(buf, 1)
    t = list(buf)
    ms = ctx.last_kernel_ms()
    if loaded.desc.n_free_tris == 0 and loaded.desc.n_meshes == 0 and loaded.desc.n_spheres <= 64:
        out = {"scene": scene, "spp": spp, "kernel_ms": round(ms, 3), "kernel": "sphere-only",
               "frac_grab_start": round(t[0] / t[4], 3), "frac_closest": round(t[1] / t[4], 3),
               "frac_shade": round(t[2] / t[4], 3), "iterations": t[3],
               "cycles_per_iteration": round(t[4] / max(t[3], 1), 1)}
        print(json.dumps(out))
        return
    out = {"scene": scene, "spp": spp, "kernel_ms": round(ms, 3),
           "descent_pop_cycles": t[0], "pass_cycles": t[1], "rounds": t[2], "passes": t[3],
           "queue_cycles": t[4], "closest_calls": t[5]}
    if t[4]:
        out["frac_descent"] = round(t[0] / t[4], 3)
        out["frac_passes"] = round(t[1] / t[4], 3)
        out["frac_rest"] = round(1 - (t[0] + t[1]) / t[4], 3)
    if t[2]:
        out["passes_per_round"] = round(t[3] / t[2], 2)
        out["cycles_per_pass"] = round(t[1] / max(t[3], 1), 1)
        out["rounds_per_call"] = round(t[2] / max(t[5], 1), 2)
        out["descent_cycles_per_round"] = round(t[0] / t[2], 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
