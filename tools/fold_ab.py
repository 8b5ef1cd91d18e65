"""A/B of the fold kernel across variant libraries (tools/build_variants.sh): fold time per render
call = render_ms - trace_ms (launch_stats), walled 1000 spp, interleaved rounds.
Usage: python tools/fold_ab.py name1 name2 ..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))


def main():
    import torch  # noqa: F401
    from rt_amd import abi, render, scheme

    sch = scheme.load_json(os.path.join(ROOT, "tests", "golden", "scenes", "walled.json"))
    ctxs = {}
    for n in sys.argv[1:]:
        lib = abi.load_library(os.path.join(ROOT, "gpu-ray_trace-rust_amd", "lib", "variants", f"librt_{n}.so"))
        ctxs[n] = render.Context(scheme.load(sch, lib=lib), lib=lib)
    res = {n: [] for n in ctxs}
    for r in range(4):
        for n, c in ctxs.items():
            c.render(None, 0, 1000, want_output=False)
            st = c.launch_stats()
            if r:
                res[n].append(round(st["render_ms"] - st["trace_ms"], 3))
    for n, v in res.items():
        print(json.dumps({"variant": n, "fold_ms": v, "best": min(v)}))


if __name__ == "__main__":
    main()
