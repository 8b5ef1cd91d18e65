"""Vector-memory load instructions of the general queue kernel by class, per sample (the
RT_VMEM_COUNT diagnostic build: make -C gpu-ray_trace-rust_amd diag -> lib/variants/librt_diag_vmem.so).
Renders one full-frame launch of each scene in a child process (the kernel's printf goes to the
child's stdout) and prints one JSON line per scene: wave-level load instructions per sample by
class, next to SQ_INSTS_VMEM_RD per sample from the committed counters of the product build.
Usage (on the GPU box): python tools/vmem_classes.py [scene[@N]:spp ...] > profiles/<tag>_vmem_lines.jsonl
(@N: an N x N frame; each line carries the product build id of the same source, which bench.py's
mesh roofline requires to match)"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["descent", "pop", "pass_ref", "pass_tri", "lead_sph", "retest", "pixq", "mesh_rec", "tex", "sph_shade",
         "pk_leaves", "passes", "rounds", "rad_stores", "starts"]
LOADS = ["descent", "pop", "pass_ref", "pass_tri", "lead_sph", "retest", "pixq", "mesh_rec", "tex", "sph_shade"]
# RT_VL classes (diag.h VL): lines / sectors / asked bytes of the load sites by class
VL_NAMES = ["descent", "pop", "pass_ref", "pass_tri", "lead_sph", "retest", "pixq", "mesh_rec", "tex"]

CHILD = r"""
import os, sys
sys.path.insert(0, os.path.join(%(root)r, "gpu-ray_trace-rust_amd"))
import torch  # noqa: F401
from rt_amd import abi, render, scheme
lib = abi.load_library(os.path.join(%(root)r, "gpu-ray_trace-rust_amd", "lib", "variants", "librt_diag_vmem.so"))
sch = scheme.load_json(os.path.join(%(root)r, "tests", "golden", "scenes", %(scene)r + ".json"))
loaded = scheme.load(sch, assets_root=os.path.join(%(root)r, "assets_pack"), lib=lib, width=%(width)s, height=%(width)s)
with render.Context(loaded, lib=lib) as c:
    c.render(None, 0, %(spp)d, want_output=False)
    c.render(None, %(spp)d, %(spp)d, want_output=False)
print("PIXELS", int(loaded.info.width) * int(loaded.info.height), flush=True)
"""


def main(specs):
    sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
    from rt_amd import abi

    build_id = abi.kernel_build_id()  # the product library built from the same source
    for spec in specs:
        # scene[@N]:spp — @N renders at N x N (spaceship_r1@4096: BASELINE config 5's frame)
        config, _, spp = spec.partition(":")
        scene, _, size = config.partition("@")
        spp = int(spp or 10)
        code = CHILD % {"root": ROOT, "scene": scene, "spp": spp, "width": int(size) if size else None}
        # serialized launches: the counters are per launch (overlapped launches would mix them)
        env = dict(os.environ, RT_DEBUG_LAUNCH="overlap=0")
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600, env=env)
        # one "RT_VC <class> <count>" line per class and launch; the second launch's (the last 24)
        vc = [l.split() for l in r.stdout.splitlines() if l.startswith("RT_VC ")]
        pix = int(re.search(r"PIXELS (\d+)", r.stdout).group(1))
        if len(vc) < 48:
            print(json.dumps({"scene": scene, "error": r.stderr[-2000:]}))
            continue
        last = {int(c): int(v) for _, c, v in vc[-24:]}
        vl = [l.split() for l in r.stdout.splitlines() if l.startswith("RT_VL ")]
        vl_last = {int(x[1]): [int(v) for v in x[2:6]] for x in vl[-16:]} if len(vl) >= 32 else {}
        d = {k: last[i] for i, k in enumerate(NAMES)}
        gn = ["pairs", "pairs_g2", "pairs_g3", "pairs_g4", "pairs_g8", "quads", "groups"]
        g = {k: last[15 + i] for i, k in enumerate(gn)}
        samples = pix * spp  # the second launch (the first warms up; each launch prints its own)
        per = {k: round(d[k] / samples, 3) for k in NAMES}
        out = {"scene": scene, "config": config, "build_id": build_id,
               "spp_per_launch": spp, "samples": samples, "per_sample": per,
               "vmem_loads_per_sample": round(sum(d[k] for k in LOADS) / samples, 2)}
        if g.get("pairs"):
            # cooperative pairs by the number of the wave's lanes at the same leaf in that round
            out["leaf_sharing"] = {"pairs_per_sample": round(g["pairs"] / samples, 2),
                                   "frac_pairs_in_groups_ge2": round(g["pairs_g2"] / g["pairs"], 4),
                                   "frac_ge3": round(g["pairs_g3"] / g["pairs"], 4),
                                   "frac_ge4": round(g["pairs_g4"] / g["pairs"], 4),
                                   "frac_ge8": round(g["pairs_g8"] / g["pairs"], 4),
                                   "quad_slots_per_pair": round(4 * g["quads"] / g["pairs"], 4),
                                   "pairs_per_group": round(g["pairs"] / g["groups"], 2)}
        if vl_last:
            # per class and sample: lanes served, distinct 128-B lines and 64-B sectors the wave
            # loads touch (the requests a load can send past L1), the bytes the distinct lane
            # addresses ask for, and lines x 128 B over those bytes (what a 128-B fetch of every
            # touched line would over-fetch)
            cls = {}
            for i, k in enumerate(VL_NAMES):
                lanes, lines, secs, asked = vl_last.get(i, [0, 0, 0, 0])
                if not lanes:
                    continue
                cls[k] = {"lanes": round(lanes / samples, 3), "lines_128": round(lines / samples, 3),
                          "sectors_64": round(secs / samples, 3), "asked_B": round(asked / samples, 1),
                          "line_B_over_asked": round(128 * lines / asked, 3) if asked else None}
            tl = sum(v["lines_128"] for v in cls.values())
            ta = sum(v["asked_B"] for v in cls.values())
            out["lines_by_class"] = cls
            out["lines_total"] = {"lines_128_per_sample": round(tl, 2), "sectors_64_per_sample":
                                  round(sum(v["sectors_64"] for v in cls.values()), 2),
                                  "asked_B_per_sample": round(ta, 1), "line_B_per_sample": round(128 * tl, 1)}
        for p in sorted(os.listdir(os.path.join(ROOT, "profiles"))):
            if p.endswith("_counters.json"):
                c = json.load(open(os.path.join(ROOT, "profiles", p)))
                if c.get("scene") == scene and c.get("vmem_rd_per_launch"):
                    out["product_sq_insts_vmem_rd_per_sample"] = (
                        round(c["vmem_rd_per_launch"] / c["samples_per_launch"], 2), p)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["biplane:10", "spaceship_r1:10", "a380:4"])
