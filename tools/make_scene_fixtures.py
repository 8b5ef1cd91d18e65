"""Regenerates tests/golden/scenes/*.json from the reference's scheme YAML files.

The GPU box has no /root/reference, so the benchmark schemes travel as the parsed scheme
(JSON of the serde data model, tagged values as {"!Tag": value}).  Run in this container:
    python tools/make_scene_fixtures.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
from rt_amd import scheme  # noqa: E402

REF = "/root/reference/schemes"
NAMES = ["walled", "triangles", "biplane", "spaceship_r1", "a380", "outside_spheres", "bounce_anim", "biplane_anim"]

if __name__ == "__main__":
    out_dir = os.path.join(ROOT, "tests", "golden", "scenes")
    os.makedirs(out_dir, exist_ok=True)
    for n in NAMES:
        src = os.path.join(REF, n + ".yml")
        if not os.path.exists(src):
            print("skip", n)
            continue
        sch = scheme.from_yml(open(src).read())
        scheme.dump_json(sch, os.path.join(out_dir, n + ".json"))
        print("wrote", n)
