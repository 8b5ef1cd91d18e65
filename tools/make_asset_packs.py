"""Packs the assets the benchmark scenes need into assets_pack/<dir>.npz.

The GPU box receives only this repository.  Each pack holds, for one directory of the
reference's assets/: every glTF document's JSON ("gltf:<name>") and binary buffers
("buf:<name>:<i>"), every PNG and JPEG decoded to 8-bit channels ("img:<relpath>", by
rt_amd.assets.decode_image — the decode the file store uses).  Run in this container:
    python tools/make_asset_packs.py [dirs...]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
from rt_amd.assets import decode_image  # noqa: E402

SRC = "/root/reference/assets"
DIRS = ["airplane_biplane", "spaceship_shuttle_r1", "skybox", "cubemap_images", "a380"]
IMG_EXT = (".png", ".jpg", ".jpeg")


def pack(d):
    base = os.path.join(SRC, d)
    out = {}
    for dirpath, _, files in os.walk(base):
        for f in sorted(files):
            full = os.path.join(dirpath, f)
            rel = os.path.relpath(full, base).replace(os.sep, "/")
            if f.endswith(".gltf"):
                doc = json.load(open(full))
                out["gltf:" + rel] = np.frombuffer(open(full, "rb").read(), dtype=np.uint8)
                for i, b in enumerate(doc.get("buffers", [])):
                    bp = os.path.join(os.path.dirname(full), b["uri"])
                    if os.path.exists(bp):
                        out[f"buf:{rel}:{i}"] = np.frombuffer(open(bp, "rb").read(), dtype=np.uint8)
            elif f.lower().endswith(IMG_EXT):
                # PNG and JPEG alike are stored decoded (one decoder, PIL, for both hosts: the
                # C++ host has no JPEG decoder)
                out["img:" + rel] = decode_image(open(full, "rb").read())
    os.makedirs(os.path.join(ROOT, "assets_pack"), exist_ok=True)
    dst = os.path.join(ROOT, "assets_pack", d + ".npz")
    np.savez_compressed(dst, **out)
    print(d, len(out), "entries", os.path.getsize(dst) // 1024, "KiB")


if __name__ == "__main__":
    for d in sys.argv[1:] or DIRS:
        pack(d)
