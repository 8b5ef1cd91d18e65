"""Matches the device's walled/biplane renders against the reference's own CPU-path renders
(tests/golden/ref_cpu_images.npz): orientation, the spp whose pixel noise matches, and per-block
mean agreement across seeds.  Prints JSON lines.  Usage: python tools/ref_image_analysis.py scene"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def u8(rgba):  # draw_scene.rs:104-108: trunc(clamp(f, 0, 1) * 255 + 0.5)
    f = np.clip(rgba[..., :3], 0, 1) * np.float32(255) + np.float32(0.5)
    return np.trunc(np.nan_to_num(f)).astype(np.int32)


def noise(img):
    return float(np.abs(np.diff(img.astype(np.float64), axis=1)).mean())


def blocks(img, b=40):
    h, w, _ = img.shape
    return img[: h // b * b, : w // b * b].reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3))


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "walled"
    import torch  # noqa: F401
    from rt_amd import render
    from conftest import load_scene

    ref = np.load(os.path.join(ROOT, "tests", "golden", "ref_cpu_images.npz"))[scene].astype(np.int32)
    sc = load_scene(scene)
    w, h = int(sc.info.width), int(sc.info.height)
    print(json.dumps({"ref_noise": noise(ref), "ref_mean": float(ref.mean())}))
    spps = [2, 4, 6, 8, 10, 12, 16, 24] if scene == "walled" else [1, 2, 3, 4, 6, 8, 12, 16, 24]
    for spp in spps:
        imgs = []
        for seed in range(4):
            sc.info.seed = 0x5EED0000 + 97 * seed + spp
            with render.Context(sc) as ctx:
                img = ctx.render(None, 0, spp).reshape(h, w, 4)
            imgs.append(u8(img))
        a = np.stack(imgs)
        flip = a[:, ::-1]
        bm_ref = blocks(ref)
        res = {"spp": spp, "noise": float(np.mean([noise(x) for x in a])), "mean": float(a.mean())}
        for tag, arr in (("noflip", a), ("flip", flip)):
            bm = np.stack([blocks(x) for x in arr])
            mu, sd = bm.mean(0), bm.std(0, ddof=1) + 0.5
            z = np.abs(bm_ref - mu) / sd
            res[tag] = {"corr": float(np.corrcoef(bm_ref.ravel(), mu.ravel())[0, 1]),
                        "frac_z_lt_4": float((z < 4).mean()), "mean_abs_block_diff": float(np.abs(bm_ref - mu).mean())}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
