"""The whole path against the reference's OWN rendered output (a statistical anchor).

tests/golden/ref_cpu_images.npz holds the reference CPU renderer's walled.png and biplane.png
(info/images_cpu_comparison, README.md:177-194; tools/make_ref_image_fixtures.py): the same
scene and estimator, run for a few seconds with thread_rng.  Its RNG cannot be reproduced, so
the check is statistical.  The device renders the frame at the spp whose pixel noise matches
the reference image, with four seeds.  The reference's 40x40-pixel block means of the 8-bit
image (draw_scene.rs:104-108, rows flipped as ui_util.rs:37-54 writes them) must fall inside the
seeds' spread: within 4 sigma for >= 98% of the 450 blocks, a correlation above 0.999, and a
mean absolute block difference under 2 (walled) / 1 (biplane) 8-bit levels.  A wrong material,
light, camera or traversal rule moves whole regions of the image and fails this.
Measured: walled at 12 spp, 99.85% of blocks within 4 sigma and mean |diff| 1.04;
biplane at 6 spp, 100% and 0.53."""
import os

import numpy as np
import pytest

from conftest import ROOT, load_scene

pytestmark = pytest.mark.gpu


def _u8(rgba):  # draw_scene.rs:104-108
    f = np.clip(rgba[..., :3], 0, 1) * np.float32(255) + np.float32(0.5)
    return np.trunc(np.nan_to_num(f)).astype(np.int32)


def _blocks(img, b=40):
    h, w, _ = img.shape
    return img[: h // b * b, : w // b * b].reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3))


def _noise(img):
    return float(np.abs(np.diff(img.astype(np.float64), axis=1)).mean())


@pytest.mark.parametrize("scene,spp,max_mad", [("walled", 12, 2.0), ("biplane", 6, 1.0)])
def test_block_means_match_the_reference_render(gpu_available, scene, spp, max_mad):
    from rt_amd import render

    ref = np.load(os.path.join(ROOT, "tests", "golden", "ref_cpu_images.npz"))[scene].astype(np.int32)
    sc = load_scene(scene)
    w, h = int(sc.info.width), int(sc.info.height)
    imgs = []
    for seed in range(4):
        sc.info.seed = 0x5EED0000 + 97 * seed + spp
        with render.Context(sc) as ctx:
            imgs.append(_u8(ctx.render(None, 0, spp).reshape(h, w, 4))[::-1])  # PNG rows flipped
    bm = np.stack([_blocks(x) for x in imgs])
    mu, sd = bm.mean(0), bm.std(0, ddof=1) + 0.5
    bref = _blocks(ref)
    z = np.abs(bref - mu) / sd
    corr = float(np.corrcoef(bref.ravel(), mu.ravel())[0, 1])
    mad = float(np.abs(bref - mu).mean())
    noise = float(np.mean([_noise(x) for x in imgs]))
    print(scene, {"corr": corr, "frac_z_lt_4": float((z < 4).mean()), "mad": mad,
                  "noise": noise, "ref_noise": _noise(ref)})
    assert corr > 0.999
    assert (z < 4).mean() >= 0.98
    assert mad < max_mad
    assert abs(noise - _noise(ref)) < 0.1 * _noise(ref)  # the reference's spp is about this one


@pytest.mark.parametrize("change", ["light_plus_10pct", "glass_as_mirror"])
def test_block_check_rejects_a_perturbed_walled(gpu_available, change):
    """Negative control: the same check on a walled.yml with a 10% brighter ceiling light, or with
    the glass spheres turned into mirrors, must fail — the test has the power to see such changes."""
    from rt_amd import render

    ref = np.load(os.path.join(ROOT, "tests", "golden", "ref_cpu_images.npz"))["walled"].astype(np.int32)
    spp = 12
    imgs = []
    for seed in range(4):
        sc = load_scene("walled")
        for i in range(sc.desc.n_spheres):
            s = sc.desc.spheres[i]
            if change == "light_plus_10pct" and s.mat.has_emissive and s.r > 4.0:
                for k in range(3):
                    s.mat.emissive[k] *= 1.1
            if change == "glass_as_mirror" and s.mat.n_in > 1.0:
                s.mat.divert = 0  # RT_DIVERT_SPEC
        sc.info.seed = 0x5EED0000 + 97 * seed + spp
        w, h = int(sc.info.width), int(sc.info.height)
        with render.Context(sc) as ctx:
            imgs.append(_u8(ctx.render(None, 0, spp).reshape(h, w, 4))[::-1])
    bm = np.stack([_blocks(x) for x in imgs])
    mu, sd = bm.mean(0), bm.std(0, ddof=1) + 0.5
    z = np.abs(_blocks(ref) - mu) / sd
    print(change, float((z < 4).mean()), float(np.abs(_blocks(ref) - mu).mean()))
    assert (z < 4).mean() < 0.98
