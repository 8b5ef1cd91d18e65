"""Parity at the production launch shapes: the device renders whole frames exactly as bench.py
and the scheme configs launch them (full-frame queue launches, the configs' resolutions, sample
offsets and batch sizes), and scattered pixels of the result are compared bit for bit with the
forward oracle run on just those pixels.  Reference loop: render_to_target_cpu
(src/render/draw_scene.rs:71-98)."""
import numpy as np
import pytest

import parity
from conftest import load_scene

pytestmark = pytest.mark.gpu


def scattered(w, h, n, seed, extra=()):
    """n distinct pixels of a w x h frame (seeded), plus the corners and the centre."""
    rng = np.random.default_rng(seed)
    pts = {(0, 0), (w - 1, 0), (0, h - 1), (w - 1, h - 1), (w // 2, h // 2)} | set(extra)
    while len(pts) < n:
        pts.add((int(rng.integers(0, w)), int(rng.integers(0, h))))
    return sorted(pts, key=lambda p: (p[1], p[0]))


def pick(frame, w, pts):
    return np.stack([frame[y * w + x] for (x, y) in pts])


def test_walled_config4_whole_run(gpu_available, oracle):
    """BASELINE config 4 as the bench runs it: walled.yml's whole 20000-spp run in its 1000-spp
    full-frame queue launches (one launch per call, 720 M items each, the running mean carried on
    the device from sample 0), then 256 scattered pixels against the oracle run over the same
    [0, 20000): bit-exact against the forward oracle, and the stated gate against the reference's
    own recursive order (radiance.rs:44,59)."""
    from rt_amd import render

    sc = load_scene("walled")
    w, h = int(sc.info.width), int(sc.info.height)
    pts = scattered(w, h, 256, seed=19)
    with render.Context(sc) as ctx:
        for s0 in range(0, 20000, 1000):
            frame = ctx.render(None, s0, 1000, want_output=(s0 == 19000))
            assert ctx.launch_stats()["n_trace_launches"] == 1  # one queue launch, as in the bench
    g = pick(frame, w, pts)
    tiles = [(x, y, 1, 1) for (x, y) in pts]
    o = oracle.render(sc, tiles, 0, 20000, accum=oracle.ACCUM_FORWARD)
    s = parity.stats(g, o)
    print("walled [0, 20000) forward", s)
    assert np.array_equal(g, o), s
    r = oracle.render(sc, tiles, 0, 20000, accum=oracle.ACCUM_RECURSIVE)
    parity.assert_reference_order(g, r, "walled [0, 20000)")


def test_spaceship_4096_config5(gpu_available, oracle):
    """spaceship_r1.yml at 4096 x 4096 (BASELINE config 5): the full frame at 4 spp in the
    scheme's batches of 25 -> here one call, 64 scattered pixels plus two 32 x 32 tiles."""
    from rt_amd import render

    sc = load_scene("spaceship_r1", width=4096, height=4096)
    w, h = 4096, 4096
    pts = scattered(w, h, 64, seed=5)
    blocks = [(2040, 2040, 32, 32), (1500, 2600, 32, 32)]
    with render.Context(sc) as ctx:
        frame = ctx.render(None, 0, 4)
    g = pick(frame, w, pts)
    o = oracle.render(sc, [(x, y, 1, 1) for (x, y) in pts], 0, 4, accum=oracle.ACCUM_FORWARD)
    s = parity.stats(g, o)
    print("spaceship 4096^2 scattered", s)
    assert np.array_equal(g, o), s
    img = frame.reshape(h, w, 4)
    gb = np.concatenate([img[y:y + bh, x:x + bw].reshape(-1, 4) for (x, y, bw, bh) in blocks])
    ob = oracle.render(sc, blocks, 0, 4, accum=oracle.ACCUM_FORWARD)
    sb = parity.stats(gb, ob)
    print("spaceship 4096^2 blocks", sb)
    assert np.array_equal(gb, ob), sb
    assert (img[..., 3] == 1.0).all()


def test_biplane_200spp_scheme_batches(gpu_available, oracle):
    """biplane.yml at BASELINE config 3's 200 spp, in the scheme's gpu_render_batch of 10
    (20 full-frame launches, the running mean carried across them)."""
    from rt_amd import render

    sc = load_scene("biplane")
    w, h = int(sc.info.width), int(sc.info.height)
    pts = scattered(w, h, 128, seed=3, extra=((600, 300), (610, 310)))
    with render.Context(sc) as ctx:
        for s0 in range(0, 200, 10):
            frame = ctx.render(None, s0, 10, want_output=(s0 == 190))
    g = pick(frame, w, pts)
    tiles = [(x, y, 1, 1) for (x, y) in pts]
    o = oracle.render(sc, tiles, 0, 200, accum=oracle.ACCUM_FORWARD)
    s = parity.stats(g, o)
    print("biplane 200 spp", s)
    assert np.array_equal(g, o), s
    r = oracle.render(sc, tiles, 0, 200, accum=oracle.ACCUM_RECURSIVE)
    parity.assert_reference_order(g, r, "biplane 200 spp")


def test_a380_batch1(gpu_available, oracle):
    """a380.yml (synthetic stand-in geometry) at its own gpu_render_batch of 1: ten one-sample
    full-frame launches."""
    from rt_amd import render

    sc = load_scene("a380")
    w, h = int(sc.info.width), int(sc.info.height)
    pts = scattered(w, h, 96, seed=38)
    with render.Context(sc) as ctx:
        for s0 in range(10):
            frame = ctx.render(None, s0, 1, want_output=(s0 == 9))
    g = pick(frame, w, pts)
    tiles = [(x, y, 1, 1) for (x, y) in pts]
    o = oracle.render(sc, tiles, 0, 10, accum=oracle.ACCUM_FORWARD)
    s = parity.stats(g, o)
    print("a380 batch 1", s)
    assert np.array_equal(g, o), s
    r = oracle.render(sc, tiles, 0, 10, accum=oracle.ACCUM_RECURSIVE)
    parity.assert_reference_order(g, r, "a380 batch 1")


# Whole frames, every pixel: the oracle's cost per sample (CPU column) makes a full
# 1200 x 600 frame at 1-10 spp a few seconds of host work, so each benchmark scene is compared on
# its entire frame, in the scheme's own batch size where that is smaller than the sample count.
# A range that starts past sample 0 continues a context that has rendered [0, s0) itself; the
# oracle continues from that context's frame (its `init`), so both run the same samples from the
# same state.
WHOLE = [
    # scene, sample_begin, samples, batch, dir_light_samp
    ("triangles", 0, 10, 10, 0),       # BASELINE config 0: 10 spp, depth 5
    ("walled", 19000, 2, 2, 0),        # the bench's scene, late in its 20000-spp run
    ("walled", 7, 1, 1, 1),            # direct-light sampling (radiance.rs:46-56,89-120)
    ("biplane", 190, 2, 1, 0),         # config 3's tail, one-sample batches (pipelined launches)
    ("spaceship_r1", 25, 1, 1, 0),
    ("a380", 3, 2, 1, 0),              # config 2's batch of 1
    ("outside_spheres", 0, 2, 1, 0),   # schemes/outside_spheres.yml as a still (lens, cube map, kd depth 1)
    ("spaceship_r1@4096", 0, 1, 1, 0),  # config 5's 4096 x 4096 frame (16.8 M pixels)
]


def _prefix_batch(name, s0):
    """The batch the context renders [0, s0) in: the scheme's own gpu_render_batch where it
    divides s0, else one call."""
    b = {"walled": 1000, "biplane": 10, "spaceship_r1": 25, "a380": 1}.get(name, s0)
    return b if s0 % b == 0 else s0


@pytest.mark.parametrize("name,s0,spp,batch,dls", WHOLE, ids=[f"{w[0]}-dls{w[4]}" for w in WHOLE])
def test_whole_frame_bit_exact(gpu_available, oracle, name, s0, spp, batch, dls):
    """Every pixel bit-exact against the forward oracle, and within the stated gate against the
    reference's recursive order (radiance.rs:44,59)."""
    from rt_amd import render

    scene, _, size = name.partition("@")
    sc = load_scene(scene, **({"width": int(size), "height": int(size)} if size else {}))
    sc.info.dir_light_samp = dls
    w, h = int(sc.info.width), int(sc.info.height)
    init = None
    with render.Context(sc) as ctx:
        if s0:  # [0, s0) on the device first: the range below continues an accumulated context
            pb = _prefix_batch(scene, s0)
            assert s0 % pb == 0
            for b in range(0, s0, pb):
                init = ctx.render(None, b, pb, want_output=(b + pb == s0))
        for b in range(s0, s0 + spp, batch):
            frame = ctx.render(None, b, batch, want_output=(b + batch == s0 + spp))
    full = [(0, 0, w, h)]
    o = oracle.render(sc, full, s0, spp, accum=oracle.ACCUM_FORWARD, init=init)
    s = parity.stats(frame, o)
    print(f"{name} whole frame {w}x{h}, samples [{s0}, {s0 + spp}), dls {dls}", s)
    assert (frame[:, 3] == 1.0).all()
    assert np.array_equal(frame, o), s
    del o
    r = oracle.render(sc, full, s0, spp, accum=oracle.ACCUM_RECURSIVE, init=init)
    parity.assert_reference_order(frame, r, f"{name} [{s0}, {s0 + spp})")
