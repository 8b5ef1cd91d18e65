"""Device path vs the CPU oracle on the other benchmark scenes: triangles.yml (free triangles,
thin lens, cube map), a380.yml (synthetic stand-in geometry), biplane.yml and spaceship_r1.yml (glTF meshes: normal maps, base colour
and metallic-roughness textures, tangents, Schlick/roughness sampling, cube-map sky)."""
import numpy as np
import pytest

import parity
from conftest import load_scene

pytestmark = pytest.mark.gpu

CROPS = {
    "triangles": [(560, 260, 64, 32), (600, 500, 32, 32), (100, 100, 32, 16)],
    "biplane": [(600, 400, 32, 32), (450, 300, 32, 32), (600, 300, 32, 16)],
    "spaceship_r1": [(450, 200, 32, 32), (600, 300, 32, 32), (750, 400, 32, 16)],
    "a380": [(350, 400, 32, 32), (450, 275, 32, 32), (750, 425, 32, 16)],
}
SPP = {"triangles": 16, "biplane": 8, "spaceship_r1": 8, "a380": 4}


@pytest.fixture(scope="module", params=sorted(CROPS))
def scene(request, gpu_available):
    return request.param, load_scene(request.param)


def test_scene_parity(scene, oracle):
    from rt_amd import render

    name, sc = scene
    crops, spp = CROPS[name], SPP[name]
    with render.Context(sc) as ctx:
        g = ctx.render(crops, 0, spp)
        counts = ctx.count_work(crops, 0, spp)
    o, oc = oracle.render(sc, crops, 0, spp, accum=oracle.ACCUM_FORWARD, counts=True)
    s = parity.stats(g, o)
    print(name, s, "\n gpu", counts, "\n oracle", oc)
    if name != "triangles":
        assert oc["mesh_hits"] > 0 and counts["mesh_hits"] > 0
    assert np.array_equal(g, o), s  # bit-identical to the forward oracle
    for k in ("samples", "segments", "nodes", "leaf_refs", "tri_tests", "sphere_tests", "mesh_hits"):
        assert counts[k] == oc[k], (k, counts[k], oc[k])


def test_scene_recursive_parity(scene, oracle):
    from rt_amd import render

    name, sc = scene
    crops, spp = CROPS[name][:1], SPP[name]
    with render.Context(sc) as ctx:
        g = ctx.render(crops, 0, spp)
    o = oracle.render(sc, crops, 0, spp, accum=oracle.ACCUM_RECURSIVE)
    s = parity.stats(g, o)
    print(name, "recursive", s)
    assert s["frac_ok"] >= parity.MIN_FRAC, s
    assert parity.frac_u8_within(g, o) >= parity.MIN_FRAC, s
    assert s["mean_rel_err"] < 1e-3


def test_debug_single_ray_scene(scene, oracle):
    """First hit only: camera (incl. the lens), traversal, cube-map lookup; no bounce."""
    from rt_amd import render

    name, _ = scene
    sc = load_scene(name)
    sc.info.debug_single_ray = 1
    crops = CROPS[name][:2]
    with render.Context(sc) as ctx:
        g = ctx.render(crops, 0, 2)
    o = oracle.render(sc, crops, 0, 2)
    s = parity.stats(g, o)
    assert s["frac_exact"] == 1.0, s  # the lens's sin/cos are glibc's (rt_libm.h)


@pytest.mark.parametrize("name", ["triangles", "biplane", "spaceship_r1"])
def test_texel_pool_u8_equals_f32(gpu_available, monkeypatch, name):
    """The 8-bit texel pool (every channel some k / 255: one RGBA8 word per texel, decoded on the
    device) renders the f32 pool's image bit for bit (RT_DEBUG_TEXELS_F32=1 forces the f32 pool)."""
    from rt_amd import render

    sc = load_scene(name, width=320, height=160)
    with render.Context(sc) as c:
        g8 = c.render(None, 0, 3)
    monkeypatch.setenv("RT_DEBUG_TEXELS_F32", "1")
    with render.Context(sc) as c:
        g32 = c.render(None, 0, 3)
    assert np.array_equal(g8, g32), parity.stats(g8, g32)


def test_texture_off_the_u8_grid_keeps_f32(gpu_available, oracle):
    """A texel that is not k / 255 (here 0.123) cannot go to the 8-bit pool: the context keeps the
    f32 pool and still renders the oracle's image."""
    import ctypes as C

    from rt_amd import render

    sc = load_scene("triangles", width=320, height=160)
    for i in range(sc.desc.n_textures):
        t = sc.desc.textures[i]
        px = C.cast(t.rgb, C.POINTER(C.c_float))
        for k in range(0, 3 * t.width * t.height, 997):
            px[k] = 0.123
    tiles = [(0, 0, 320, 160)]
    with render.Context(sc) as c:
        g = c.render(tiles, 0, 2)
    o = oracle.render(sc, tiles, 0, 2, accum=oracle.ACCUM_FORWARD)
    assert np.array_equal(g, o), parity.stats(g, o)
