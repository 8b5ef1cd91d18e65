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
