"""The general kernel's cooperative leaf tests (trace.hip coop_leaf: 64 (ray, ref) pairs per pass,
the first strict minimum by an LDS atomicMin on (length, position)) and both traversals against
the oracle, on triangle sets built to make the closest-hit decision hard
(closest_hit.rs:6-30 over triangle/generic.rs:102-137, kdtree.rs:66-104):
- fans sharing a vertex and strips sharing edges (rays through a shared edge hit both triangles
  at the same length: the first in leaf order must win);
- exact duplicates and coplanar overlapping triangles (ties over a whole area);
- slivers, a zero-area triangle (never hit: det = 0) and walls spanning the scene (in many leaves);
- light spheres among them and an emissive sphere around all of it, so full paths bounce
  between the triangles (diffuse, DiffSpec, mirror and dielectric materials) and every pixel's
  value carries every hit of its paths.
Whole paths, forward accumulation (the device's order), half of the scenes through a
thin-lens camera: bit-exact, for the stack and the stackless traversal and with camera-ray packets
off."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _tri(v, mat, rgb):
    v = np.asarray(v, np.float64)
    n = np.cross(v[1] - v[0], v[2] - v[0])
    nn = np.linalg.norm(n)
    n = n / nn if nn > 0 else np.array([0.0, 0.0, 1.0])
    return {"!FreeTriangle": {"verts": [[float(x) for x in p] for p in np.float32(v)],
                              "norm": [float(x) for x in n], "rgb": [float(x) for x in rgb], "mat": mat}}


def _adversarial_triangles(seed: int) -> dict:
    rng = np.random.default_rng(1000 + seed)
    mats = [{"divert_ray": "Diff"}, {"divert_ray": {"!DiffSpec": {"diffp": 0.3}}}, {"divert_ray": "Spec"},
            {"divert_ray": {"!Dielectric": {"n_out": 1.0, "n_in": 1.5}}}]
    members = []

    def add(v):
        members.append(_tri(v, mats[int(rng.integers(0, 4))], rng.uniform(0.3, 0.95, 3)))

    # two walls (floor and back): two triangles each, sharing their diagonal
    for ax in (1, 2):
        for side in (-8.0,):
            q = np.zeros((4, 3))
            o1, o2 = (ax + 1) % 3, (ax + 2) % 3
            for k, (s1, s2) in enumerate(((-8, -8), (8, -8), (8, 8), (-8, 8))):
                q[k, ax], q[k, o1], q[k, o2] = side, s1, s2
            add([q[0], q[1], q[2]])
            add([q[0], q[2], q[3]])
    while len(members) < 60:
        kind = int(rng.integers(0, 5))
        c = rng.uniform(-5.0, 5.0, 3)
        if kind == 0:  # fan around a shared vertex
            r = rng.uniform(0.5, 2.5)
            u, w = rng.normal(size=3), rng.normal(size=3)
            a0 = rng.uniform(0, 2 * np.pi)
            pts = [c + r * (np.cos(a0 + t) * u + np.sin(a0 + t) * w) for t in np.linspace(0, 2 * np.pi, 6)]
            for k in range(5):
                add([c, pts[k], pts[k + 1]])
        elif kind == 1:  # exact duplicate of an earlier triangle (a different material)
            prev = members[int(rng.integers(0, len(members)))]["!FreeTriangle"]["verts"]
            add(prev)
        elif kind == 2:  # coplanar overlapping pair
            a, b = rng.normal(size=3), rng.normal(size=3)
            v = [c, c + 2 * a, c + 2 * b]
            add(v)
            add([c + 0.5 * a, c + 2.5 * a, c + 0.5 * a + 2 * b])
        elif kind == 3:  # sliver, and a zero-area triangle on its edge
            a = rng.normal(size=3)
            add([c, c + 3 * a, c + 3 * a + 1e-3 * rng.normal(size=3)])
            add([c, c + 1.5 * a, c + 3 * a])
        else:  # a strip sharing edges
            a, b = rng.normal(size=3), rng.normal(size=3)
            for k in range(3):
                add([c + k * a, c + (k + 1) * a, c + k * a + b])
    members = members[:60]
    for k in range(2):  # lights among the triangles
        members.insert(int(rng.integers(0, len(members))),
                       {"!Sphere": {"c": [float(x) for x in rng.uniform(-5, 5, 3)], "r": float(rng.uniform(0.5, 1.5)),
                                    "coloring": {"!Solid": [0.0, 0.0, 0.0]},
                                    "mat": {"divert_ray": "Diff", "emissive": [4.0, 3.0 + k, 2.0]}}})
    # an emissive sky sphere around everything: every escaping path carries the throughput of
    # every triangle it met, so a wrong hit anywhere on the path shows in the pixel
    members.append({"!Sphere": {"c": [0.0, 0.0, 0.0], "r": 60.0, "coloring": {"!Solid": [0.0, 0.0, 0.0]},
                                "mat": {"divert_ray": "Diff", "emissive": [0.7, 0.8, 1.0]}}})
    o = rng.uniform(-4.0, 4.0, 3) if seed % 2 == 0 else np.array([0.0, 0.0, 7.5])
    d = rng.normal(size=3) if seed % 2 == 0 else np.array([0.0, 0.0, -1.0])
    d = 5.0 * d / np.linalg.norm(d)
    cam = {"d": [float(x) for x in d], "o": [float(x) for x in o], "screen_height": 5.0,
           "screen_width": 8.0, "up": [0, 1, 0], "view_eulers": [0, 0, 0]}
    if seed >= 4:
        cam["lens_r"] = 0.05  # a thin lens: camera rays from different origins (generate.rs:39-66)
    return {"cam": cam,
            "render_info": {"gpu_render_batch": 1, "height": 96, "width": 160, "kd_tree_depth": 17,
                            "rad_info": {"debug_single_ray": False, "dir_light_samp": False,
                                         "russ_roull_info": {"assured_depth": 3, "max_thres": 0.5}},
                            "samps_per_pix": 4, "use_gpu": True},
            "scene_members": members}


@pytest.mark.parametrize("seed", range(8))
def test_adversarial_triangles_bit_exact(gpu_available, oracle, monkeypatch, seed):
    import parity
    from rt_amd import render, scheme

    sc = scheme.load(_adversarial_triangles(seed))
    assert sc.desc.n_free_tris >= 55
    tiles = [(0, 0, 160, 96)]
    o = oracle.render(sc, tiles, 0, 4, accum=oracle.ACCUM_FORWARD)
    assert np.isfinite(o).all() and o[:, :3].max() > 0  # the lights are seen
    for env in ({}, {"RT_DEBUG_KD_RESTART": "1"}, {"RT_DEBUG_PACKET": "0"}):
        for k in ("RT_DEBUG_KD_RESTART", "RT_DEBUG_PACKET"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with render.Context(sc) as c:
            g = c.render(tiles, 0, 4)
        assert np.array_equal(g, o), (env, parity.stats(g, o))


def _axis_aligned_triangles(seed: int) -> dict:
    """Unit cubes on an integer grid, each face two triangles: every triangle lies in an
    axis-aligned plane through integer coordinates, neighbouring cubes share faces (exact
    duplicates, opposite normals) and edges, and the camera looks down an axis, so primary rays
    have zero direction components (the reference's EPS clamp, kdtree.rs:75) and hit edges,
    corners and split planes exactly."""
    rng = np.random.default_rng(2000 + seed)
    mats = [{"divert_ray": "Diff"}, {"divert_ray": "Spec"}, {"divert_ray": {"!DiffSpec": {"diffp": 0.5}}}]
    members = []
    cells = {tuple(int(x) for x in rng.integers(-3, 3, 3)) for _ in range(9)}
    for (x, y, z) in sorted(cells):
        m = mats[int(rng.integers(0, 3))]
        rgb = rng.uniform(0.3, 0.95, 3)
        for ax in range(3):
            for side in (0, 1):
                o1, o2 = (ax + 1) % 3, (ax + 2) % 3
                q = np.zeros((4, 3))
                for k, (s1, s2) in enumerate(((0, 0), (1, 0), (1, 1), (0, 1))):
                    q[k, ax], q[k, o1], q[k, o2] = side, s1, s2
                q += np.array([x, y, z], np.float64)
                members.append(_tri([q[0], q[1], q[2]], m, rgb))
                members.append(_tri([q[0], q[2], q[3]], m, rgb))
    members.append({"!Sphere": {"c": [0.0, 0.0, 0.0], "r": 40.0, "coloring": {"!Solid": [0.0, 0.0, 0.0]},
                                "mat": {"divert_ray": "Diff", "emissive": [0.9, 0.8, 0.7]}}})
    ax = seed % 3
    o = [0.0, 0.0, 0.0]
    o[ax] = 9.0
    d = [0.0, 0.0, 0.0]
    d[ax] = -4.0
    up = [0, 1, 0] if ax != 1 else [0, 0, 1]
    return {"cam": {"d": d, "o": o, "screen_height": 4.0, "screen_width": 6.0, "up": up, "view_eulers": [0, 0, 0]},
            "render_info": {"gpu_render_batch": 1, "height": 96, "width": 144, "kd_tree_depth": 17,
                            "rad_info": {"debug_single_ray": False, "dir_light_samp": False,
                                         "russ_roull_info": {"assured_depth": 3, "max_thres": 0.5}},
                            "samps_per_pix": 4, "use_gpu": True},
            "scene_members": members}


@pytest.mark.parametrize("seed", range(6))
def test_axis_aligned_triangles_bit_exact(gpu_available, oracle, monkeypatch, seed):
    import parity
    from rt_amd import render, scheme

    sc = scheme.load(_axis_aligned_triangles(seed))
    tiles = [(0, 0, 144, 96)]
    o = oracle.render(sc, tiles, 0, 4, accum=oracle.ACCUM_FORWARD)
    assert np.isfinite(o).all() and (o[:, :3].sum(1) > 0).mean() > 0.99
    for env in ({}, {"RT_DEBUG_KD_RESTART": "1"}, {"RT_DEBUG_PACKET": "0"}):
        for k in ("RT_DEBUG_KD_RESTART", "RT_DEBUG_PACKET"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        with render.Context(sc) as c:
            g = c.render(tiles, 0, 4)
        assert np.array_equal(g, o), (env, parity.stats(g, o))
