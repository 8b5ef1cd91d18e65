"""Edge cases through the C ABI, on the device, against the oracle: scenes with nothing in them or
one primitive, a 1 x 1 frame, sample indices past 2^32, zero-sample calls and rejected arguments.
The reference behaviour is render_to_target_cpu / closest_ray_hit (draw_scene.rs:49-101,
closest_hit.rs:6-30, kdtree.rs:58-64 with an empty element list going straight to the
unconditional renderables)."""
import copy

import numpy as np
import pytest

import parity

pytestmark = pytest.mark.gpu


def _scheme(members, w=48, h=32, depth=5):
    from rt_amd import scheme

    base = scheme.load_json(__import__("conftest").SCENES + "/walled.json")
    d = copy.deepcopy(base)
    d["scene_members"] = members
    d["render_info"]["width"] = w
    d["render_info"]["height"] = h
    d["render_info"]["rad_info"]["russ_roull_info"]["assured_depth"] = depth
    return scheme.load(d)


def _walled_members():
    from rt_amd import scheme

    return scheme.load_json(__import__("conftest").SCENES + "/walled.json")["scene_members"]


TRI = {"!FreeTriangle": {"mat": {"divert_ray": {"!DiffSpec": {"diffp": 0.5}}}, "norm": [0, 0, 1],
                         "rgb": [0.9, 0.6, 0.3], "verts": [[-6, -4, -20], [6, -4, -20], [0, 6, -20]]}}
LIGHT = {"!Sphere": {"c": [0.0, 10.0, -15.0], "coloring": {"!Solid": [0.0, 0.0, 0.0]},
                     "mat": {"divert_ray": "Diff", "emissive": [5.0, 5.0, 5.0]}, "r": 5.0}}


@pytest.mark.parametrize("members", [[], [LIGHT], [TRI], [TRI, LIGHT]], ids=["empty", "one_sphere", "one_triangle", "triangle_and_light"])
def test_tiny_scenes_bit_exact(gpu_available, oracle, members):
    """No renderable at all (every ray misses: black), one sphere (the sphere-only kernel), one
    free triangle and a triangle beside an emitter (the general kernel), whole frame, bit for bit
    against the forward oracle."""
    from rt_amd import render

    sc = _scheme(members)
    tiles = [(0, 0, 48, 32)]
    with render.Context(sc) as c:
        g = c.render(tiles, 0, 6)
    o = oracle.render(sc, tiles, 0, 6, accum=oracle.ACCUM_FORWARD)
    assert np.array_equal(g, o), parity.stats(g, o)
    if not members:
        assert not g[:, :3].any() and (g[:, 3] == 1.0).all()


def test_one_pixel_frame(gpu_available, oracle):
    """A 1 x 1 frame (n_pix = 1: the queue's item split takes its n_pix == 1 branch)."""
    from rt_amd import render

    sc = _scheme(_walled_members(), w=1, h=1)
    with render.Context(sc) as c:
        g = c.render([(0, 0, 1, 1)], 0, 64)
    o = oracle.render(sc, [(0, 0, 1, 1)], 0, 64, accum=oracle.ACCUM_FORWARD)
    assert np.array_equal(g, o), parity.stats(g, o)


def test_sample_indices_past_2_32(gpu_available, oracle, walled):
    """Samples 2^32 + 3 .. 2^32 + 7: the (pixel, sample) stream key is 64-bit on both sides
    (include/rt_rng.h), and the accumulator fold's n = sample index as f32."""
    from rt_amd import render

    tiles = [(600, 300, 16, 8)]
    s0 = (1 << 32) + 3
    with render.Context(walled) as c:
        g = c.render(tiles, s0, 4)
    o = oracle.render(walled, tiles, s0, 4, accum=oracle.ACCUM_FORWARD)
    assert np.array_equal(g, o), parity.stats(g, o)


def test_zero_sample_call_leaves_the_image(gpu_available, walled):
    """rt_render with sample_count 0 folds nothing: the returned pixels are the accumulator as
    the previous call left it."""
    from rt_amd import render

    tiles = [(580, 290, 24, 12)]
    with render.Context(walled) as c:
        a = c.render(tiles, 0, 5)
        b = c.render(tiles, 5, 0)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("tiles", [[(1190, 0, 16, 4)], [(0, 598, 4, 4)], [(0, 0, 0, 4)]],
                         ids=["past_right_edge", "past_bottom_edge", "zero_width"])
def test_bad_tiles_are_rejected(gpu_available, walled, tiles):
    """A tile reaching outside the frame, or an empty one, is RT_ERR_INVALID_ARG, and the
    context stays usable."""
    from rt_amd import abi, render

    with render.Context(walled) as c:
        with pytest.raises(abi.RtError) as e:
            c.render(tiles, 0, 1)
        assert e.value.status == abi.RT_ERR_INVALID_ARG
        g = c.render([(0, 0, 8, 8)], 0, 1)
    assert g.shape == (64, 4) and (g[:, 3] == 1.0).all()


def test_empty_leaves_with_stale_offsets(gpu_available, monkeypatch):
    """A caller-supplied tree whose empty leaves keep large ref offsets (every third leaf of
    spaceship_r1's tree emptied, its offset pointed at the last ref): the upload's ref-list
    dedupe shrinks the ref array ~25x, so such an offset would lie far past the packed list.
    Camera-ray packets (closest_packet, scalar loads ahead of the leaf's tests), the cooperative
    search and the stackless kernels must read nothing for an empty leaf: all give the same image,
    and it differs from the full tree's (the emptied leaves are visited)."""
    from rt_amd import render
    from conftest import load_scene

    sc = load_scene("spaceship_r1", width=320, height=160)
    tree = render.KdTree(sc.desc, int(sc.info.kd_tree_depth))
    nodes = tree.nodes.copy()
    leaves = np.flatnonzero((nodes[:, 1] & 3) == 3)
    emptied = leaves[::3]
    nodes[emptied, 0] = 0
    nodes[emptied, 1] = ((tree.n_refs - 1) << 2) | 3
    t = tree.as_struct(nodes=nodes)
    imgs = {}
    for cfg in (("1", "0"), ("0", "0"), ("1", "1")):
        monkeypatch.setenv("RT_DEBUG_PACKET", cfg[0])
        monkeypatch.setenv("RT_DEBUG_KD_RESTART", cfg[1])
        with render.Context(sc, tree=t) as c:
            imgs[cfg] = c.render(None, 0, 2)
    ref = imgs[("1", "0")]
    for cfg, g in imgs.items():
        assert np.array_equal(g, ref), (cfg, parity.stats(g, ref))
    monkeypatch.setenv("RT_DEBUG_PACKET", "1")
    monkeypatch.setenv("RT_DEBUG_KD_RESTART", "0")
    with render.Context(sc) as c:
        full = c.render(None, 0, 2)
    assert not np.array_equal(full, ref)


def test_shortcut_needs_bounds_around_every_sphere(gpu_available):
    """closest_small's in_return_leaf stands in for the root slab test only when the tree's bounds
    contain every sphere's box (runtime.hip small_ok).  With the builder's tree the
    shortcut runs (a few node visits per sample against the reference's hundreds); a caller tree
    whose bounds cut the +x wall sphere's box must take the plain traversal, which does at least
    the reference's node work (the kd-restart only adds visits)."""
    from rt_amd import render
    from conftest import load_scene

    sc = load_scene("walled", width=80, height=40)
    tree = render.KdTree(sc.desc, int(sc.info.kd_tree_depth))
    with render.Context(sc, tree=tree.as_struct()) as c:
        dev, ref = c.count_work(None, 0, 2, device=True), c.count_work(None, 0, 2)
    assert dev["segments"] == ref["segments"] and dev["nodes"] < 0.01 * ref["nodes"], (dev, ref)
    tree.bounds[1] = tree.bounds[1] * 0.5  # x max: 1015 -> 507, inside the wall sphere's [15, 1015]
    with render.Context(sc, tree=tree.as_struct()) as c:
        dev_cut, ref_cut = c.count_work(None, 0, 2, device=True), c.count_work(None, 0, 2)
    assert dev_cut["nodes"] >= ref_cut["nodes"] > 0.5 * ref["nodes"], (dev_cut, ref_cut)
