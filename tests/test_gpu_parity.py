"""Device path vs the CPU oracle on the same seeded inputs (walled.yml: 13 spheres, full
depth-17 KD tree).  Crops keep the oracle to seconds; full-frame properties (batching and
tiling invariance) are checked bit-exactly on the device alone."""
import ctypes as C

import numpy as np
import pytest

import parity
from conftest import load_scene

pytestmark = pytest.mark.gpu

CROPS = [(560, 260, 64, 32), (100, 400, 64, 32), (900, 80, 64, 32), (1168, 584, 32, 16)]
SPP = 16


@pytest.fixture(scope="module")
def ctx(gpu_available, walled):
    from rt_amd import render

    with render.Context(walled, device=0) as c:
        yield c


@pytest.fixture(scope="module")
def oracle_fwd(oracle, walled):
    return oracle.render(walled, CROPS, 0, SPP, accum=oracle.ACCUM_FORWARD)


def test_debug_single_ray_bit_exact(gpu_available, oracle):
    """debug_single_ray (radiance.rs:31-32): first-hit emission only — camera + KD traversal +
    closest-hit selection, no transcendental: bit-exact."""
    from rt_amd import render

    sc = load_scene("walled")
    sc.info.debug_single_ray = 1
    with render.Context(sc) as c:
        g = c.render(CROPS, 0, 4)
    o = oracle.render(sc, CROPS, 0, 4)
    assert np.array_equal(g, o), parity.stats(g, o)


def test_walled_forward_parity(ctx, oracle_fwd):
    g = ctx.render(CROPS, 0, SPP)
    s = parity.stats(g, oracle_fwd)
    print("forward", s)
    # same operation order and glibc's transcendentals (include/rt_libm.h): bit-identical
    assert np.array_equal(g, oracle_fwd), s


def test_walled_recursive_parity(ctx, oracle, walled):
    """Against the reference's own recursive accumulation order (radiance.rs:44,59)."""
    o = oracle.render(walled, CROPS, 0, SPP, accum=oracle.ACCUM_RECURSIVE)
    g = ctx.render(CROPS, 0, SPP)
    s = parity.stats(g, o)
    print("recursive", s)
    assert s["frac_ok"] >= parity.MIN_FRAC, s
    assert s["mean_rel_err"] < 1e-3


def test_batching_is_bit_invariant(ctx):
    """Running mean keyed on the absolute sample index: one launch == split launches."""
    one = ctx.render(CROPS, 0, 12)
    ctx.render(CROPS, 0, 5, want_output=False)
    two = ctx.render(CROPS, 5, 7)
    assert np.array_equal(one, two)


def test_tiling_is_bit_invariant(ctx):
    whole = ctx.render([(560, 260, 64, 32)], 0, 6)
    quads = ctx.render([(560, 260, 32, 16), (592, 260, 32, 16), (560, 276, 32, 16), (592, 276, 32, 16)], 0, 6)
    q = quads.reshape(4, 16, 32, 4)
    rebuilt = np.zeros((32, 64, 4), np.float32)
    rebuilt[:16, :32], rebuilt[:16, 32:], rebuilt[16:, :32], rebuilt[16:, 32:] = q
    assert np.array_equal(whole.reshape(32, 64, 4), rebuilt)


def test_odd_tiles_and_frame_edges(ctx, oracle, walled):
    tiles = [(0, 0, 1, 1), (1199, 599, 1, 1), (3, 7, 17, 9), (1181, 590, 19, 10)]
    g = ctx.render(tiles, 0, 4)
    o = oracle.render(walled, tiles, 0, 4, accum=oracle.ACCUM_FORWARD)
    assert np.array_equal(g, o), parity.stats(g, o)


def test_work_counts_match_oracle(ctx, oracle, walled):
    """The device visits the same KD nodes / leaf refs as the reference's traversal."""
    crops = CROPS[:2]
    _, oc = oracle.render(walled, crops, 0, 8, accum=oracle.ACCUM_FORWARD, counts=True)
    gc = ctx.count_work(crops, 0, 8)
    print("oracle", oc, "\ngpu", gc)
    for k in ("samples", "segments", "nodes", "leaf_refs", "sphere_tests", "hits"):
        assert gc[k] == oc[k], (k, gc[k], oc[k])  # bit-identical paths: identical work


def test_device_output_pointer(ctx):
    import torch

    g = ctx.render(CROPS[:1], 0, 3)
    buf = torch.empty((64 * 32, 4), dtype=torch.float32, device="cuda:0")
    ctx.render_device(buf.data_ptr(), CROPS[:1], 0, 3)
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy(), g)


@pytest.mark.parametrize("scene_name,crop,spp", [("walled", (560, 260, 64, 32), 16),
                                                  ("walled", (100, 40, 32, 32), 16),
                                                  ("spaceship_r1", (450, 200, 32, 32), 8)])
def test_dir_light_samp_parity(gpu_available, oracle, scene_name, crop, spp):
    """Direct-light sampling (radiance.rs:46-56,89-120) on the device vs the oracle: the forward
    oracle defers each vertex's DLS term exactly as the kernel does; the recursive one is the
    reference's order (gate of DESIGN.md §3)."""
    from rt_amd import render

    sc = load_scene(scene_name)
    sc.info.dir_light_samp = 1
    with render.Context(sc) as ctx:
        g = ctx.render([crop], 0, spp)
    f = oracle.render(sc, [crop], 0, spp, accum=oracle.ACCUM_FORWARD)
    r = oracle.render(sc, [crop], 0, spp, accum=oracle.ACCUM_RECURSIVE)
    plain = oracle.render(load_scene(scene_name), [crop], 0, spp, accum=oracle.ACCUM_FORWARD)
    sf, sr = parity.stats(g, f), parity.stats(g, r)
    print(scene_name, "vs forward", sf, "\n vs recursive", sr, "\n DLS effect", float(np.abs(f - plain).max()))
    assert np.array_equal(g, f), sf
    assert sr["frac_ok"] >= parity.MIN_FRAC, sr
    assert parity.frac_u8_within(g, r) >= parity.MIN_FRAC
    if scene_name == "walled":
        assert float(np.abs(f - plain).max()) > 1e-3  # the crop exercises DLS


def test_dir_light_samp_diffspec_emitter(gpu_available, oracle):
    """DLS towards a DiffSpec emitter: the light's hit_info seeds it with one draw
    (sphere.rs:76, uniform_diff_spec.rs:33-36), which the reference makes only after the whole
    recursive subtree (radiance.rs:44-56,108), so it shifts no path draw.  Device, forward oracle
    and recursive oracle must agree; device == forward oracle bit for bit."""
    import json
    import os

    from conftest import SCENES
    from rt_amd import render, scheme

    d = json.load(open(os.path.join(SCENES, "walled.json")))
    n_emit = 0
    for m in d["scene_members"]:
        mat = m.get("!Sphere", {}).get("mat", {})
        if "emissive" in mat:
            mat["divert_ray"] = {"!DiffSpec": {"diffp": 0.6}}
            n_emit += 1
    assert n_emit == 2
    d["render_info"]["rad_info"]["dir_light_samp"] = True
    sc = scheme.load(d)
    crop = [(560, 260, 48, 24), (100, 40, 24, 24)]
    with render.Context(sc) as ctx:
        g = ctx.render(crop, 0, 12)
    f = oracle.render(sc, crop, 0, 12, accum=oracle.ACCUM_FORWARD)
    r = oracle.render(sc, crop, 0, 12, accum=oracle.ACCUM_RECURSIVE)
    sf, sr = parity.stats(g, f), parity.stats(g, r)
    print("diffspec emitter: vs forward", sf, "\n vs recursive", sr)
    assert np.array_equal(g, f), sf
    assert sr["frac_ok"] >= parity.MIN_FRAC, sr
    assert sr["mean_rel_err"] < 1e-3


def test_dir_light_samp_schedules_agree(gpu_available, monkeypatch):
    from rt_amd import render

    sc = load_scene("walled")
    sc.info.dir_light_samp = 1
    tiles = [(560, 260, 40, 20), (3, 5, 9, 7)]
    monkeypatch.setenv("RT_DEBUG_SCHED", "direct")
    with render.Context(sc) as c1:
        ref = c1.render(tiles, 0, 9)
    monkeypatch.setenv("RT_DEBUG_SCHED", "queue")
    with render.Context(sc) as c2:
        assert np.array_equal(c2.render(tiles, 0, 9), ref)


@pytest.mark.parametrize("k,spp", [(2, 37), (4, 37), (8, 21), (2, 300)])
def test_lanes_per_pixel_bit_invariant(gpu_available, walled, monkeypatch, k, spp):
    """K lanes per pixel + fold kernel (multi-GPU occupancy path) == K = 1, bit for bit,
    including remainders and several sample chunks (300 > 64 * 2)."""
    from rt_amd import render

    crops = CROPS[:2] if spp < 100 else [(560, 260, 16, 8)]
    monkeypatch.setenv("RT_DEBUG_SCHED", "direct:1")
    with render.Context(walled) as c1:
        ref = c1.render(crops, 0, spp)
        ref2 = c1.render(crops, spp, 5)
    monkeypatch.setenv("RT_DEBUG_SCHED", f"direct:{k}")
    with render.Context(walled) as ck:
        g = ck.render(crops, 0, spp)
        g2 = ck.render(crops, spp, 5)
    assert np.array_equal(g, ref)
    assert np.array_equal(g2, ref2)


def test_device_work_is_a_subset_of_the_reference(ctx):
    """The small-scene bound only skips work: same samples/segments/hits, fewer nodes."""
    ref = ctx.count_work(CROPS[:1], 0, 4)
    dev = ctx.count_work(CROPS[:1], 0, 4, device=True)
    print("reference", ref, "\ndevice", dev)
    for k in ("samples", "segments", "hits"):
        assert dev[k] == ref[k], k
    assert dev["nodes"] < ref["nodes"] and dev["leaf_refs"] <= ref["leaf_refs"]


@pytest.mark.parametrize("scene_name,spp", [("walled", 37), ("walled", 5), ("biplane", 3), ("spaceship_r1", 2)])
def test_queue_schedule_bit_invariant(gpu_available, monkeypatch, scene_name, spp):
    """Queue schedule (persistent lanes over (pixel, sample) items + in-order fold) == direct
    one-lane-per-pixel schedule, bit for bit, over several tiles and a second sample range."""
    from rt_amd import render

    sc = load_scene(scene_name)
    w, h = sc.info.width, sc.info.height
    tiles = [(w // 2 - 40, h // 2 - 20, 80, 40), (0, 0, 7, 3), (w - 33, h - 9, 33, 9)]
    monkeypatch.setenv("RT_DEBUG_SCHED", "direct")
    with render.Context(sc) as c1:
        ref = c1.render(tiles, 0, spp)
        ref2 = c1.render(tiles, spp, 4)
    monkeypatch.setenv("RT_DEBUG_SCHED", "queue")
    with render.Context(sc) as cq:
        g = cq.render(tiles, 0, spp)
        g2 = cq.render(tiles, spp, 4)
    assert np.array_equal(g, ref)
    assert np.array_equal(g2, ref2)


@pytest.mark.parametrize("scene_name,spp", [("walled", 23), ("biplane", 5)])
def test_split_queue_launches_bit_invariant(gpu_available, monkeypatch, scene_name, spp):
    """A radiance cap small enough to split one call into several queue launches (each with
    its own drain and fold) == one launch, bit for bit (runtime.hip's chunk loop; the bench's
    1000-spp step is one launch under the default 16 GiB cap)."""
    from rt_amd import render

    sc = load_scene(scene_name)
    w, h = sc.info.width, sc.info.height
    tiles = [(w // 2 - 40, h // 2 - 20, 80, 40), (w - 33, h - 9, 33, 9)]
    n_pix = 80 * 40 + 33 * 9
    monkeypatch.delenv("RT_DEBUG_LAUNCH", raising=False)
    with render.Context(sc) as c1:
        ref = c1.render(tiles, 0, spp)
    monkeypatch.setenv("RT_DEBUG_LAUNCH", f"radiance_floats={3 * n_pix * 4}")  # 4 samples per launch
    with render.Context(sc) as cs:
        g = cs.render(tiles, 0, spp)
        n_split = cs.launch_stats()["n_trace_launches"]
    assert n_split == -(-spp // 4), n_split
    assert np.array_equal(g, ref)


def _adversarial_spheres(seed: int) -> dict:
    """<= 32 spheres built to make the closest-hit decision hard: duplicates (exact ties),
    concentric shells 1e-4 apart, tangent pairs, tiny spheres, deep overlaps and r = 500 walls
    (hits near their poles).  Each sphere emits a distinct colour, so a first-hit image says
    which sphere every camera ray returned."""
    rng = np.random.default_rng(seed)
    sph = []
    for c, r in (((515.0, 0.0, -10.0), 500.0), ((-515.0, 0.0, -10.0), 500.0),
                 ((0.0, -510.0, -10.0), 500.0), ((0.0, 0.0, -530.0), 500.0)):
        sph.append((c, r))
    while len(sph) < 30:
        kind = rng.integers(0, 5)
        c = rng.uniform(-6.0, 6.0, 3).astype(np.float32)
        r = np.float32(rng.uniform(0.2, 3.0))
        if kind == 0:                        # exact duplicate of an earlier sphere
            sph.append(sph[rng.integers(4, len(sph))] if len(sph) > 4 else (tuple(c), r))
        elif kind == 1:                      # concentric shells
            sph.append((tuple(c), r))
            sph.append((tuple(c), np.float32(r + 1e-4)))
        elif kind == 2:                      # tangent pair
            u = rng.normal(size=3)
            u /= np.linalg.norm(u)
            r2 = np.float32(rng.uniform(0.2, 2.0))
            sph.append((tuple(c), r))
            sph.append((tuple(np.float32(c + (r + r2) * u)), r2))
        elif kind == 3:                      # tiny sphere
            sph.append((tuple(c), np.float32(rng.uniform(1e-3, 2e-2))))
        else:
            sph.append((tuple(c), r))
    sph = sph[:30]
    members = []
    for i, (c, r) in enumerate(sph):
        em = [(i + 1) / 32.0, ((i * 7) % 31 + 1) / 32.0, ((i * 13) % 29 + 1) / 32.0]
        members.append({"!Sphere": {"c": [float(x) for x in c], "r": float(r),
                                    "coloring": {"!Solid": [0.5, 0.5, 0.5]},
                                    "mat": {"divert_ray": "Diff", "emissive": em}}})
    # camera: inside the cluster; on a sphere's surface looking out; grazing the floor wall
    # (hits near its pole); inside the floor wall sphere
    i = int(rng.integers(4, len(sph)))
    u = rng.normal(size=3)
    u /= np.linalg.norm(u)
    d = rng.normal(size=3)
    d[1] *= 0.3
    kind = seed % 4
    if kind == 0:
        o = rng.uniform(-4.0, 4.0, 3)
    elif kind == 1:
        o = np.float32(np.array(sph[i][0]) + sph[i][1] * u)
        d = u + 0.3 * rng.normal(size=3)
    elif kind == 2:
        o = np.array([rng.uniform(-3, 3), -9.9, rng.uniform(-8, 2)])
        d[1] = -abs(d[1]) * 0.2
    else:
        o = np.array([0.0, -10.5, -10.0])
    d = 5.0 * d / np.linalg.norm(d)
    return {"cam": {"d": [float(x) for x in d], "o": [float(x) for x in o], "screen_height": 5.0,
                    "screen_width": 10.0, "up": [0, 1, 0], "view_eulers": [0, 0, 0]},
            "render_info": {"gpu_render_batch": 1, "height": 96, "width": 160, "kd_tree_depth": 17,
                            "rad_info": {"debug_single_ray": True, "dir_light_samp": False,
                                         "russ_roull_info": {"assured_depth": 5, "max_thres": 0.5}},
                            "samps_per_pix": 1, "use_gpu": True},
            "scene_members": members}


@pytest.mark.parametrize("seed", range(12))
def test_small_scene_closest_sphere_bit_exact(gpu_available, oracle, seed):
    """closest_small's exact shortcuts (descent floor, pmin leaf, no traversal when the closest
    sphere is provably in the returning leaf) against the oracle's full KD traversal, first hit
    only, on adversarial sphere sets: the returned sphere must match for every ray."""
    from rt_amd import render, scheme

    sc = scheme.load(_adversarial_spheres(seed))
    tiles = [(0, 0, 160, 96)]
    with render.Context(sc) as c:
        g = c.render(tiles, 0, 3)
    o = oracle.render(sc, tiles, 0, 3)
    assert np.array_equal(g, o), parity.stats(g, o)


def test_sphere_scene_beyond_small_bound(gpu_available, oracle):
    """A sphere-only scene with a sphere centred at 2^59: the host clears small_ok
    (runtime.hip), so the sphere-only kernel runs the full KD traversal instead of
    closest_small, whose root arithmetic assumes coordinates below 2^58.  Still the oracle's
    image, bit for bit."""
    from rt_amd import render, scheme

    d = _adversarial_spheres(1)
    d["scene_members"].append({"!Sphere": {"c": [2.0 ** 59, 1.0, -4.0], "r": 1.0,
                                           "coloring": {"!Solid": [0.5, 0.5, 0.5]},
                                           "mat": {"divert_ray": "Diff", "emissive": [1.0, 0.0, 0.0]}}})
    sc = scheme.load(d)
    tiles = [(0, 0, 160, 96)]
    with render.Context(sc) as c:
        g = c.render(tiles, 0, 3)
    o = oracle.render(sc, tiles, 0, 3)
    assert np.array_equal(g, o), parity.stats(g, o)


def test_wide_frame_without_pixel_table(gpu_available, oracle):
    """A frame over 65535 pixels wide cannot use the packed (y << 16 | x) pixel table
    (runtime.hip prepare_tiles): the kernels fall back to the binary search over the tiles.
    Both paths must give the oracle's pixels, for one tile and for several."""
    from rt_amd import render

    sc = load_scene("walled", width=70000, height=3)
    tiles = [(0, 0, 40, 1), (69990, 2, 10, 1), (35000, 1, 33, 2)]
    with render.Context(sc) as c:
        g = c.render(tiles, 0, 4)
        g1 = c.render([(34990, 0, 64, 3)], 0, 4)
    o = oracle.render(sc, tiles, 0, 4, accum=oracle.ACCUM_FORWARD)
    o1 = oracle.render(sc, [(34990, 0, 64, 3)], 0, 4, accum=oracle.ACCUM_FORWARD)
    assert np.array_equal(g, o), parity.stats(g, o)
    assert np.array_equal(g1, o1), parity.stats(g1, o1)


@pytest.mark.parametrize("scene_name,spp,batch", [("walled", 12, 3), ("biplane", 6, 1), ("spaceship_r1", 6, 2)])
def test_async_pipeline_bit_invariant(gpu_available, monkeypatch, scene_name, spp, batch):
    """rt_render_device_async: consecutive batches overlap on two pipeline slots (trace i + 1
    during trace i's drain; folds chained by events) == synchronous batches, bit for bit — also
    with each batch split into several queue launches (small radiance cap) and with a
    direct-schedule call in between."""
    import torch

    from rt_amd import render

    sc = load_scene(scene_name)
    w, h = sc.info.width, sc.info.height
    tiles = [(w // 2 - 48, h // 2 - 24, 96, 48), (0, 0, 9, 5)]
    n = 96 * 48 + 9 * 5
    with render.Context(sc) as c1:
        ref = c1.render(tiles, 0, spp)
    for pipe, cap in (("2", None), ("0", None), ("2", str(3 * n * 2))):  # cap: 2 samples per launch
        # overlapped launches, or each after the last fold
        monkeypatch.setenv("RT_DEBUG_LAUNCH", f"overlap={pipe}" + (f",radiance_floats={cap}" if cap else ""))
        with render.Context(sc) as ca:
            out = torch.full((n, 4), -1.0, dtype=torch.float32, device="cuda:0")
            stream = torch.cuda.current_stream().cuda_stream
            for s0 in range(0, spp, batch):
                ca.render_device_async(out.data_ptr(), tiles, s0, batch, stream=stream)
            got = out.cpu().numpy()  # ordered after the last fold on torch's stream
            ca.synchronize()
            st = ca.launch_stats()
            assert st["n_trace_launches"] >= spp // batch
        assert np.array_equal(got, ref), (pipe, cap, parity.stats(got, ref))
    # a synchronous call between async ones
    assert spp >= 3 * batch
    monkeypatch.delenv("RT_DEBUG_LAUNCH", raising=False)
    with render.Context(sc) as cm:
        out = torch.zeros((n, 4), dtype=torch.float32, device="cuda:0")
        cm.render_device_async(out.data_ptr(), tiles, 0, batch)
        mid = cm.render(tiles, batch, batch)  # synchronous
        for s0 in range(2 * batch, spp, batch):
            cm.render_device_async(out.data_ptr(), tiles, s0, batch)
        cm.synchronize()
        torch.cuda.synchronize()
        got = out.cpu().numpy()
    with render.Context(sc) as c2:
        ref2 = c2.render(tiles, 0, 2 * batch)
    assert np.array_equal(mid, ref2)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("scene_name,spp,batch", [("walled", 6, 2), ("biplane", 12, 1)])
def test_render_to_target_pipelined_equals_batches(gpu_available, scene_name, spp, batch):
    """rt_render_to_target keeps up to 7 batches in flight (each into its own output buffer,
    reused after its read-back): every RGBA8 frame handed to the update hook, in order, equals
    the synchronous batch loop's."""
    from rt_amd import render

    sc = load_scene(scene_name, width=160, height=96)
    frames = []
    render.render_to_target(sc, spp, batch, update_hook=lambda t, done: frames.append((done, t.copy())))
    assert [d for d, _ in frames] == list(range(batch, spp + 1, batch))
    with render.Context(sc) as c:
        for i, s0 in enumerate(range(0, spp, batch)):
            img = c.render(None, s0, batch)
            assert np.array_equal(frames[i][1].reshape(-1, 4), render.rgba_to_u8(img)), s0


@pytest.mark.parametrize("scene_name,spp", [("walled", 9), ("triangles", 4), ("biplane", 3), ("spaceship_r1", 3),
                                            ("a380", 2)])
def test_stackless_traversal_bit_invariant(gpu_available, oracle, monkeypatch, scene_name, spp):
    """Stackless kd-restart with push-down (RT_DEBUG_KD_RESTART=1: after a leaf, descend again from the
    deepest node above the first push, entry = the leaf's exit) and the stack traversal
    (RT_DEBUG_KD_RESTART=0) each render the forward oracle's image (the reference's stack traversal,
    kdtree.rs:66-104), bit for bit, in the queue kernels."""
    from rt_amd import render

    sc = load_scene(scene_name)
    w, h = sc.info.width, sc.info.height
    tiles = [(w // 2 - 64, h // 2 - 32, 128, 64), (0, h - 16, 48, 16)]
    o = oracle.render(sc, tiles, 0, spp, accum=oracle.ACCUM_FORWARD)
    for rs in ("0", "1"):
        monkeypatch.setenv("RT_DEBUG_KD_RESTART", rs)
        with render.Context(sc) as c:
            g = c.render(tiles, 0, spp)
        assert np.array_equal(g, o), (rs, parity.stats(g, o))
    monkeypatch.delenv("RT_DEBUG_KD_RESTART")


@pytest.mark.parametrize("scene_name,spp", [("triangles", 4), ("biplane", 3), ("spaceship_r1", 3), ("a380", 2)])
def test_packet_traversal_bit_invariant(gpu_available, oracle, monkeypatch, scene_name, spp):
    """Camera-ray packets (closest_packet: scalar-loaded nodes and leaf refs, per-lane
    near / far / push on the lane's own interval, deferred lanes, kd-restart from the packet's
    restart node, hand-over to the cooperative search), the cooperative search alone
    (RT_DEBUG_PACKET=0) and the row-order queue (RT_DEBUG_PIX_BLOCK=1) each render the forward oracle's image
    (kdtree.rs:66-104), bit for bit, on two tiles and a full frame."""
    from rt_amd import render

    sc = load_scene(scene_name, width=320, height=160)
    w, h = sc.info.width, sc.info.height
    tiles = [(w // 2 - 64, h // 2 - 32, 128, 64), (0, h - 16, 48, 16)]
    o_tiles = oracle.render(sc, tiles, 0, spp, accum=oracle.ACCUM_FORWARD)
    o_full = oracle.render(sc, [(0, 0, w, h)], 0, 2 * spp, accum=oracle.ACCUM_FORWARD)
    for cfg in (("1", "8"), ("0", "1"), ("1", "1"), ("0", "8")):
        monkeypatch.setenv("RT_DEBUG_PACKET", cfg[0])
        monkeypatch.setenv("RT_DEBUG_PIX_BLOCK", cfg[1])
        with render.Context(sc) as c:
            got = c.render(tiles, 0, spp)
        assert np.array_equal(got, o_tiles), (cfg, parity.stats(got, o_tiles))
        with render.Context(sc) as c:  # whole frame, two calls: [0, spp) then [spp, 2 spp)
            c.render(None, 0, spp, want_output=False)
            full = c.render(None, spp, spp)
        assert np.array_equal(full, o_full), (cfg, parity.stats(full, o_full))


@pytest.mark.parametrize("scene_name,spp", [("triangles", 4), ("biplane", 2), ("walled", 6)])
def test_queue_shards_bit_invariant(gpu_available, oracle, monkeypatch, scene_name, spp):
    """The queue's items in 1, 3, 8 or 32 shards with a counter each (trace.hip qgrab: a wave
    starts on its own shard and walks on when it is exhausted; the last shard may end inside a
    grab) render the forward oracle's image bit for bit, on a frame whose item count is not a
    multiple of 64 and on tiles; the sphere-only kernel ignores the shards (one counter)."""
    from rt_amd import render

    sc = load_scene(scene_name, width=203, height=97)  # 19,691 pixels: shards end off the 64 grid
    w, h = sc.info.width, sc.info.height
    tiles = [(w // 2 - 40, h // 2 - 20, 80, 40), (0, h - 7, 33, 7)]
    o_full = oracle.render(sc, [(0, 0, w, h)], 0, spp, accum=oracle.ACCUM_FORWARD)
    o_tiles = oracle.render(sc, tiles, 0, spp, accum=oracle.ACCUM_FORWARD)
    for n in ("1", "3", "8", "32"):
        monkeypatch.setenv("RT_DEBUG_LAUNCH", f"shards={n}")
        with render.Context(sc) as c:
            full = c.render(None, 0, spp)
            got = c.render(tiles, 0, spp)
        assert np.array_equal(full, o_full), (n, parity.stats(full, o_full))
        assert np.array_equal(got, o_tiles), (n, parity.stats(got, o_tiles))


def test_small_launch_pipeline_bit_invariant(gpu_available, oracle, monkeypatch):
    """Small overlapped launches (a380's batch of 1 spp): 12 pipeline slots, each launch behind a
    busy pipeline on 1/8 of the resident grid (runtime.hip slots_for_queues / small_grid_div),
    async calls back to back, equal the oracle over the same samples bit for bit — also with 1/2
    and 1/16 of the grid and 3 slots."""
    import torch

    from rt_amd import render

    sc = load_scene("a380", width=160, height=80)
    w, h = sc.info.width, sc.info.height
    spp = 6
    o = oracle.render(sc, [(0, 0, w, h)], 0, spp, accum=oracle.ACCUM_FORWARD)
    for slots, div in (("12", "8"), ("12", "2"), ("3", "16")):
        monkeypatch.setenv("RT_DEBUG_LAUNCH", f"slots={slots},grid_div={div}")
        with render.Context(sc) as c:
            out = torch.zeros((w * h, 4), dtype=torch.float32, device="cuda:0")
            stream = torch.cuda.current_stream().cuda_stream
            for s0 in range(spp):  # one sample per call: every launch is small
                c.render_device_async(out.data_ptr(), [(0, 0, w, h)], s0, 1, stream=stream)
            c.synchronize()
            torch.cuda.synchronize()
            got = out.cpu().numpy().reshape(h, w, 4)
        assert np.array_equal(got, o.reshape(h, w, 4)), (slots, div, parity.stats(got, o.reshape(h, w, 4)))


def test_sphere_scene_with_lens_bit_exact(gpu_available, oracle):
    """walled.yml with its commented-out lens (`lens_r: 0.1`): the sphere-only kernel keeps the
    per-lane path starts for lens cameras (RT_START_BATCH covers lens-free ones), and both render
    the forward oracle's bits (generate.rs:24-66)."""
    import json
    import os

    from conftest import SCENES
    from rt_amd import render, scheme

    d = json.load(open(os.path.join(SCENES, "walled.json")))
    d["cam"]["lens_r"] = 0.1
    sc = scheme.load(d)
    assert sc.cam.has_lens == 1
    crop = [(560, 260, 48, 24), (0, 0, 16, 16)]
    with render.Context(sc) as ctx:
        g = ctx.render(crop, 3, 8)
    f = oracle.render(sc, crop, 3, 8, accum=oracle.ACCUM_FORWARD)
    s = parity.stats(g, f)
    print("walled with lens", s)
    assert np.array_equal(g, f), s
