"""The multi-device frame at the C ABI (rt_frame_*, rt_render_to_target_devices; frame.hip) on the
one GPU there is: N contexts on device 0, each rendering its stripes, one gather per frame.  The
assembled frame must equal one context's frame bit for bit — the stripe deal, the placement and
the frame-end gather of SURVEY.md §8e, reachable by the reference's render thread
(renderer.rs:43-60 -> render_to_target_gpu, draw_scene.rs:17-47) without torch.  BASELINE config
5's split (spaceship_r1 at 4096 x 4096 over 8 contexts: 8-row stripes, 64 per context) runs here
at 1 spp."""
import numpy as np
import pytest

from conftest import load_scene

pytestmark = pytest.mark.gpu


def one_context(loaded, begin, count):
    from rt_amd import render

    w, h = int(loaded.info.width), int(loaded.info.height)
    with render.Context(loaded, device=0) as ctx:
        return ctx.render([(0, 0, w, h)], begin, count).reshape(h, w, 4)


@pytest.mark.parametrize("scene,n", [("walled", 2), ("walled", 8), ("biplane", 3), ("triangles", 8)])
def test_frame_equals_one_context(gpu_available, scene, n):
    from rt_amd import render

    loaded = load_scene(scene)
    ref = one_context(loaded, 0, 4)
    with render.Frame(loaded, [0] * n) as f:
        f.render(0, 1)
        f.render(1, 3)  # split calls equal one call
        got = f.gather()
        st = f.stats()
    assert st["n_gathers"] == 1 and st["n_parts"] == n and st["n_peer_copies"] == 0, st
    assert (got[..., 3] == 1.0).all()
    assert np.array_equal(got, ref)


def test_frame_gathers_twice(gpu_available):
    """A second frame after a gather: the renders after the gather wait for it (stream order), and
    the second gather returns the mean over every sample so far."""
    from rt_amd import render

    loaded = load_scene("walled")
    with render.Frame(loaded, [0, 0, 0], stripe=5) as f:
        f.render(0, 2)
        first = f.gather()
        f.render(2, 2)
        second = f.gather()
        assert f.stats()["n_gathers"] == 2
    assert np.array_equal(first, one_context(loaded, 0, 2))
    assert np.array_equal(second, one_context(loaded, 0, 4))


def test_config5_split_on_one_gpu(gpu_available):
    """spaceship_r1 at 4096 x 4096 (BASELINE config 5) over 8 contexts: stripes of 8 rows, 64 per
    context, one gather; 1 spp.  Equal to one context bit for bit."""
    from rt_amd import render

    loaded = load_scene("spaceship_r1", width=4096, height=4096)
    ref = one_context(loaded, 0, 1)
    with render.Frame(loaded, [0] * 8) as f:
        assert [f.part(k)["n_tiles"] for k in range(8)] == [64] * 8
        f.render(0, 1)
        got = f.gather()
        st = f.stats()
    assert st["stripe_rows"] == 8 and st["n_gathers"] == 1, st
    assert np.array_equal(got, ref)


def test_render_to_target_devices_equals_one_device(gpu_available):
    """rt_render_to_target_devices over 3 contexts: the RGBA8 target after every batch equals
    rt_render_to_target's (hooks in order)."""
    from rt_amd import render

    loaded = load_scene("triangles")
    one, many = [], []
    t1 = render.render_to_target(loaded, 6, 2, 0, update_hook=lambda t, d: one.append((d, t.copy())))
    t3 = render.render_to_target_devices(loaded, 6, 2, [0, 0, 0], update_hook=lambda t, d: many.append((d, t.copy())))
    assert [d for d, _ in one] == [d for d, _ in many] == [2, 4, 6]
    for (_, a), (_, b) in zip(one, many):
        assert np.array_equal(a, b)
    assert np.array_equal(t1, t3)


# ---- the remote-device branch (staging buffers, peer copies, event hand-offs) on one GPU ----
# RT_DEBUG_FRAME_STAGING=1 gathers every context but the first as if it sat on another device:
# its buffer goes through hipMemcpyPeerAsync (device 0 -> device 0) into a staging buffer on the
# first device, placement reads the staging buffer, the next render waits for the copy (`copied`)
# and the next copy waits for the placement (`placed`).  frame.hip:258-310.

@pytest.mark.parametrize("scene,n", [("walled", 2), ("walled", 8), ("triangles", 8)])
def test_frame_staging_gathers_twice(gpu_available, monkeypatch, scene, n):
    from rt_amd import render

    monkeypatch.setenv("RT_DEBUG_FRAME_STAGING", "1")
    loaded = load_scene(scene)
    with render.Frame(loaded, [0] * n) as f:
        f.render(0, 2)
        first = f.gather()
        f.render(2, 1)
        f.render(3, 1)
        second = f.gather()
        st = f.stats()
    assert st["n_gathers"] == 2 and st["n_peer_copies"] == 2 * (n - 1), st
    assert st["peer_copy_ms_max"] > 0.0, st
    assert np.array_equal(first, one_context(loaded, 0, 2))
    assert np.array_equal(second, one_context(loaded, 0, 4))


def test_config5_split_through_staging(gpu_available, monkeypatch):
    """BASELINE config 5's 8-way split (spaceship_r1 4096 x 4096, 64 stripes of 8 rows per context)
    with 7 of the 8 contexts gathered through staging, two gathers in a row."""
    from rt_amd import render

    monkeypatch.setenv("RT_DEBUG_FRAME_STAGING", "1")
    loaded = load_scene("spaceship_r1", width=4096, height=4096)
    ref1 = one_context(loaded, 0, 1)
    ref2 = one_context(loaded, 0, 2)
    with render.Frame(loaded, [0] * 8) as f:
        f.render(0, 1)
        got1 = f.gather()
        f.render(1, 1)
        got2 = f.gather()
        st = f.stats()
    assert st["stripe_rows"] == 8 and st["n_gathers"] == 2 and st["n_peer_copies"] == 14, st
    assert np.array_equal(got1, ref1)
    assert np.array_equal(got2, ref2)


def test_render_to_target_devices_through_staging(gpu_available, monkeypatch):
    """rt_render_to_target_devices with 3 contexts, 2 of them gathered through staging: every
    batch's RGBA8 target (three gathers, pipelined) equals rt_render_to_target's."""
    from rt_amd import render

    monkeypatch.setenv("RT_DEBUG_FRAME_STAGING", "1")
    loaded = load_scene("triangles")
    one, many = [], []
    render.render_to_target(loaded, 6, 2, 0, update_hook=lambda t, d: one.append((d, t.copy())))
    render.render_to_target_devices(loaded, 6, 2, [0, 0, 0], update_hook=lambda t, d: many.append((d, t.copy())))
    assert [d for d, _ in one] == [d for d, _ in many] == [2, 4, 6]
    for (_, a), (_, b) in zip(one, many):
        assert np.array_equal(a, b)
