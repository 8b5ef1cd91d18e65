"""rt_render_batches_device_async and the batch groups of rt_render_to_target: consecutive batches
traced by one launch and folded batch by batch must give every batch's frame exactly as one call
per batch does — also when the radiance cap splits the batches over launches at batch boundaries
(whole batches per launch) or inside batches (a batch's fold in parts, across two launches)."""
import numpy as np
import pytest

import parity
from conftest import load_scene


def _per_batch_frames(sc, tiles, spp, batch):
    from rt_amd import render

    with render.Context(sc) as c:
        return [c.render(tiles, s0, batch) for s0 in range(0, spp, batch)]


@pytest.mark.gpu
@pytest.mark.parametrize("scene_name,spp,batch,cap", [
    ("biplane", 12, 1, None),   # one launch, 12 folds
    ("a380", 6, 1, None),
    ("walled", 12, 3, None),
    ("biplane", 12, 2, 5),      # launches of 2 whole batches (cap 5 samples)
    ("walled", 12, 4, 3),       # batches of 4 over launches of 3 samples: folds in parts
    ("triangles", 10, 5, 2),
])
def test_batches_equal_one_call_per_batch(gpu_available, monkeypatch, scene_name, spp, batch, cap):
    import torch

    from rt_amd import render

    sc = load_scene(scene_name)
    w, h = int(sc.info.width), int(sc.info.height)
    tiles = [(w // 2 - 40, h // 2 - 20, 80, 40), (3, 1, 17, 9)]
    n = 80 * 40 + 17 * 9
    ref = _per_batch_frames(sc, tiles, spp, batch)
    if cap:
        monkeypatch.setenv("RT_DEBUG_LAUNCH", f"radiance_floats={3 * n * cap}")
    nb = spp // batch
    with render.Context(sc) as c:
        outs = [torch.full((n, 4), -1.0, dtype=torch.float32, device="cuda:0") for _ in range(nb)]
        ptrs = [o.data_ptr() for o in outs]
        ptrs[1] = 0  # a batch whose frame is not wanted: the accumulator still advances
        stream = torch.cuda.current_stream().cuda_stream
        c.render_batches_device_async(ptrs, tiles, 0, batch, stream=stream)
        got = [o.cpu().numpy() for o in outs]  # ordered after the folds on torch's stream
        c.synchronize()
        st = c.launch_stats()
    want_launches = 1 if not cap else -(-spp // (cap // batch * batch if cap >= batch else cap))
    assert st["n_trace_launches"] == want_launches, st
    for k in range(nb):
        if k == 1:
            assert (got[k] == -1.0).all()
            continue
        assert np.array_equal(got[k], ref[k]), (k, parity.stats(got[k], ref[k]))


@pytest.mark.gpu
def test_render_to_target_groups_reuse_buffers(gpu_available, monkeypatch):
    """rt_render_to_target with batch groups of 3 (RT_DEBUG_LAUNCH group_items) and more batches than its
    ring of output buffers: every frame the hook sees, in order, equals the synchronous loop's."""
    from rt_amd import render

    sc = load_scene("biplane", width=160, height=96)
    # ring = 3 batches x 2 groups < 14 batches
    monkeypatch.setenv("RT_DEBUG_LAUNCH", f"group_items={3 * 160 * 96},slots=2")
    frames = []
    render.render_to_target(sc, 14, 1, update_hook=lambda t, done: frames.append((done, t.copy())))
    assert [d for d, _ in frames] == list(range(1, 15))
    ref = _per_batch_frames(sc, None, 14, 1)
    for i in range(14):
        assert np.array_equal(frames[i][1].reshape(-1, 4), render.rgba_to_u8(ref[i])), i
