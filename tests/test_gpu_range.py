"""rt_render_range: the mean over one sample range alone — what one batch of the reference's GPU
path returns (block_and_get_single_result, src/render/gpu_utils.rs:681-724; its kernel folds the
batch with a running mean from zero, src/render/trace.wgsl:277-318) before render_to_target_gpu
folds the batches (src/render/draw_scene.rs:36).  Checked against the oracle run over the same
range with the same mean origin, on every schedule the runtime has, and the context's cumulative
mean must be left alone."""
import numpy as np
import pytest

import parity
from conftest import load_scene

pytestmark = pytest.mark.gpu

WALLED_TILES = [(560, 260, 64, 32), (3, 5, 9, 7)]
N_WALLED = 64 * 32 + 9 * 7

CASES = [
    ("walled", WALLED_TILES, 10, 7, {}),
    ("walled", WALLED_TILES, 10, 7, {"RT_DEBUG_SCHED": "direct"}),                       # lanes per pixel + fold
    ("walled", WALLED_TILES, 10, 9, {"RT_DEBUG_LAUNCH": f"radiance_floats={3 * N_WALLED * 2}"}),  # 5 launches
    ("walled", WALLED_TILES, 0, 5, {}),                                              # range from sample 0
    ("biplane", [(600, 300, 32, 16)], 4, 5, {}),
    ("biplane", [(600, 300, 32, 16)], 4, 5, {"RT_DEBUG_LAUNCH": "overlap=2"}),
]


@pytest.mark.parametrize("name,tiles,s0,count,env", CASES,
                         ids=[f"{c[0]}-{c[2]}+{c[3]}-{'-'.join(c[4]) or 'default'}" for c in CASES])
def test_render_range_mean(gpu_available, oracle, monkeypatch, name, tiles, s0, count, env):
    from rt_amd import render

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sc = load_scene(name)
    with render.Context(sc) as c:
        if s0:
            c.render(tiles, 0, s0, want_output=False)  # cumulative [0, s0)
        rng = c.render_range(tiles, s0, count)         # [s0, s0 + count) alone
        again = c.render_range(tiles, s0, count)       # a range call keeps no state of its own
        after = c.render(tiles, s0, count)             # the cumulative mean continues untouched
    assert (rng[:, 3] == 1.0).all()
    o_rng = oracle.render(sc, tiles, s0, count, accum=oracle.ACCUM_FORWARD, mean_base=s0)
    assert np.array_equal(rng, o_rng), parity.stats(rng, o_rng)
    assert np.array_equal(again, rng)
    o_all = oracle.render(sc, tiles, 0, s0 + count, accum=oracle.ACCUM_FORWARD)
    assert np.array_equal(after, o_all), parity.stats(after, o_all)
    r = oracle.render(sc, tiles, s0, count, accum=oracle.ACCUM_RECURSIVE, mean_base=s0)
    parity.assert_reference_order(rng, r, f"{name} range [{s0}, {s0 + count})")


def test_batch_means_fold_to_the_frame_mean(gpu_available, walled):
    """render_to_target_gpu's fold of equal batches' means (draw_scene.rs:30-44) approximates the
    cumulative mean of the same samples: the two estimators agree to float rounding."""
    from rt_amd import render

    tiles = [(560, 260, 32, 16)]
    with render.Context(walled) as c:
        means = [c.render_range(tiles, b, 4) for b in range(0, 16, 4)]
        cum = c.render(tiles, 0, 16)
    acc = np.zeros_like(means[0])
    for i, m in enumerate(means):
        n = np.float32(i)
        acc[:, :3] = (m[:, :3] + acc[:, :3] * n) / (n + np.float32(1))
    assert np.allclose(acc[:, :3], cum[:, :3], rtol=1e-5, atol=1e-6)
