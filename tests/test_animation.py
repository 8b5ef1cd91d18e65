"""Animation: renderer.rs:65-207 + builder/inner.rs:113-249 in the C++
host (rt_scheme_frames / rt_scheme_frame) and rt_render's frame loop.  The frame count, the
per-frame clock and the member replacement follow the reference's code; the keyframe crate's
easing arithmetic (keyframe 1.1.1, not vendored) is restated — parity unpinned for the
interpolated values between keyframes, pinned at keyframe times and for the ease endpoints."""
import copy
import json
import os

import numpy as np
import pytest

from conftest import ASSETS, SCENES
from test_host_cpp import assert_same, canonical


def _native(name):
    from rt_amd import scheme

    return scheme.NativeScheme(open(os.path.join(SCENES, name + ".json")).read(), ASSETS)


def test_frame_counts():
    # extract_anim: (last keyframe time / (1 / framerate)) as usize
    assert _native("bounce_anim").n_frames() == int(5.6 / (1.0 / 24.0)) == 134
    assert _native("biplane_anim").n_frames() == 180
    assert _native("walled").n_frames() == 0


def test_bounce_frames_at_keyframes_and_between():
    doc = json.load(open(os.path.join(SCENES, "bounce_anim.json")))
    n = _native("bounce_anim")
    sph = [m["!Sphere"] for m in doc["scene_members"] if "!Sphere" in m]
    anim_idx = next(i for i, s in enumerate(sph) if s.get("animation"))
    keys = sph[anim_idx]["animation"]["keyframes"]
    def c(f):
        fr = n.frame(f)  # keep the frame alive while its description is read
        return list(fr.desc.spheres[anim_idx].c)

    assert c(0) == [float(np.float32(v)) for v in keys[0]["translation"]]
    assert c(24) == [float(np.float32(v)) for v in keys[1]["translation"]]  # t = 1 s, keyframe 1
    # frame 12 (t = 0.5): EaseInQuad from 5 to -10 at progress 0.5 -> 5 - 15 * 0.25
    assert c(12)[1] == pytest.approx(1.25, abs=1e-5)
    ys = [c(f)[1] for f in range(0, 25)]
    assert all(a >= b for a, b in zip(ys, ys[1:]))  # monotone between two keyframes


def _python_scheme_with(doc, name, updates):
    from rt_amd import scheme

    d = copy.deepcopy(doc)
    for idx, fields in updates.items():
        (tag, m), = d["scene_members"][idx].items()
        m.update(fields)
    return scheme.load(d, assets_root=ASSETS)


@pytest.mark.parametrize("name,frame", [("bounce_anim", 7), ("biplane_anim", 95)])
def test_frame_is_the_still_scheme_with_moved_members(name, frame):
    """A frame's description equals the Python host's description of the same scheme with the
    animated members' c / translation / euler_angles set to the frame's values."""
    doc = json.load(open(os.path.join(SCENES, name + ".json")))
    fr = _native(name).frame(frame)
    updates = {}
    sph_i = 0
    for mi, m in enumerate(doc["scene_members"]):
        (tag, v), = m.items()
        if tag == "!Sphere":
            if v.get("animation"):
                updates[mi] = {"c": [float(x) for x in fr.desc.spheres[sph_i].c]}
            sph_i += 1
    if name == "biplane_anim":
        # the model's translation / euler angles at this frame, restated independently here
        m = doc["scene_members"][0]["!Model"]
        keys = m["animation"]["keyframes"]
        ease = {"EaseInOutQuad": lambda x: 2 * x * x if x < 0.5 else -2 * x * x + 4 * x - 1,
                "EaseInCubic": lambda x: x * x * x}
        tpf = 1.0 / float(np.float32(doc["render_info"]["framerate"]))
        dur = float(np.float32(keys[-1]["time"]))
        clock = 0.0
        for _ in range(frame):
            clock = min(clock + tpf, dur)
        k = max(i for i, kf in enumerate(keys) if float(np.float32(kf["time"])) <= clock)
        a, b = keys[k], keys[k + 1]
        ta, tb = float(np.float32(a["time"])), float(np.float32(b["time"]))
        y = ease[a["ease_type"]](min(max((clock - ta) / (tb - ta), 0.0), 1.0))
        lerp = lambda u, v: [float(np.float32(float(np.float32(p)) + (float(np.float32(q)) - float(np.float32(p))) * y))  # noqa: E731
                             for p, q in zip(u, v)]
        updates[0] = {"translation": lerp(a["translation"], b["translation"]),
                      "euler_angles": lerp(a["euler_angles"], b["euler_angles"])}
    py = _python_scheme_with(doc, name, updates)
    got = canonical(fr.desc, fr.cam, fr.info)
    want = canonical(py.desc, py.cam, py.info)
    assert_same(got, want)


def test_unknown_ease_type_is_rejected():
    from rt_amd import abi, scheme

    doc = json.load(open(os.path.join(SCENES, "bounce_anim.json")))
    for m in doc["scene_members"]:
        (tag, v), = m.items()
        if tag == "!Sphere" and v.get("animation"):
            v["animation"]["keyframes"][0]["ease_type"] = "Wobble"
    with pytest.raises(abi.RtError):
        scheme.NativeScheme(json.dumps(doc), ASSETS).frame(0)


@pytest.mark.gpu
def test_rt_render_animation_frames(gpu_available, tmp_path):
    """rt_render on an animated scheme: anim_frames/<n>.png for n = 1.. (renderer.rs:162), each
    the frame's scene rendered as a still; --frames r/N shards frames over processes."""
    import subprocess

    from rt_amd import render
    from test_host_cpp import RT_RENDER, read_png_rgba

    d = str(tmp_path / "frames")
    args = [RT_RENDER, os.path.join(SCENES, "bounce_anim.json"), "--assets", ASSETS, "--frames-dir", d,
            "--width", "48", "--height", "96", "--spp", "2", "--batch", "1", "--max-frames", "3"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert sorted(os.listdir(d)) == ["1.png", "2.png", "3.png"]
    fr = _native("bounce_anim").frame(1)
    fr.info.width, fr.info.height = 48, 96
    want = render.render_to_target(fr, 2, 1)
    assert np.array_equal(read_png_rgba(os.path.join(d, "2.png")), want[::-1])
    d2 = str(tmp_path / "odd")
    r = subprocess.run(args[:5] + [d2] + args[6:] + ["--frames", "1/2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert sorted(os.listdir(d2)) == ["2.png"]


@pytest.mark.gpu
@pytest.mark.parametrize("frame", [0, 37, 133])
def test_bounce_frame_against_oracle(gpu_available, oracle, frame):
    """An animation frame (bounce_anim.yml: frame 0, frame 37 between keyframes, the last frame)
    rendered on the device equals the forward oracle run on that frame's own scene description,
    bit for bit, and is within the stated gate of the reference's recursive order
    (renderer.rs:65-207 renders each frame as a still through the same path)."""
    import parity
    from rt_amd import render

    fr = _native("bounce_anim").frame(frame)
    fr.info.width, fr.info.height = 150, 300
    tiles = [(0, 0, 150, 300)]
    with render.Context(fr) as c:
        g = c.render(tiles, 0, 4)
    o = oracle.render(fr, tiles, 0, 4, accum=oracle.ACCUM_FORWARD)
    assert np.array_equal(g, o), parity.stats(g, o)
    assert g[:, :3].max() > 0
    r = oracle.render(fr, tiles, 0, 4, accum=oracle.ACCUM_RECURSIVE)
    parity.assert_reference_order(g, r, f"bounce_anim frame {frame}")
