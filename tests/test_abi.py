"""The C-ABI library loads on CPU and exports every function include/rt_abi.h declares;
ctypes mirrors match the header's layout; host-side (no GPU) entry points behave."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def header_functions():
    src = open(os.path.join(ROOT, "include", "rt_abi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src))
    return {n for n in names if not n.startswith("rt_update_hook")}


def test_exports_every_declared_symbol(rtlib):
    from rt_amd import abi

    declared = header_functions()
    assert declared, "no functions parsed from rt_abi.h"
    assert declared == set(abi.EXPORTS), f"mirror drift: {declared ^ set(abi.EXPORTS)}"
    for name in declared:
        assert hasattr(rtlib, name), name


def test_struct_sizes_match_header():
    from rt_amd import abi

    # sizes fixed by rt_abi.h (16-byte friendly records, like assert_gpu_aligned gpu_structs.rs:18-22)
    assert C.sizeof(abi.rt_material) == 32
    assert C.sizeof(abi.rt_sphere) == 64
    assert C.sizeof(abi.rt_free_triangle) == 96
    assert C.sizeof(abi.rt_kd_node) == 8
    assert C.sizeof(abi.rt_tile) == 16


def test_version_and_status(rtlib):
    assert rtlib.rt_abi_version() == 1
    assert rtlib.rt_status_string(-6).decode().startswith("samps_per_pix")


def test_camera_conversion_identity(rtlib):
    from rt_amd import scheme

    cam = scheme.camera({"d": [0, 0, -5.0], "o": [0, -1, 0], "up": [0, 2, 0], "view_eulers": [0, 0, 0],
                         "screen_width": 10.0, "screen_height": 5.0})
    assert list(cam.d) == [0.0, 0.0, -5.0]
    assert list(cam.up) == [0.0, 1.0, 0.0]  # up normalised (builder/mod.rs:70)
    assert cam.has_lens == 0


def test_camera_conversion_rotation(rtlib):
    """cam.rs:66-74: R = from_euler_angles(r, p, y) = Rz(y) Ry(p) Rx(r)."""
    from rt_amd import scheme

    e = [-0.5, 1.4, 0.0]
    cam = scheme.camera({"d": [0, 0, 4], "o": [-30, 0, 0], "up": [0, 1, 0], "view_eulers": e,
                         "screen_width": 10.0, "screen_height": 5.0})
    r, p, y = e
    Rx = np.array([[1, 0, 0], [0, np.cos(r), -np.sin(r)], [0, np.sin(r), np.cos(r)]])
    Ry = np.array([[np.cos(p), 0, np.sin(p)], [0, 1, 0], [-np.sin(p), 0, np.cos(p)]])
    Rz = np.array([[np.cos(y), -np.sin(y), 0], [np.sin(y), np.cos(y), 0], [0, 0, 1]])
    R = Rz @ Ry @ Rx
    np.testing.assert_allclose(list(cam.d), R @ [0, 0, 4], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(list(cam.up), R @ [0, 1, 0], rtol=1e-6, atol=1e-6)


def test_rgba_to_u8_matches_rgb_f_to_u8(rtlib):
    from rt_amd import render

    vals = np.array([[0.0, 0.5, 1.0, 1.0], [-1.0, 2.0, np.nan, 1.0], [0.00196, 0.998, 0.5019608, 1.0]],
                    dtype=np.float32)
    out = render.rgba_to_u8(vals)
    f = np.clip(vals[:, :3], 0, 1) * np.float32(255) + np.float32(0.5)
    want = np.nan_to_num(np.trunc(f), nan=0).astype(np.uint8)
    assert np.array_equal(out[:, :3], want)
    assert np.all(out[:, 3] == 255)
    assert out[1].tolist() == [0, 255, 0, 255]  # NaN -> 0 (Rust `as u8`)


def test_render_to_target_rejects_bad_batch(rtlib, walled):
    from rt_amd import abi

    target = np.zeros((walled.info.height, walled.info.width, 4), np.uint8)
    st = rtlib.rt_render_to_target(C.byref(walled.desc), C.byref(walled.cam), C.byref(walled.info), 10, 3, 0,
                                   target.ctypes.data_as(C.POINTER(C.c_uint8)), None, None)
    assert st == abi.RT_ERR_BATCH  # renderer.rs:56-57 panics; the ABI returns a status


def test_create_without_device_fails_cleanly(rtlib, walled):
    """On a machine with no gfx950 the ABI reports RT_ERR_NO_DEVICE instead of falling back."""
    from rt_amd import abi

    n = C.c_int()
    assert rtlib.rt_device_count(C.byref(n)) == 0
    if n.value:
        pytest.skip("a gfx950 device is present")
    ctx = C.c_void_p()
    st = rtlib.rt_create(C.byref(walled.desc), C.byref(walled.cam), C.byref(walled.info), None, 0, C.byref(ctx))
    assert st == abi.RT_ERR_NO_DEVICE and not ctx.value


@pytest.mark.parametrize("before,after", [(None, "16"), ("4", "4"), ("12", "12"), ("junk", "junk")])
def test_hw_queues_set_only_when_unset(before, after):
    """Importing rt_amd sets GPU_MAX_HW_QUEUES to 16 when it is unset (the launch pipeline's
    streams each need a hardware queue) and keeps any explicit value: that is the
    caller's choice (bench.py makes its own, and reports it)."""
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("GPU_MAX_HW_QUEUES", None)
    if before is not None:
        env["GPU_MAX_HW_QUEUES"] = before
    code = ("import os, sys; sys.path.insert(0, %r); import rt_amd; print(os.environ['GPU_MAX_HW_QUEUES'])"
            % os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.strip() == after


def test_hw_queues_report():
    """rt_amd.hw_queues() says who set the value and whether HIP had already started."""
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("GPU_MAX_HW_QUEUES", None)
    code = ("import sys, json; sys.path.insert(0, %r); import rt_amd; print(json.dumps(rt_amd.hw_queues()))"
            % os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    import json
    r = json.loads(out.stdout)
    assert r == {"value": "16", "source": "rt_amd", "hip_started_before_import": False}


def test_hw_queues_untouched_after_hip_started():
    """With HIP already started (here a stand-in torch whose cuda.is_initialized() is True) the
    queues are fixed: rt_amd must not write GPU_MAX_HW_QUEUES, or the library would size its
    pipeline for 16 queues HIP never made.  It stays unset, the library then assumes
    HIP's default of 4, and hw_queues() says HIP had started."""
    import json
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("GPU_MAX_HW_QUEUES", None)
    code = ("import os, sys, types, json, warnings; warnings.simplefilter('ignore'); "
            "t = types.ModuleType('torch'); t.cuda = types.SimpleNamespace(is_initialized=lambda: True); "
            "sys.modules['torch'] = t; sys.path.insert(0, %r); import rt_amd; "
            "print(json.dumps([os.environ.get('GPU_MAX_HW_QUEUES'), rt_amd.hw_queues()]))"
            % os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    v, r = json.loads(out.stdout)
    assert v is None
    assert r == {"value": None, "source": None, "hip_started_before_import": True}


def test_committed_counters_belong_to_this_build():
    """bench.py prices each config's roofline with the committed rocprofv3 counters of the SAME
    device code (profiles/*_counters.json, keyed on the .hip_fatbin hash): every bench config's
    counters must carry the build id of the library this tree builds, or the round's bench line
    would report `null` fractions.  A kernel change therefore needs a re-profile
    (tools/gpu_profile_all.sh) before it is committed."""
    import glob
    import json
    import sys

    sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
    from rt_amd import abi

    bid = abi.kernel_build_id()
    found = {}
    for p in glob.glob(os.path.join(ROOT, "profiles", "*_counters.json")):
        d = json.load(open(p))
        if d.get("build_id") == bid:
            found.setdefault(d.get("scene"), set()).add(d.get("samples_per_launch"))
    # the bench's configs (bench.py CONFIGS and the walled headline) at their launch shapes: a
    # config's batches are traced in groups of up to bench.GROUP_ITEMS samples (a380: 10 batches of
    # 1 spp in one launch, biplane: 2 batches of 10 spp)
    want = {"walled": 720_000_000, "a380": 7_200_000, "biplane": 14_400_000, "spaceship_r1": 419_430_400,
            "triangles": 7_200_000}
    missing = {s: n for s, n in want.items() if n not in found.get(s, set())}
    assert not missing, f"no committed counters of build {bid} for {missing}: re-profile"
