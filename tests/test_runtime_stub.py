"""The runtime's host logic on the CPU, against a stand-in HIP runtime (tests/stub_hip: one fake
gfx950, host memory, kernel launches counted and not run), LD_PRELOADed into a child process.

The launch pipeline asks whether the previous fold is still running (hipEventQuery) before a
small launch, to size its share of the grid.  A query that fails — a faulted earlier launch —
must end the call with RT_ERR_HIP and the query's message, not be read as "not busy" and
cleared; a not-ready query is no error."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

HIP_NOT_READY, HIP_LAUNCH_FAILURE = 600, 719

CHILD = r"""
import ctypes as C, json, os, sys
sys.path.insert(0, os.path.join(%(root)r, "gpu-ray_trace-rust_amd"))
from rt_amd import abi, scheme
stub = C.CDLL(%(stub)r)  # the preloaded object: same handle
lib = abi.load_library()
loaded = scheme.load(scheme.load_json(os.path.join(%(root)r, "tests", "golden", "scenes", "walled.json")), lib=lib)
ctx = C.c_void_p()
res = {"create": lib.rt_create(C.byref(loaded.desc), C.byref(loaded.cam), C.byref(loaded.info), None, 0, C.byref(ctx))}
tile = abi.rt_tile(0, 0, 64, 8)
out = (C.c_float * (4 * 64 * 8))()
calls = []
for q in %(queries)r:
    stub.stub_hip_set_query(q)
    before = stub.stub_hip_launches()
    st = lib.rt_render_device_async(ctx, C.byref(tile), 1, len(calls), 1, C.cast(out, C.POINTER(C.c_float)), None)
    calls.append({"query": q, "status": st, "launches": stub.stub_hip_launches() - before,
                  "error": lib.rt_last_error(ctx).decode()})
res["calls"] = calls
res["destroy"] = lib.rt_destroy(ctx)
print("RESULT", json.dumps(res))
"""


@pytest.fixture(scope="module")
def stub_lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("stub_hip")
    out = str(d / "libstub_hip.so")
    src = os.path.join(ROOT, "tests", "stub_hip")
    cmd = ["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           f"-Wl,--version-script={src}/stub_hip.map", "-o", out, f"{src}/stub_hip.cpp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        pytest.skip("cannot build the stub HIP runtime here: " + r.stderr[-300:])
    return out


def run_child(stub, queries):
    env = dict(os.environ, LD_PRELOAD=stub, RT_DEBUG_LAUNCH="slots=4")
    code = CHILD % {"root": ROOT, "stub": stub, "queries": queries}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(line[0][7:])


def test_failed_fold_query_is_reported(stub_lib):
    """Calls 1-2: the previous fold is still running (not ready): both enqueue a trace and a fold.
    Call 3: the query fails: RT_ERR_HIP, nothing launched, rt_last_error names the query.  Call
    4: the query succeeds again: the context is still usable."""
    r = run_child(stub_lib, [HIP_NOT_READY, HIP_NOT_READY, HIP_LAUNCH_FAILURE, 0])
    assert r["create"] == 0, r
    c = r["calls"]
    assert [x["status"] for x in c[:2]] == [0, 0], c
    assert all(x["launches"] == 2 for x in c[:2]), c  # trace + fold
    assert c[2]["status"] == -3, c  # RT_ERR_HIP
    assert c[2]["launches"] == 0, c
    assert "hipEventQuery" in c[2]["error"] and "launch failure" in c[2]["error"], c
    assert c[3]["status"] == 0 and c[3]["launches"] == 2, c
    assert r["destroy"] == 0


CHILD_BATCHES = r"""
import ctypes as C, json, os, sys
sys.path.insert(0, os.path.join(%(root)r, "gpu-ray_trace-rust_amd"))
from rt_amd import abi, scheme
stub = C.CDLL(%(stub)r)
lib = abi.load_library()
loaded = scheme.load(scheme.load_json(os.path.join(%(root)r, "tests", "golden", "scenes", "walled.json")), lib=lib)
def log(since):
    buf = (C.c_int * 4096)()
    n = stub.stub_hip_launch_log(buf, 4096)
    return list(buf[since:n])
res = {}
# the device batch loop: 10 batches of 1 spp over the 1200 x 600 frame
ctx = C.c_void_p()
assert lib.rt_create(C.byref(loaded.desc), C.byref(loaded.cam), C.byref(loaded.info), None, 0, C.byref(ctx)) == 0
tile = abi.rt_tile(0, 0, int(loaded.info.width), int(loaded.info.height))
n0 = stub.stub_hip_launches()
outs = (C.c_void_p * 10)(*[C.c_void_p(0x1000 * (k + 1)) for k in range(10)])
res["batches"] = lib.rt_render_batches_device_async(ctx, C.byref(tile), 1, 0, 1, 10, outs, None)
res["batches_log"] = log(n0)
n0 = stub.stub_hip_launches()
res["zero"] = lib.rt_render_batches_device_async(ctx, C.byref(tile), 1, 10, 1, 0, outs, None)
res["zero_log"] = log(n0)
lib.rt_destroy(ctx)
# render_to_target_gpu: 12 spp in batches of 1 -> one group, hook after every batch in order
seen = []
HOOK = C.CFUNCTYPE(None, C.c_void_p, C.c_uint32)
hook = HOOK(lambda user, done: seen.append(int(done)))
target = (C.c_uint8 * (4 * int(loaded.info.width) * int(loaded.info.height)))()
n0 = stub.stub_hip_launches()
res["target"] = lib.rt_render_to_target(C.byref(loaded.desc), C.byref(loaded.cam), C.byref(loaded.info), 12, 1, 0,
                                        target, C.cast(hook, C.c_void_p), None)
res["target_log"] = log(n0)
res["hook"] = seen
print("RESULT", json.dumps(res))
"""


def test_batches_trace_once_and_fold_per_batch(stub_lib):
    """rt_render_batches_device_async: 10 batches of 1 spp (0.72 M samples each) are one trace
    launch (block 128) and ten folds (block 256), in that order; zero batches launch nothing.
    rt_render_to_target at 12 spp in batches of 1 traces them as one group (the frames of every
    batch still come out, in order: the hook sees 1, 2, ..., 12)."""
    env = dict(os.environ, LD_PRELOAD=stub_lib)
    code = CHILD_BATCHES % {"root": ROOT, "stub": stub_lib}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(line[0][7:])
    assert res["batches"] == 0 and res["batches_log"] == [128] + [256] * 10, res
    assert res["zero"] == 0 and res["zero_log"] == [], res
    assert res["target"] == 0, res
    assert res["target_log"] == [128] + [256] * 12, res
    assert res["hook"] == list(range(1, 13)), res


CHILD_SLOTS = r"""
import ctypes as C, json, os, sys
sys.path.insert(0, os.path.join(%(root)r, "gpu-ray_trace-rust_amd"))
from rt_amd import abi, scheme
stub = C.CDLL(%(stub)r)
lib = abi.load_library()
assets = os.path.join(%(root)r, "assets_pack")
loaded = scheme.load(scheme.load_json(os.path.join(%(root)r, "tests", "golden", "scenes", %(scene)r)),
                     assets_root=assets if os.path.isdir(assets) else None, lib=lib)
ctx = C.c_void_p()
assert lib.rt_create(C.byref(loaded.desc), C.byref(loaded.cam), C.byref(loaded.info), None, 0, C.byref(ctx)) == 0
w, h = int(loaded.info.width), int(loaded.info.height)
out = C.c_void_p(0x1000)  # never written: the stub runs no kernel
res = {}
begin = 0
for name, tw, th, spp, calls in %(cases)r:
    stub.stub_hip_set_query(600)  # hipErrorNotReady: every earlier fold still running
    tile = abi.rt_tile(0, 0, min(tw, w), min(th, h))
    n0 = stub.stub_hip_launches()
    st = [lib.rt_render_device_async(ctx, C.byref(tile), 1, begin + k * spp, spp, C.cast(out, C.POINTER(C.c_float)), None)
          for k in range(calls)]
    begin += calls * spp
    blk = (C.c_int * 4096)(); strm = (C.c_int * 4096)(); grid = (C.c_int * 4096)()
    n = stub.stub_hip_launch_log(blk, 4096)
    stub.stub_hip_launch_detail(strm, grid, 4096)
    traces = [(strm[i], grid[i]) for i in range(n0, n) if blk[i] == 128]
    res[name] = {"status": st, "items": tile.w * tile.h * spp, "streams": [s for s, _ in traces],
                 "grids": [g for _, g in traces]}
lib.rt_destroy(ctx)
print("RESULT", json.dumps(res))
"""


def run_slots(stub, scene, queues, cases):
    env = dict(os.environ, LD_PRELOAD=stub, GPU_MAX_HW_QUEUES=str(queues))
    for k in ("RT_DEBUG_LAUNCH",):
        env.pop(k, None)
    code = CHILD_SLOTS % {"root": ROOT, "stub": stub, "scene": scene, "cases": cases}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(line[0][7:])


def rotation(streams):
    """The number of distinct streams, and that the launches cycle through them in a fixed order."""
    k = len(set(streams))
    assert all(streams[i] == streams[i + k] for i in range(len(streams) - k)), streams
    return k


# the stub's device: 256 CUs x 16 resident workgroups = a full grid of 4096
FULL_GRID = 4096


@pytest.mark.parametrize("queues,small,mid,small_grid", [(16, 12, 6, FULL_GRID // 8), (12, 8, 4, FULL_GRID // 4),
                                                          (4, 2, 2, FULL_GRID), (32, 12, 6, FULL_GRID // 8)])
def test_pipeline_slots_follow_launch_size(stub_lib, queues, small, mid, small_grid):
    """The round-4 slot rules (runtime.hip slots_for_queues / mid_slots_for / small_grid_div) on
    the sphere-only scene: with GPU_MAX_HW_QUEUES = q, launches of at most 2^21 samples rotate
    over min(12, q - 4) streams and, behind a busy pipeline, take 1/8 (12 slots) or 1/4 (8 slots)
    of the grid; launches of 2^21 .. 2^23 over half that many (2 .. 6) with the full grid; larger
    ones over 2.  The first launch of a context (nothing in flight) keeps the full grid."""
    r = run_slots(stub_lib, "walled.json", queues,
                  [("small", 64, 8, 1, 30), ("mid", 1200, 600, 6, 14), ("large", 1200, 600, 16, 6)])
    for name in ("small", "mid", "large"):
        assert all(s == 0 for s in r[name]["status"]), r[name]
        assert len(r[name]["streams"]) == len(r[name]["status"]), r[name]
    assert r["small"]["items"] <= 1 << 21 < r["mid"]["items"] <= 1 << 23 < r["large"]["items"]
    assert rotation(r["small"]["streams"]) == small
    assert r["small"]["grids"][0] == FULL_GRID and set(r["small"]["grids"][1:]) == {small_grid}, r["small"]["grids"]
    assert rotation(r["mid"]["streams"]) == mid
    assert set(r["mid"]["grids"]) == {FULL_GRID}
    assert rotation(r["large"]["streams"]) == 2
    assert set(r["large"]["grids"]) == {FULL_GRID}
    # the slots are one set: the mid and large launches reuse the small launches' first streams
    assert set(r["mid"]["streams"]) <= set(r["small"]["streams"]) or small < mid


@pytest.mark.parametrize("queues,slots,grid", [(16, 6, FULL_GRID // 2), (4, 2, FULL_GRID)])
def test_tiny_scene_pipeline(stub_lib, queues, slots, grid):
    """A tiny scene (triangles.json: 6 primitives, 8 item-counter shards) runs launches of up to
    2^24 samples as small ones, over the mid-size slot count with half the grid when that is >= 4
    slots (round 4: triangles at 16 queues 16,700 -> 17,100 Msamples/s)."""
    r = run_slots(stub_lib, "triangles.json", queues, [("frames", 1200, 600, 10, 3 * slots)])
    f = r["frames"]
    assert all(s == 0 for s in f["status"]), f
    assert 1 << 21 < f["items"] <= 1 << 24
    assert rotation(f["streams"]) == slots
    assert f["grids"][0] == FULL_GRID and set(f["grids"][1:]) == {grid}, f["grids"]
