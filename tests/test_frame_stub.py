"""The multi-device frame of the C ABI (frame.hip) on the CPU, against the stand-in
HIP runtime (tests/stub_hip, several fake gfx950 devices, copies really made in host memory and
logged with their shapes, kernel launches logged with their device and not run).

Pins the stripe deal (each context's launches on its own device), that a frame is gathered ONCE
(one peer copy per context on another device, one strided placement per context on the first
device, one read-back), the placement's pitches (context k's j-th stripe is frame stripe
j * n + k), a shorter last stripe, and that rt_render_to_target_devices gathers once per batch
and calls the hook after every batch in order."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT
from test_runtime_stub import stub_lib  # noqa: F401  (the module fixture building the stub)

CHILD = r"""
import ctypes as C, json, os, sys
sys.path.insert(0, os.path.join(%(root)r, "gpu-ray_trace-rust_amd"))
from rt_amd import abi, scheme
stub = C.CDLL(%(stub)r)
stub.stub_hip_set_devices(%(ndev)d)
lib = abi.load_library()
loaded = scheme.load(scheme.load_json(os.path.join(%(root)r, "tests", "golden", "scenes", "walled.json")), lib=lib)
if %(height)d:
    loaded.info.height = %(height)d
def launches(since):
    blk = (C.c_int * 4096)(); dev = (C.c_int * 4096)()
    n = stub.stub_hip_launch_log(blk, 4096)
    stub.stub_hip_launch_devices(dev, 4096)
    return [(blk[i], dev[i]) for i in range(since, n)]
def copies(since):
    buf = (C.c_longlong * (6 * 4096))()
    n = stub.stub_hip_copy_log(buf, 4096)
    return [list(buf[6 * i: 6 * i + 6]) for i in range(since, n)]
def ncopies():
    buf = (C.c_longlong * (6 * 4096))()
    return stub.stub_hip_copy_log(buf, 4096)
res = {}
devs = %(devices)r
f = C.c_void_p()
arr = (C.c_int * len(devs))(*devs)
res["create"] = lib.rt_frame_create(C.byref(loaded.desc), C.byref(loaded.cam), C.byref(loaded.info), None, arr,
                                    len(devs), %(stripe)d, C.byref(f))
if res["create"] == 0:
    res["parts"] = []
    for k in range(len(devs)):
        d, ctx, nt = C.c_int(), C.c_void_p(), C.c_uint32()
        lib.rt_frame_part(f, k, C.byref(d), C.byref(ctx), C.byref(nt))
        res["parts"].append([d.value, nt.value])
    n0, c0 = stub.stub_hip_launches(), ncopies()
    res["render"] = [lib.rt_frame_render(f, 0, 2), lib.rt_frame_render(f, 2, 2)]
    res["render_launches"] = launches(n0)
    res["render_copies"] = copies(c0)
    w, h = int(loaded.info.width), int(loaded.info.height)
    out = (C.c_float * (4 * w * h))()
    n0, c0 = stub.stub_hip_launches(), ncopies()
    res["gather"] = lib.rt_frame_gather(f, out, None)
    res["gather_launches"] = launches(n0)
    res["gather_copies"] = copies(c0)
    s = abi.rt_frame_stats()
    res["stats_status"] = lib.rt_frame_get_stats(f, C.byref(s))
    res["stats"] = {k: getattr(s, k) for k, _ in abi.rt_frame_stats._fields_}
    res["destroy"] = lib.rt_frame_destroy(f)
seen = []
HOOK = C.CFUNCTYPE(None, C.c_void_p, C.c_uint32)
hook = HOOK(lambda user, done: seen.append(int(done)))
w, h = int(loaded.info.width), int(loaded.info.height)
target = (C.c_uint8 * (4 * w * h))()
c0 = ncopies()
res["target"] = lib.rt_render_to_target_devices(C.byref(loaded.desc), C.byref(loaded.cam), C.byref(loaded.info), 12, 3,
                                                arr, len(devs), target, C.cast(hook, C.c_void_p), None)
res["target_copies"] = copies(c0)
res["hook"] = seen
print("RESULT", json.dumps(res))
"""

PEER, STRIDED, LINEAR = 1, 2, 3
ROW = 1200 * 16  # bytes per RGBA f32 row of the 1200-wide walled frame


def run(stub, devices, ndev, stripe=0, height=0, staging=False):
    env = dict(os.environ, LD_PRELOAD=stub)
    env.pop("RT_DEBUG_FRAME_STAGING", None)
    if staging:
        env["RT_DEBUG_FRAME_STAGING"] = "1"
    code = CHILD % {"root": ROOT, "stub": stub, "devices": devices, "ndev": ndev, "stripe": stripe, "height": height}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(line[0][7:])


def test_four_devices_one_gather(stub_lib):  # noqa: F811
    """Four contexts on four devices, walled 1200 x 600: stripes of 6 rows (600 = 25 x 6 x 4), every
    context's trace + fold launches on its own device, and after two render calls ONE gather: three
    peer copies (devices 1-3, 150 rows each), four strided placements (25 stripes of 6 rows each,
    destination pitch 4 stripes), one read-back of the 1200 x 600 frame."""
    r = run(stub_lib, [0, 1, 2, 3], 4)
    assert r["create"] == 0, r
    assert r["parts"] == [[0, 25], [1, 25], [2, 25], [3, 25]], r["parts"]
    assert r["render"] == [0, 0]
    # two calls x four contexts x (trace 128, fold 256), each on its context's device
    by_dev = {}
    for blk, dev in r["render_launches"]:
        by_dev.setdefault(dev, []).append(blk)
    assert by_dev == {d: [128, 256, 128, 256] for d in range(4)}, r["render_launches"]
    assert r["render_copies"] == []  # no gather while rendering
    assert r["gather"] == 0 and r["gather_launches"] == []
    g = r["gather_copies"]
    peers = [c for c in g if c[0] == PEER]
    assert [(c[1], c[2]) for c in peers] == [(1, 150 * ROW), (2, 150 * ROW), (3, 150 * ROW)], peers
    placed = [c for c in g if c[0] == STRIDED]
    assert placed == [[STRIDED, 0, 6 * ROW, 25, 4 * 6 * ROW, 6 * ROW]] * 4, placed
    assert [c for c in g if c[0] == LINEAR] == [[LINEAR, 0, 600 * ROW, 1, 0, 0]]  # the read-back
    assert [c[0] for c in g] == [PEER] * 3 + [STRIDED] * 4 + [LINEAR]  # copies before placement
    s = r["stats"]
    assert r["stats_status"] == 0 and s["n_gathers"] == 1 and s["n_peer_copies"] == 3, s
    assert s["n_parts"] == 4 and s["stripe_rows"] == 6
    assert r["destroy"] == 0


def test_shorter_last_stripe(stub_lib):  # noqa: F811
    """Stripes of 7 rows over 600 rows and 3 contexts: 85 full stripes and one of 5 rows, the last,
    which is context 85 % 3 = 1's: it is placed by one linear copy after its strided copy."""
    r = run(stub_lib, [0, 0, 0], 1, stripe=7)
    assert r["create"] == 0, r
    g = r["gather_copies"]
    assert [c for c in g if c[0] == PEER] == []  # one device: no peer copies
    placed = [c for c in g if c[0] in (STRIDED, LINEAR)]
    full = [len(range(k, 85, 3)) for k in range(3)]  # 29, 28, 28 full stripes
    assert placed[:2] == [[STRIDED, 0, 7 * ROW, full[0], 3 * 7 * ROW, 7 * ROW],
                          [STRIDED, 0, 7 * ROW, full[1], 3 * 7 * ROW, 7 * ROW]], placed
    assert placed[2] == [LINEAR, 0, 5 * ROW, 1, 0, 0], placed  # context 1's last, 5-row stripe
    assert placed[3] == [STRIDED, 0, 7 * ROW, full[2], 3 * 7 * ROW, 7 * ROW], placed
    assert placed[4] == [LINEAR, 0, 600 * ROW, 1, 0, 0]  # the read-back
    assert r["stats"]["n_gathers"] == 1 and r["stats"]["n_peer_copies"] == 0


def test_render_to_target_devices_gathers_per_batch(stub_lib):  # noqa: F811
    """12 spp in batches of 3 over contexts on devices 0 and 1: four batches, one gather each (one
    peer copy, two placements, one read-back), the hook after every batch in order."""
    r = run(stub_lib, [0, 1], 2)
    assert r["target"] == 0, r
    assert r["hook"] == [3, 6, 9, 12]
    kinds = [c[0] for c in r["target_copies"]]
    assert kinds.count(PEER) == 4 and kinds.count(STRIDED) == 8, kinds
    assert [c for c in r["target_copies"] if c[0] == LINEAR and c[2] == 600 * ROW].__len__() == 4


def test_forced_staging_on_one_device(stub_lib):  # noqa: F811
    """RT_DEBUG_FRAME_STAGING=1 with four contexts on ONE device: contexts 1-3 are gathered through
    the remote branch (a peer copy device 0 -> device 0 into a staging buffer each, before the
    placements), exactly the copies of four contexts on four devices; without the knob the same
    contexts make no peer copy."""
    r = run(stub_lib, [0, 0, 0, 0], 1, staging=True)
    assert r["create"] == 0, r
    g = r["gather_copies"]
    peers = [c for c in g if c[0] == PEER]
    assert [(c[1], c[2]) for c in peers] == [(0, 150 * ROW)] * 3, peers
    assert [c[0] for c in g] == [PEER] * 3 + [STRIDED] * 4 + [LINEAR]
    assert r["stats"]["n_peer_copies"] == 3 and r["stats"]["n_gathers"] == 1
    kinds = [c[0] for c in r["target_copies"]]  # rt_render_to_target_devices: 4 batches
    assert kinds.count(PEER) == 12 and kinds.count(STRIDED) == 16, kinds
    r0 = run(stub_lib, [0, 0, 0, 0], 1)
    assert [c for c in r0["gather_copies"] if c[0] == PEER] == []


def test_bad_arguments(stub_lib):  # noqa: F811
    """A device ordinal past the devices present is RT_ERR_NO_DEVICE, and nothing leaks."""
    r = run(stub_lib, [0, 5], 2)
    assert r["create"] == -5, r


@pytest.mark.parametrize("height,world", [(600, 1), (600, 2), (600, 7), (600, 8), (4096, 8), (37, 5), (5, 5)])
def test_stripe_deal_matches_python(rtlib, height, world):
    """rt_stripe_rows / rt_stripe_tiles (the library's deal) equal rt_amd.shard's (bench.py's)."""
    from rt_amd import render, shard

    assert rtlib.rt_stripe_rows(height, world) == shard.stripe_rows(height, world)
    for k in range(world):
        assert render.stripe_tiles(1200, height, k, world, lib=rtlib) == shard.rank_tiles(1200, height, k, world)
