"""The C++ host above the boundary (rt_scheme_load: YAML / JSON scheme, glTF, asset packs;
rt_write_png) against the Python host (rt_amd/scheme.py, rt_amd/gltf.py): the same scheme
must give bit-identical rt_scene_desc / rt_camera / rt_render_info contents.  CPU only."""
import ctypes as C
import glob
import json
import os
import zlib

import numpy as np
import pytest

from conftest import ASSETS, ROOT, SCENES, load_scene

REF_SCHEMES = "/root/reference/schemes"
SCENE_NAMES = ["walled", "triangles", "biplane", "spaceship_r1", "a380"]


def _raw(struct):
    return bytes(memoryview(struct).cast("B"))


def _f32(ptr, n):
    return np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n and ptr else np.zeros(0, np.float32)


def canonical(desc, cam, info):
    """Every value an rt_scene_desc reaches, as comparable Python / numpy objects."""
    out = {"elems": [(desc.elems[i].kind, desc.elems[i].index) for i in range(desc.n_elems)],
           "spheres": [_raw(desc.spheres[i]) for i in range(desc.n_spheres)],
           "free_tris": [_raw(desc.free_tris[i]) for i in range(desc.n_free_tris)],
           "cube_maps": [_raw(desc.cube_maps[i]) for i in range(desc.n_cube_maps)],
           "cam": _raw(cam), "info": _raw(info), "textures": [], "meshes": []}
    for i in range(desc.n_textures):
        t = desc.textures[i]
        out["textures"].append((t.width, t.height, _f32(t.rgb, 3 * t.width * t.height)))
    for m in range(desc.n_meshes):
        mesh = desc.meshes[m]
        prims = []
        for p in range(mesh.n_prims):
            pr = mesh.prims[p]
            nv, nt = pr.n_verts, pr.n_tris
            prims.append({
                "n": (nv, nt), "poses": _f32(pr.poses, 3 * nv), "norms": _f32(pr.norms, 3 * nv),
                "indices": np.ctypeslib.as_array(pr.indices, shape=(3 * nt,)).copy(),
                "tangents": _f32(pr.tangents, 3 * nv), "bcf": list(pr.base_color_factor),
                "tex": (pr.base_color_tex, pr.normal_tex, pr.metal_rough_tex),
                "uv": [_f32(pr.base_color_uv, 2 * nv), _f32(pr.normal_uv, 2 * nv), _f32(pr.metal_rough_uv, 2 * nv)],
                "scalars": np.array([pr.normal_scale, pr.metal, pr.rough], np.float32)})
        out["meshes"].append((np.array(list(mesh.trans_mat), np.float32), prims))
    return out


def assert_same(a, b, path="desc"):
    if isinstance(a, np.ndarray):
        assert a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8)), path
    elif isinstance(a, dict):
        assert a.keys() == b.keys(), path
        for k in a:
            assert_same(a[k], b[k], f"{path}.{k}")
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            assert_same(x, y, f"{path}[{i}]")
    else:
        assert a == b, path


@pytest.mark.parametrize("name", SCENE_NAMES)
def test_cpp_json_load_equals_python(name):
    from rt_amd import scheme

    py = load_scene(name)
    cpp = scheme.NativeScheme(open(os.path.join(SCENES, name + ".json")).read(), ASSETS)
    assert_same(canonical(cpp.desc, cpp.cam, cpp.info), canonical(py.desc, py.cam, py.info))
    assert cpp.spp == py.spp and cpp.batch == py.batch


def _yaml_text(obj):
    """This repo's JSON scheme form written back as YAML with local tags."""
    import yaml

    class Tagged:
        def __init__(self, tag, value):
            self.tag, self.value = tag, value

    def conv(v):
        if isinstance(v, dict) and len(v) == 1 and next(iter(v)).startswith("!"):
            (k, val), = v.items()
            return Tagged(k, conv(val))
        if isinstance(v, dict):
            return {k: conv(x) for k, x in v.items()}
        if isinstance(v, list):
            return [conv(x) for x in v]
        return v

    class Dumper(yaml.SafeDumper):
        pass

    def rep(dumper, t):
        if isinstance(t.value, dict):
            return dumper.represent_mapping(t.tag, t.value)
        if isinstance(t.value, list):
            return dumper.represent_sequence(t.tag, t.value, flow_style=True)
        return dumper.represent_scalar(t.tag, "" if t.value is None else str(t.value))

    Dumper.add_representer(Tagged, rep)
    return yaml.dump(conv(obj), Dumper=Dumper, default_flow_style=False, sort_keys=False)


@pytest.mark.parametrize("name", ["walled", "triangles", "spaceship_r1"])
def test_cpp_yaml_load_equals_json_load(name):
    from rt_amd import scheme

    doc = json.load(open(os.path.join(SCENES, name + ".json")))
    a = scheme.NativeScheme(json.dumps(doc), ASSETS)
    b = scheme.NativeScheme(_yaml_text(doc), ASSETS)
    assert_same(canonical(a.desc, a.cam, a.info), canonical(b.desc, b.cam, b.info))


def _norm(v):
    if isinstance(v, dict):
        return {k: _norm(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if isinstance(v, bool):
        return str(v).lower()
    if v is None:
        return None
    s = str(v)
    try:
        return float(s)
    except ValueError:
        return s


def _cpp_doc(rtlib, text, fmt=0):
    fn = rtlib.rtx_doc_to_json
    fn.restype = C.c_longlong
    fn.argtypes = [C.c_char_p, C.c_ulonglong, C.c_uint, C.c_char_p, C.c_ulonglong]
    raw = text.encode()
    n = fn(raw, len(raw), fmt, None, 0)
    assert n >= 0, "C++ parser rejected the document"
    buf = C.create_string_buffer(n)
    fn(raw, len(raw), fmt, buf, n)
    return json.loads(buf.raw[:n].decode())


@pytest.mark.skipif(not os.path.isdir(REF_SCHEMES), reason="reference schemes are only in the build container")
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(REF_SCHEMES, "*.yml"))))
def test_cpp_yaml_parser_matches_pyyaml_on_reference_schemes(rtlib, path):
    from rt_amd import scheme

    text = open(path).read()
    assert _norm(_cpp_doc(rtlib, text)) == _norm(scheme.from_yml(text))


def test_write_png_roundtrip(rtlib, tmp_path):
    from rt_amd import abi

    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (5, 7, 4), dtype=np.uint8)
    p = str(tmp_path / "o.png")
    abi.check(rtlib, rtlib.rt_write_png(p.encode(), img.ctypes.data_as(C.POINTER(C.c_uint8)), 7, 5, 1))
    raw = open(p, "rb").read()
    assert raw[:8] == b"\x89PNG\r\n\x1a\n"
    # decode the single IDAT by hand: filter byte 0 + RGBA rows, flipped
    i, data = 8, b""
    while i < len(raw):
        n = int.from_bytes(raw[i:i + 4], "big")
        if raw[i + 4:i + 8] == b"IDAT":
            data += raw[i + 8:i + 8 + n]
        i += 12 + n
    rows = np.frombuffer(zlib.decompress(data), np.uint8).reshape(5, 1 + 7 * 4)
    assert (rows[:, 0] == 0).all()
    assert np.array_equal(rows[:, 1:].reshape(5, 7, 4), img[::-1])


RT_RENDER = os.path.join(ROOT, "gpu-ray_trace-rust_amd", "lib", "rt_render")


def read_png_rgba(path):
    raw = open(path, "rb").read()
    i, data, w, h = 8, b"", 0, 0
    while i < len(raw):
        n = int.from_bytes(raw[i:i + 4], "big")
        kind = raw[i + 4:i + 8]
        if kind == b"IHDR":
            w, h = int.from_bytes(raw[i + 8:i + 12], "big"), int.from_bytes(raw[i + 12:i + 16], "big")
        elif kind == b"IDAT":
            data += raw[i + 8:i + 8 + n]
        i += 12 + n
    rows = np.frombuffer(zlib.decompress(data), np.uint8).reshape(h, 1 + 4 * w)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].reshape(h, w, 4)


def test_rt_render_cli_usage():
    import subprocess

    r = subprocess.run([RT_RENDER], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage: rt_render" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name,devs", [("walled", []), ("triangles", []), ("walled", ["--devices", "0,0,0"]),
                                       ("biplane", ["--gpus", "1"])])
def test_rt_render_cli_equals_python_host(gpu_available, tmp_path, name, devs):
    """C++ host end to end (scheme -> rt_render_to_target -> flipped PNG) == the Python host's
    render_to_target on the same scheme, pixel for pixel; with --devices, one frame over several
    contexts (rt_render_to_target_devices) gives the same PNG."""
    import subprocess

    from rt_amd import render, scheme

    out = str(tmp_path / "render_out.png")
    r = subprocess.run([RT_RENDER, os.path.join(SCENES, name + ".json"), "no_ui", "--assets", ASSETS, "--out", out,
                        "--width", "96", "--height", "48", "--spp", "6", "--batch", "3"] + devs,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    png = read_png_rgba(out)
    loaded = scheme.load(scheme.load_json(os.path.join(SCENES, name + ".json")), assets_root=ASSETS, width=96, height=48)
    target = render.render_to_target(loaded, 6, 3)
    assert np.array_equal(png, target[::-1])
