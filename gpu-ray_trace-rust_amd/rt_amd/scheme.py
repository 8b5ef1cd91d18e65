"""Scheme loading: the reference's scheme YAML -> rt_scene_desc / rt_camera / rt_render_info.

Mirrors `Scheme::from_yml` (src/builder/mod.rs:63-72) and the member conversions of
src/builder/inner.rs:21-110 (serde externally-tagged enums `!Sphere`, `!FreeTriangle`,
`!DistantCubeMap`, `!Model`; `Coloring::Solid`; `DivertRayMethod`).  Numbers are parsed as
f64 and rounded to f32, as serde does for f32 fields.  f32 arithmetic on the host
(FreeTriangle normalisation, inner.rs:48) is done in numpy float32 scalars — one IEEE rounding
per operation, nalgebra's operation order.  The camera conversion runs in the C++ host
(rt_camera_from_scheme).

A parsed scheme is a plain dict (tagged values as {"!Tag": value}); `dump_json` / `load_json`
store it without the YAML so the GPU box (which has no /root/reference) can load benchmark
scenes from tests/golden/scenes/*.json.
"""
from __future__ import annotations

import ctypes as C
import json
import os
from dataclasses import dataclass, field

import numpy as np

from . import abi

F32 = np.float32
DEFAULT_SEED = 0x5EED0001


def _load_yaml(text: str) -> dict:
    import yaml

    class _Loader(yaml.SafeLoader):
        pass

    def _tagged(loader, suffix, node):
        if isinstance(node, yaml.MappingNode):
            v = loader.construct_mapping(node, deep=True)
        elif isinstance(node, yaml.SequenceNode):
            v = loader.construct_sequence(node, deep=True)
        else:
            v = loader.construct_scalar(node)
        return {"!" + suffix: v}

    _Loader.add_multi_constructor("!", _tagged)
    return yaml.load(text, Loader=_Loader)


def from_yml(text: str) -> dict:
    """Scheme::from_yml (builder/mod.rs:64-67): parse only; corrections happen at conversion."""
    return _load_yaml(text)


def dump_json(scheme: dict, path: str) -> None:
    with open(path, "w") as f:
        json.dump(scheme, f, indent=1, sort_keys=True)


def load_json(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


def _f(x) -> np.float32:
    return F32(float(x))


def _v3(v) -> np.ndarray:
    return np.array([_f(e) for e in v], dtype=F32)


def _normalize(v: np.ndarray) -> np.ndarray:
    x, y, z = (F32(e) for e in v)
    n = np.sqrt(F32(F32(x * x + y * y) + z * z))
    return np.array([x / n, y / n, z / n], dtype=F32)


def _tag(v):
    """('Tag', value) of an externally tagged enum value; unit variants are plain strings."""
    if isinstance(v, dict) and len(v) == 1:
        (k, val), = v.items()
        if k.startswith("!"):
            return k[1:], val
    if isinstance(v, str):
        return v, None
    raise ValueError(f"not an enum value: {v!r}")


def _material(m: dict) -> abi.rt_material:
    """UniformDiffuseSpec (material/uniform_diff_spec.rs:7-19)."""
    out = abi.rt_material()
    em = m.get("emissive")
    if em is not None:
        out.has_emissive = 1
        out.emissive[:] = [float(e) for e in _v3(em)]
    kind, val = _tag(m["divert_ray"])
    if kind == "Spec":
        out.divert = abi.RT_DIVERT_SPEC
    elif kind == "Diff":
        out.divert = abi.RT_DIVERT_DIFF
    elif kind == "DiffSpec":
        out.divert = abi.RT_DIVERT_DIFFSPEC
        out.diffp = float(_f(val["diffp"]))
    elif kind == "Dielectric":
        out.divert = abi.RT_DIVERT_DIELECTRIC
        out.n_out = float(_f(val["n_out"]))
        out.n_in = float(_f(val["n_in"]))
    else:
        raise ValueError(f"unknown divert_ray {kind}")
    return out


def resolve_asset(path: str, assets_root: str) -> str:
    """Scheme asset paths are relative to the reference's run directory ("../../assets/..."):
    they resolve against `assets_root` (the directory holding `assets/`'s contents)."""
    parts = [p for p in path.replace("\\", "/").split("/") if p not in ("", ".", "..")]
    if parts and parts[0] == "assets":
        parts = parts[1:]
    return os.path.join(assets_root, *parts)


def load_texture(store, path: str) -> np.ndarray:
    """image::open(..).into_rgb32f() (builder/pr/distant_cube_map.rs:19-23): 8-bit channels
    -> c / 255 in f32, alpha dropped.  Decoded with PIL (JPEG decoders may differ from the
    image crate by 1 LSB — parity unpinned; oracle and device read the same texels)."""
    from .assets import to_rgb32f

    img = store.image(path)
    if img is None:
        raise FileNotFoundError(path)
    return to_rgb32f(img)


@dataclass
class SceneDesc:
    """Owns every array an rt_scene_desc points into (keep it alive while the desc is used)."""
    elems: list = field(default_factory=list)
    spheres: list = field(default_factory=list)
    free_tris: list = field(default_factory=list)
    cube_maps: list = field(default_factory=list)
    textures: list = field(default_factory=list)      # (h, w, 3) float32 arrays
    meshes: list = field(default_factory=list)        # rt_amd.gltf.MeshData
    _keep: list = field(default_factory=list)
    desc: abi.rt_scene_desc | None = None

    def add_texture(self, arr: np.ndarray) -> int:
        self.textures.append(np.ascontiguousarray(arr, dtype=F32))
        return len(self.textures) - 1

    def build(self) -> abi.rt_scene_desc:
        d = abi.rt_scene_desc()
        keep = self._keep
        keep.clear()

        def arr(ctype, items):
            a = (ctype * max(1, len(items)))(*items)
            keep.append(a)
            return a

        d.n_elems = len(self.elems)
        d.elems = arr(abi.rt_elem, [abi.rt_elem(k, i) for k, i in self.elems])
        d.n_spheres = len(self.spheres)
        d.spheres = arr(abi.rt_sphere, self.spheres)
        d.n_free_tris = len(self.free_tris)
        d.free_tris = arr(abi.rt_free_triangle, self.free_tris)
        d.n_cube_maps = len(self.cube_maps)
        d.cube_maps = arr(abi.rt_cube_map, self.cube_maps)
        texs = []
        for t in self.textures:
            tx = abi.rt_texture(t.shape[1], t.shape[0], t.ctypes.data_as(abi.P_f))
            texs.append(tx)
        d.n_textures = len(texs)
        d.textures = arr(abi.rt_texture, texs)
        meshes = [m.to_abi(keep) for m in self.meshes]
        d.n_meshes = len(meshes)
        d.meshes = arr(abi.rt_mesh, meshes)
        self.desc = d
        return d


@dataclass
class LoadedScheme:
    scheme: dict
    scene: SceneDesc
    desc: abi.rt_scene_desc
    cam: abi.rt_camera
    info: abi.rt_render_info
    spp: int
    batch: int | None


def render_info(ri: dict, seed: int = DEFAULT_SEED, width: int | None = None,
                height: int | None = None) -> abi.rt_render_info:
    """RenderInfo (render/cpu_utils.rs:4-15) + RadianceInfo (radiance.rs:8-18)."""
    out = abi.rt_render_info()
    out.width = int(width if width is not None else ri["width"])
    out.height = int(height if height is not None else ri["height"])
    out.kd_tree_depth = int(ri["kd_tree_depth"])
    rad = ri["rad_info"]
    out.assured_depth = int(rad["russ_roull_info"]["assured_depth"])
    out.max_thres = float(_f(rad["russ_roull_info"]["max_thres"]))
    out.debug_single_ray = 1 if rad["debug_single_ray"] else 0
    out.dir_light_samp = 1 if rad["dir_light_samp"] else 0
    out.seed = int(seed)
    return out


def camera(cam: dict, lib=None) -> abi.rt_camera:
    """From<pr::Cam> for scene::Cam (builder/pr/cam.rs:19-81) via the C++ host."""
    lib = lib or abi.load_library()
    d, o, up, e = (np.ascontiguousarray(_v3(cam[k]), dtype=F32) for k in ("d", "o", "up", "view_eulers"))
    out = abi.rt_camera()
    lens = cam.get("lens_r")
    st = lib.rt_camera_from_scheme(d.ctypes.data_as(abi.P_f), o.ctypes.data_as(abi.P_f),
                                   up.ctypes.data_as(abi.P_f), float(_f(cam["screen_width"])),
                                   float(_f(cam["screen_height"])), 1 if lens is not None else 0,
                                   float(_f(lens)) if lens is not None else 0.0,
                                   e.ctypes.data_as(abi.P_f), C.byref(out))
    abi.check(lib, st)
    return out


def scene_from_members(members: list, assets_root: str | None) -> SceneDesc:
    """Vec<Member> conversion (builder/inner.rs:21-64) in renderable order."""
    from .assets import open_store

    sc = SceneDesc()
    store = open_store(assets_root)
    tex_cache: dict[str, int] = {}
    for m in members:
        kind, v = _tag(m)
        if kind == "Sphere":
            s = abi.rt_sphere()
            s.c[:] = [float(e) for e in _v3(v["c"])]
            s.r = float(_f(v["r"]))
            ck, cv = _tag(v["coloring"])
            if ck != "Solid":
                raise ValueError(f"unknown coloring {ck}")
            s.rgb[:] = [float(e) for e in _v3(cv)]
            s.mat = _material(v["mat"])
            sc.elems.append((abi.RT_ELEM_SPHERE, len(sc.spheres)))
            sc.spheres.append(s)
        elif kind == "FreeTriangle":
            t = abi.rt_free_triangle()
            for i in range(3):
                t.verts[i][:] = [float(e) for e in _v3(v["verts"][i])]
            t.norm[:] = [float(e) for e in _normalize(_v3(v["norm"]))]  # inner.rs:48
            t.rgb[:] = [float(e) for e in _v3(v["rgb"])]
            t.mat = _material(v["mat"])
            sc.elems.append((abi.RT_ELEM_FREE_TRI, len(sc.free_tris)))
            sc.free_tris.append(t)
        elif kind == "DistantCubeMap":
            if assets_root is None:
                raise ValueError("DistantCubeMap needs assets_root")
            cm = abi.rt_cube_map()
            for fi, name in enumerate(("neg_x", "pos_x", "neg_y", "pos_y", "neg_z", "pos_z")):
                path, us, vs = v[name]
                if path not in tex_cache:
                    tex_cache[path] = sc.add_texture(load_texture(store, path))
                cm.face[fi] = abi.rt_cube_face(tex_cache[path], float(_f(us)), float(_f(vs)))
            sc.elems.append((abi.RT_ELEM_CUBE_MAP, len(sc.cube_maps)))
            sc.cube_maps.append(cm)
        elif kind == "Model":
            from . import gltf  # noqa: PLC0415 - only needed for mesh scenes

            if assets_root is None:
                raise ValueError("Model needs assets_root")
            sc.meshes.extend(gltf.model_to_meshes(v, assets_root, sc))
        else:
            raise ValueError(f"unknown scene member {kind}")
    return sc


def load(scheme: dict, assets_root: str | None = None, seed: int = DEFAULT_SEED,
         width: int | None = None, height: int | None = None, lib=None) -> LoadedScheme:
    ri = scheme["render_info"]
    sc = scene_from_members(scheme["scene_members"], assets_root)
    desc = sc.build()
    return LoadedScheme(scheme=scheme, scene=sc, desc=desc, cam=camera(scheme["cam"], lib),
                        info=render_info(ri, seed, width, height), spp=int(ri["samps_per_pix"]),
                        batch=ri.get("gpu_render_batch"))


class NativeScheme:
    """A scheme loaded by the C++ host (rt_scheme_load): the same LoadedScheme fields, with the
    description owned by the library.  `text` is YAML or this repo's JSON form."""

    def __init__(self, text: str, assets_root: str | None, fmt: int | None = None, seed: int = DEFAULT_SEED,
                 width: int | None = None, height: int | None = None, lib=None):
        self.lib = lib or abi.load_library()
        if fmt is None:
            fmt = abi.RT_SCHEME_JSON if text.lstrip().startswith("{") else abi.RT_SCHEME_YAML
        raw = text.encode()
        self.ptr = C.c_void_p()
        st = self.lib.rt_scheme_load(raw, len(raw), fmt, assets_root.encode() if assets_root else None, int(seed),
                                     C.byref(self.ptr))
        if st != abi.RT_OK:
            raise abi.RtError(st, (self.lib.rt_scheme_last_error() or b"").decode())
        v = abi.rt_scheme_view()
        abi.check(self.lib, self.lib.rt_scheme_view_get(self.ptr, C.byref(v)))
        self.view = v
        self.desc = v.scene.contents
        self.cam = v.cam.contents
        self.info = v.info.contents
        if width is not None:
            self.info.width = int(width)
        if height is not None:
            self.info.height = int(height)
        self.spp = int(v.samps_per_pix)
        self.batch = int(v.gpu_render_batch) or None

    @classmethod
    def _wrap(cls, lib, ptr):
        self = cls.__new__(cls)
        self.lib, self.ptr = lib, ptr
        v = abi.rt_scheme_view()
        abi.check(lib, lib.rt_scheme_view_get(ptr, C.byref(v)))
        self.view, self.desc, self.cam, self.info = v, v.scene.contents, v.cam.contents, v.info.contents
        self.spp, self.batch = int(v.samps_per_pix), int(v.gpu_render_batch) or None
        return self

    def n_frames(self) -> int:
        """rt_scheme_frames: frames of an animated scheme (0 otherwise)."""
        n = C.c_uint32()
        st = self.lib.rt_scheme_frames(self.ptr, C.byref(n))
        if st != abi.RT_OK:
            raise abi.RtError(st, (self.lib.rt_scheme_last_error() or b"").decode())
        return int(n.value)

    def frame(self, i: int) -> "NativeScheme":
        """rt_scheme_frame: animation frame i as a still scheme."""
        p = C.c_void_p()
        st = self.lib.rt_scheme_frame(self.ptr, int(i), C.byref(p))
        if st != abi.RT_OK:
            raise abi.RtError(st, (self.lib.rt_scheme_last_error() or b"").decode())
        return NativeScheme._wrap(self.lib, p)

    def close(self):
        if self.ptr:
            self.lib.rt_scheme_free(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
