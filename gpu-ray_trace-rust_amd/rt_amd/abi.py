"""ctypes mirror of include/rt_abi.h and the loader of lib/librt_amd.so.

The structures here are byte-for-byte the C ABI (checked against the header's sizes by
tests/test_abi.py).  `load_library()` raises when the shared library is missing: there is no
Python or CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "lib", "librt_amd.so")

RT_OK = 0
RT_ERR_INVALID_ARG = -1
RT_ERR_OOM = -2
RT_ERR_HIP = -3
RT_ERR_UNSUPPORTED = -4
RT_ERR_NO_DEVICE = -5
RT_ERR_BATCH = -6

RT_DIVERT_SPEC, RT_DIVERT_DIFF, RT_DIVERT_DIFFSPEC, RT_DIVERT_DIELECTRIC = 0, 1, 2, 3
RT_ELEM_SPHERE, RT_ELEM_FREE_TRI, RT_ELEM_CUBE_MAP = 0, 1, 2
RT_FACE_NEG_X, RT_FACE_POS_X, RT_FACE_NEG_Y, RT_FACE_POS_Y, RT_FACE_NEG_Z, RT_FACE_POS_Z = range(6)
RT_KD_LEAF = 3
RT_COUNT_REFERENCE, RT_COUNT_DEVICE = 0, 1

f3 = C.c_float * 3
P_f = C.POINTER(C.c_float)
P_u32 = C.POINTER(C.c_uint32)


class rt_material(C.Structure):
    _fields_ = [("emissive", f3), ("has_emissive", C.c_uint32), ("divert", C.c_uint32),
                ("diffp", C.c_float), ("n_out", C.c_float), ("n_in", C.c_float)]


class rt_sphere(C.Structure):
    _fields_ = [("c", f3), ("r", C.c_float), ("rgb", f3), ("_pad0", C.c_uint32), ("mat", rt_material)]


class rt_free_triangle(C.Structure):
    _fields_ = [("verts", f3 * 3), ("norm", f3), ("rgb", f3), ("_pad0", C.c_uint32), ("mat", rt_material)]


class rt_texture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("rgb", P_f)]


class rt_cube_face(C.Structure):
    _fields_ = [("texture", C.c_int32), ("us", C.c_float), ("vs", C.c_float)]


class rt_cube_map(C.Structure):
    _fields_ = [("face", rt_cube_face * 6)]


class rt_mesh_prim(C.Structure):
    _fields_ = [("n_verts", C.c_uint32), ("n_tris", C.c_uint32), ("poses", P_f), ("norms", P_f),
                ("indices", P_u32), ("tangents", P_f), ("base_color_factor", f3),
                ("base_color_tex", C.c_int32), ("base_color_uv", P_f), ("normal_tex", C.c_int32),
                ("normal_scale", C.c_float), ("normal_uv", P_f), ("metal_rough_tex", C.c_int32),
                ("metal_rough_uv", P_f), ("metal", C.c_float), ("rough", C.c_float)]


class rt_mesh(C.Structure):
    _fields_ = [("trans_mat", C.c_float * 16), ("n_prims", C.c_uint32), ("prims", C.POINTER(rt_mesh_prim))]


class rt_elem(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("index", C.c_uint32)]


class rt_scene_desc(C.Structure):
    _fields_ = [("n_elems", C.c_uint32), ("elems", C.POINTER(rt_elem)),
                ("n_spheres", C.c_uint32), ("spheres", C.POINTER(rt_sphere)),
                ("n_free_tris", C.c_uint32), ("free_tris", C.POINTER(rt_free_triangle)),
                ("n_cube_maps", C.c_uint32), ("cube_maps", C.POINTER(rt_cube_map)),
                ("n_meshes", C.c_uint32), ("meshes", C.POINTER(rt_mesh)),
                ("n_textures", C.c_uint32), ("textures", C.POINTER(rt_texture))]


class rt_camera(C.Structure):
    _fields_ = [("d", f3), ("o", f3), ("up", f3), ("screen_width", C.c_float),
                ("screen_height", C.c_float), ("has_lens", C.c_uint32), ("lens_r", C.c_float)]


class rt_render_info(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("kd_tree_depth", C.c_uint32),
                ("assured_depth", C.c_int32), ("max_thres", C.c_float), ("debug_single_ray", C.c_uint32),
                ("dir_light_samp", C.c_uint32), ("_pad0", C.c_uint32), ("seed", C.c_uint64)]


class rt_tile(C.Structure):
    _fields_ = [("x0", C.c_uint32), ("y0", C.c_uint32), ("w", C.c_uint32), ("h", C.c_uint32)]


class rt_kd_node(C.Structure):
    _fields_ = [("a", C.c_uint32), ("b", C.c_uint32)]


class rt_kd_tree(C.Structure):
    _fields_ = [("n_nodes", C.c_uint32), ("n_refs", C.c_uint32), ("max_leaf_depth", C.c_uint32),
                ("n_unconditional", C.c_uint32), ("bounds", C.c_float * 6),
                ("nodes", C.POINTER(rt_kd_node)), ("refs", P_u32), ("unconditional", P_u32)]


class rt_launch_stats(C.Structure):
    _fields_ = [("render_ms", C.c_float), ("trace_ms", C.c_float), ("n_trace_launches", C.c_uint32),
                ("n_timed_launches", C.c_uint32)]


class rt_work_counts(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("samples", "segments", "nodes", "leaf_refs", "sphere_tests",
                                           "tri_tests", "hits", "mesh_hits")]


class rt_frame_stats(C.Structure):
    _fields_ = [("render_ms_max", C.c_float), ("peer_copy_ms_max", C.c_float), ("place_ms", C.c_float),
                ("n_parts", C.c_uint32), ("stripe_rows", C.c_uint32), ("n_gathers", C.c_uint32),
                ("n_peer_copies", C.c_uint32)]


RT_SCHEME_YAML, RT_SCHEME_JSON = 0, 1


class rt_scheme_view(C.Structure):
    _fields_ = [("scene", C.POINTER(rt_scene_desc)), ("cam", C.POINTER(rt_camera)),
                ("info", C.POINTER(rt_render_info)), ("samps_per_pix", C.c_uint32),
                ("gpu_render_batch", C.c_uint32), ("use_gpu", C.c_uint32), ("animation", C.c_uint32)]


# Every symbol the header declares (tests/test_abi.py checks the library exports them all).
EXPORTS = {
    "rt_abi_version": (C.c_int, []),
    "rt_status_string": (C.c_char_p, [C.c_int]),
    "rt_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rt_camera_from_scheme": (C.c_int, [P_f, P_f, P_f, C.c_float, C.c_float, C.c_uint32, C.c_float, P_f,
                                        C.POINTER(rt_camera)]),
    "rt_kd_build": (C.c_int, [C.POINTER(rt_scene_desc), C.c_uint32, C.POINTER(C.POINTER(rt_kd_tree))]),
    "rt_kd_free": (None, [C.POINTER(rt_kd_tree)]),
    "rt_create": (C.c_int, [C.POINTER(rt_scene_desc), C.POINTER(rt_camera), C.POINTER(rt_render_info),
                            C.POINTER(rt_kd_tree), C.c_int, C.POINTER(C.c_void_p)]),
    "rt_render": (C.c_int, [C.c_void_p, C.POINTER(rt_tile), C.c_uint32, C.c_uint64, C.c_uint32, P_f]),
    "rt_render_device": (C.c_int, [C.c_void_p, C.POINTER(rt_tile), C.c_uint32, C.c_uint64, C.c_uint32,
                                   C.c_void_p]),
    "rt_render_device_async": (C.c_int, [C.c_void_p, C.POINTER(rt_tile), C.c_uint32, C.c_uint64, C.c_uint32,
                                         C.c_void_p, C.c_void_p]),
    "rt_render_batches_device_async": (C.c_int, [C.c_void_p, C.POINTER(rt_tile), C.c_uint32, C.c_uint64,
                                                 C.c_uint32, C.c_uint32, C.POINTER(C.c_void_p), C.c_void_p]),
    "rt_render_range": (C.c_int, [C.c_void_p, C.POINTER(rt_tile), C.c_uint32, C.c_uint64, C.c_uint32, P_f]),
    "rt_synchronize": (C.c_int, [C.c_void_p]),
    "rt_last_kernel_ms": (C.c_int, [C.c_void_p, P_f]),
    "rt_last_launch_stats": (C.c_int, [C.c_void_p, C.POINTER(rt_launch_stats)]),
    "rt_count_work": (C.c_int, [C.c_void_p, C.POINTER(rt_tile), C.c_uint32, C.c_uint64, C.c_uint32,
                                C.POINTER(rt_work_counts)]),
    "rt_count_work_ex": (C.c_int, [C.c_void_p, C.POINTER(rt_tile), C.c_uint32, C.c_uint64, C.c_uint32,
                                   C.c_uint32, C.POINTER(rt_work_counts)]),
    "rt_last_error": (C.c_char_p, [C.c_void_p]),
    "rt_destroy": (C.c_int, [C.c_void_p]),
    "rt_rgba_to_u8": (C.c_int, [P_f, C.c_uint64, C.POINTER(C.c_uint8)]),
    "rt_render_to_target": (C.c_int, [C.POINTER(rt_scene_desc), C.POINTER(rt_camera),
                                      C.POINTER(rt_render_info), C.c_uint32, C.c_uint32, C.c_int,
                                      C.POINTER(C.c_uint8), C.c_void_p, C.c_void_p]),
    "rt_stripe_rows": (C.c_uint32, [C.c_uint32, C.c_uint32]),
    "rt_stripe_tiles": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.POINTER(rt_tile), C.c_uint32, C.POINTER(C.c_uint32)]),
    "rt_frame_create": (C.c_int, [C.POINTER(rt_scene_desc), C.POINTER(rt_camera), C.POINTER(rt_render_info),
                                  C.POINTER(rt_kd_tree), C.POINTER(C.c_int), C.c_uint32, C.c_uint32,
                                  C.POINTER(C.c_void_p)]),
    "rt_frame_render": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32]),
    "rt_frame_gather": (C.c_int, [C.c_void_p, P_f, C.c_void_p]),
    "rt_frame_synchronize": (C.c_int, [C.c_void_p]),
    "rt_frame_get_stats": (C.c_int, [C.c_void_p, C.POINTER(rt_frame_stats)]),
    "rt_frame_part": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_int), C.POINTER(C.c_void_p),
                                C.POINTER(C.c_uint32)]),
    "rt_frame_last_error": (C.c_char_p, [C.c_void_p]),
    "rt_frame_destroy": (C.c_int, [C.c_void_p]),
    "rt_render_to_target_devices": (C.c_int, [C.POINTER(rt_scene_desc), C.POINTER(rt_camera),
                                              C.POINTER(rt_render_info), C.c_uint32, C.c_uint32,
                                              C.POINTER(C.c_int), C.c_uint32, C.POINTER(C.c_uint8), C.c_void_p,
                                              C.c_void_p]),
    "rt_scheme_load": (C.c_int, [C.c_char_p, C.c_uint64, C.c_uint32, C.c_char_p, C.c_uint64,
                                 C.POINTER(C.c_void_p)]),
    "rt_scheme_view_get": (C.c_int, [C.c_void_p, C.POINTER(rt_scheme_view)]),
    "rt_scheme_last_error": (C.c_char_p, []),
    "rt_scheme_free": (C.c_int, [C.c_void_p]),
    "rt_scheme_frames": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "rt_scheme_frame": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]),
    "rt_write_png": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint8), C.c_uint32, C.c_uint32, C.c_uint32]),
}

_LIB = None


def load_library(path: str | None = None):
    """Loads librt_amd.so (built by `make -C gpu-ray_trace-rust_amd`); raises if absent."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    # torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's).  A process gets one
    # HIP runtime: when torch is importable let it load first, so both use the same one.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(p):
        raise RuntimeError(f"{p} is missing: build the HIP extension first (__graft_entry__.build())")
    lib = C.CDLL(p)
    for name, (res, args) in EXPORTS.items():
        if path is not None and not hasattr(lib, name):
            continue  # an older build loaded for A/B (tools/variant_bench.py)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _LIB = lib
    return lib


def kernel_build_id(path: str | None = None) -> str:
    """Identity of the library's device code: sha256 (16 hex digits) of its .hip_fatbin ELF
    section.  Host-side changes leave it alone; any kernel change moves it.  Keys the committed
    rocprofv3 counters (profiles/*_counters.json) to the build they were measured on."""
    import hashlib
    import struct

    b = open(path or LIB_PATH, "rb").read()
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    names = secs[shstrndx][4]
    for s in secs:
        name = b[names + s[0]: b.index(b"\0", names + s[0])]
        if name == b".hip_fatbin":
            return hashlib.sha256(b[s[4]: s[4] + s[5]]).hexdigest()[:16]
    raise RuntimeError("no .hip_fatbin section in " + (path or LIB_PATH))


class RtError(RuntimeError):
    def __init__(self, status: int, msg: str = ""):
        self.status = status
        super().__init__(f"rt status {status}: {msg}")


def check(lib, status: int, ctx=None):
    if status != RT_OK:
        detail = lib.rt_status_string(status).decode()
        if ctx:
            detail += " — " + (lib.rt_last_error(ctx) or b"").decode()
        raise RtError(status, detail)
