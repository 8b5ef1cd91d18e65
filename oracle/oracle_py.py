"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/_build/liboracle.so.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker / CPU baseline; never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
ACCUM_RECURSIVE, ACCUM_FORWARD = 0, 1

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        P_f = C.POINTER(C.c_float)
        _lib.oracle_render.restype = C.c_int
        _lib.oracle_render.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64,
                                       C.c_uint32, C.c_int, C.c_int, P_f, C.c_void_p]
        _lib.oracle_render_ex.restype = C.c_int
        _lib.oracle_render_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64,
                                          C.c_uint32, C.c_int, C.c_int, C.c_uint64, P_f, C.c_void_p]
        _lib.oracle_mix_counts.restype = None
        _lib.oracle_mix_counts.argtypes = [C.POINTER(C.c_uint64), C.c_int]
        _lib.oracle_kd_dump.restype = C.c_int
        _lib.oracle_kd_dump.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                        C.POINTER(C.c_uint32), P_f]
        _lib.oracle_mesh_normal_transforms.restype = C.c_int
        _lib.oracle_mesh_normal_transforms.argtypes = [C.c_void_p, P_f, C.c_uint64]
        _lib.oracle_aabb_entry_exit.restype = C.c_int
        _lib.oracle_aabb_entry_exit.argtypes = [P_f, P_f, P_f, C.POINTER(C.c_int), P_f, C.POINTER(C.c_int), P_f]
        _lib.oracle_raylen_cmp.restype = C.c_int
        _lib.oracle_raylen_cmp.argtypes = [C.c_float, C.c_float]
        _lib.oracle_chunk_to_pix.restype = None
        _lib.oracle_chunk_to_pix.argtypes = [C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        _lib.oracle_sphere_intersect.restype = C.c_int
        _lib.oracle_sphere_intersect.argtypes = [P_f, C.c_float, P_f, P_f, P_f]
        _lib.oracle_triangle_intersect.restype = C.c_int
        _lib.oracle_triangle_intersect.argtypes = [P_f, P_f, P_f, P_f, P_f, P_f]
        _lib.oracle_rng_stream.restype = None
        _lib.oracle_rng_stream.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, P_f]
        _lib.oracle_camera_ray.restype = None
        _lib.oracle_camera_ray.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int32, C.c_int32, C.c_uint64,
                                           C.c_uint64, P_f, P_f]
        _lib.oracle_refract.restype = None
        _lib.oracle_refract.argtypes = [P_f, P_f, C.c_float, C.c_float, C.c_float, P_f, P_f]
    return _lib


class Counts(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("samples", "segments", "nodes", "leaf_refs", "sphere_tests",
                                           "tri_tests", "hits", "mesh_hits")]


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def render(loaded, tiles, sample_begin=0, sample_count=1, threads=0, accum=ACCUM_RECURSIVE,
           init=None, counts=False, mean_base=0):
    """oracle_render over `tiles` (list of (x0, y0, w, h)) -> (npix, 4) float32 [, counts].
    `init`: the accumulator at sample_begin (used when sample_begin > mean_base); `mean_base`:
    the running mean's n is sample - mean_base (sample_begin: the mean of this range alone)."""
    from rt_amd import abi  # the scene structs are the ABI's; the oracle does not call the product

    npix = int(sum(t[2] * t[3] for t in tiles))
    out = np.zeros((npix, 4), dtype=np.float32) if init is None else np.array(init, dtype=np.float32).copy()
    tarr = (abi.rt_tile * len(tiles))(*[abi.rt_tile(*map(int, t)) for t in tiles])
    cnt = Counts()
    st = lib().oracle_render_ex(C.addressof(loaded.desc), C.addressof(loaded.cam), C.addressof(loaded.info),
                                C.addressof(tarr), len(tiles), int(sample_begin), int(sample_count), int(threads),
                                int(accum), int(mean_base), _fp(out), C.addressof(cnt) if counts else None)
    if st != 0:
        raise RuntimeError(f"oracle_render status {st}")
    if counts:
        return out, {k: int(getattr(cnt, k)) for k, _ in Counts._fields_}
    return out


def kd_dump(desc, max_depth):
    n_refs = C.c_uint32()
    bounds = np.zeros(6, np.float32)
    nn = lib().oracle_kd_dump(C.addressof(desc), int(max_depth), None, 0, None, 0, C.byref(n_refs), _fp(bounds))
    if nn < 0:
        raise RuntimeError(f"oracle_kd_dump {nn}")
    rows = np.zeros((max(nn, 1), 4), np.uint32)
    refs = np.zeros(max(n_refs.value, 1), np.uint32)
    lib().oracle_kd_dump(C.addressof(desc), int(max_depth), rows.ctypes.data, nn, refs.ctypes.data,
                         n_refs.value, C.byref(n_refs), _fp(bounds))
    return rows[:nn], refs[:n_refs.value], bounds


def mesh_normal_transforms(desc, n_tris):
    out = np.zeros((max(n_tris, 1), 3, 3), np.float32)
    k = lib().oracle_mesh_normal_transforms(C.addressof(desc), _fp(out), n_tris)
    if k < 0:
        raise RuntimeError("oracle_mesh_normal_transforms failed")
    return out[:k]


MIX_FIELDS = ("spec", "diff", "diffspec_diff", "diffspec_spec", "dielectric", "rr_draws", "draws", "mesh",
              "sphere_disc_positive") + tuple(f"node_d{d}" for d in range(40))


def mix_counts(reset=True):
    """Shading mix of the counted renders (render(..., counts=True)) since the last reset."""
    out = (C.c_uint64 * len(MIX_FIELDS))()
    lib().oracle_mix_counts(out, int(reset))
    return dict(zip(MIX_FIELDS, (int(v) for v in out)))
