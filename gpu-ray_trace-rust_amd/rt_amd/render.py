"""Python host over the C ABI: what renderer.rs / draw_scene.rs do around the `use_gpu` switch.

`Context` owns one rt_ctx (one device); `render_to_target` is render_to_target_gpu
(src/render/draw_scene.rs:17-47) — spp/batch launches, RGBA8 after each, update hook.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .scheme import LoadedScheme


def tiles_array(tiles) -> tuple:
    arr = (abi.rt_tile * len(tiles))(*[abi.rt_tile(*map(int, t)) for t in tiles])
    return arr, len(tiles)


def tile_pixels(tiles) -> int:
    return int(sum(int(t[2]) * int(t[3]) for t in tiles))


class KdTree:
    """A host-built KD tree (rt_kd_build) exposed as numpy views; freed on close()."""

    def __init__(self, desc: abi.rt_scene_desc, max_depth: int, lib=None):
        self.lib = lib or abi.load_library()
        self.ptr = C.POINTER(abi.rt_kd_tree)()
        abi.check(self.lib, self.lib.rt_kd_build(C.byref(desc), int(max_depth), C.byref(self.ptr)))
        t = self.ptr.contents
        self.n_nodes, self.n_refs, self.max_leaf_depth = t.n_nodes, t.n_refs, t.max_leaf_depth
        self.bounds = np.array(list(t.bounds), dtype=np.float32)
        nodes = np.ctypeslib.as_array(C.cast(t.nodes, C.POINTER(C.c_uint32)), shape=(t.n_nodes, 2)) if t.n_nodes else np.zeros((0, 2), np.uint32)
        self.nodes = nodes.copy()
        self.refs = np.ctypeslib.as_array(t.refs, shape=(t.n_refs,)).copy() if t.n_refs else np.zeros(0, np.uint32)
        self.unconditional = (np.ctypeslib.as_array(t.unconditional, shape=(t.n_unconditional,)).copy()
                              if t.n_unconditional else np.zeros(0, np.uint32))

    def as_struct(self, nodes=None, refs=None) -> "abi.rt_kd_tree":
        """This tree (or the same tree with `nodes` / `refs` replaced) as an rt_kd_tree for
        rt_create; the numpy arrays it points into are kept on the returned struct."""
        nodes = np.ascontiguousarray(self.nodes if nodes is None else nodes, dtype=np.uint32)
        refs = np.ascontiguousarray(self.refs if refs is None else refs, dtype=np.uint32)
        unc = np.ascontiguousarray(self.unconditional, dtype=np.uint32)
        t = abi.rt_kd_tree()
        t.n_nodes, t.n_refs = len(nodes), len(refs)
        t.max_leaf_depth, t.n_unconditional = self.max_leaf_depth, len(unc)
        t.bounds = (C.c_float * 6)(*self.bounds.tolist())
        t.nodes = nodes.ctypes.data_as(C.POINTER(abi.rt_kd_node))
        t.refs = refs.ctypes.data_as(abi.P_u32)
        t.unconditional = unc.ctypes.data_as(abi.P_u32)
        t._keep = (nodes, refs, unc)
        return t

    def canonical_dfs(self):
        """Depth-first pre-order rows {is_leaf, axis, split bits | count, first ref} + refs —
        the same dump oracle_kd_dump produces from its pointer tree."""
        rows, refs = [], []
        if self.n_nodes == 0:
            return np.zeros((0, 4), np.uint32), np.zeros(0, np.uint32)
        stack = [0]
        while stack:
            i = stack.pop()
            a, b = int(self.nodes[i, 0]), int(self.nodes[i, 1])
            if (b & 3) == abi.RT_KD_LEAF:
                off = b >> 2
                rows.append((1, 0, a, len(refs)))
                refs.extend(self.refs[off:off + a].tolist())
            else:
                rows.append((0, b & 3, a, len(refs)))
                low = b >> 2
                stack.append(low + 1)
                stack.append(low)
        return np.array(rows, dtype=np.uint32), np.array(refs, dtype=np.uint32)

    def close(self):
        if self.ptr:
            self.lib.rt_kd_free(self.ptr)
            self.ptr = C.POINTER(abi.rt_kd_tree)()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One rt_ctx on one gfx950 device (rt_create / rt_render / rt_destroy)."""

    def __init__(self, loaded: LoadedScheme, device: int = 0, lib=None, tree: "abi.rt_kd_tree | None" = None):
        """`tree`: a caller-supplied flattened KD tree (rt_kd_tree; NULL: rt_create builds one
        with the scheme's kd_tree_depth)."""
        self.lib = lib or abi.load_library()
        self.loaded = loaded
        self.ctx = C.c_void_p()
        st = self.lib.rt_create(C.byref(loaded.desc), C.byref(loaded.cam), C.byref(loaded.info),
                                C.byref(tree) if tree is not None else None, int(device), C.byref(self.ctx))
        abi.check(self.lib, st)

    @property
    def width(self) -> int:
        return int(self.loaded.info.width)

    @property
    def height(self) -> int:
        return int(self.loaded.info.height)

    def full_tile(self):
        return [(0, 0, self.width, self.height)]

    def render(self, tiles=None, sample_begin: int = 0, sample_count: int = 1,
               want_output: bool = True) -> np.ndarray | None:
        tiles = tiles or self.full_tile()
        arr, n = tiles_array(tiles)
        out = np.empty((tile_pixels(tiles), 4), dtype=np.float32) if want_output else None
        ptr = out.ctypes.data_as(abi.P_f) if want_output else None
        abi.check(self.lib, self.lib.rt_render(self.ctx, arr, n, int(sample_begin), int(sample_count), ptr),
                  self.ctx)
        return out

    def render_range(self, tiles=None, sample_begin: int = 0, sample_count: int = 1) -> np.ndarray:
        """The mean over [sample_begin, sample_begin + sample_count) alone (rt_render_range): one
        batch's result of the reference's GPU path (gpu_utils.rs:681-724)."""
        tiles = tiles or self.full_tile()
        arr, n = tiles_array(tiles)
        out = np.empty((tile_pixels(tiles), 4), dtype=np.float32)
        abi.check(self.lib, self.lib.rt_render_range(self.ctx, arr, n, int(sample_begin), int(sample_count),
                                                     out.ctypes.data_as(abi.P_f)), self.ctx)
        return out

    def render_device(self, dev_ptr: int, tiles=None, sample_begin: int = 0, sample_count: int = 1):
        tiles = tiles or self.full_tile()
        arr, n = tiles_array(tiles)
        abi.check(self.lib, self.lib.rt_render_device(self.ctx, arr, n, int(sample_begin), int(sample_count),
                                                      C.c_void_p(dev_ptr)), self.ctx)

    def render_device_async(self, dev_ptr: int, tiles=None, sample_begin: int = 0, sample_count: int = 1,
                            stream: int = 0):
        """Enqueues the render and returns; `stream` is the caller's hipStream_t (0: the legacy
        default stream, torch's default).  rt_synchronize / synchronize() waits for it."""
        tiles = tiles or self.full_tile()
        arr, n = tiles_array(tiles)
        abi.check(self.lib, self.lib.rt_render_device_async(self.ctx, arr, n, int(sample_begin), int(sample_count),
                                                            C.c_void_p(dev_ptr), C.c_void_p(stream or None)),
                  self.ctx)

    def render_batches_device_async(self, dev_ptrs, tiles=None, sample_begin: int = 0, batch: int = 1,
                                    stream: int = 0):
        """render_to_target_gpu's batch loop on the device (rt_render_batches_device_async):
        len(dev_ptrs) batches of `batch` samples from sample_begin, batch k's frame into
        dev_ptrs[k] (0: not written).  Enqueued on `stream` like render_device_async."""
        tiles = tiles or self.full_tile()
        arr, n = tiles_array(tiles)
        outs = (C.c_void_p * len(dev_ptrs))(*[C.c_void_p(p or None) for p in dev_ptrs])
        abi.check(self.lib, self.lib.rt_render_batches_device_async(
            self.ctx, arr, n, int(sample_begin), int(batch), len(dev_ptrs), outs, C.c_void_p(stream or None)),
            self.ctx)

    def synchronize(self):
        abi.check(self.lib, self.lib.rt_synchronize(self.ctx), self.ctx)

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        abi.check(self.lib, self.lib.rt_last_kernel_ms(self.ctx, C.byref(ms)), self.ctx)
        return float(ms.value)

    def launch_stats(self) -> dict:
        """{render_ms, trace_ms, n_trace_launches, n_timed_launches} of the last render call
        (trace_ms sums the n_timed_launches first launches of the window)."""
        st = abi.rt_launch_stats()
        abi.check(self.lib, self.lib.rt_last_launch_stats(self.ctx, C.byref(st)), self.ctx)
        return {"render_ms": float(st.render_ms), "trace_ms": float(st.trace_ms),
                "n_trace_launches": int(st.n_trace_launches), "n_timed_launches": int(st.n_timed_launches)}

    def count_work(self, tiles=None, sample_begin: int = 0, sample_count: int = 1, device: bool = False) -> dict:
        """Work counters: the reference algorithm's (default) or the device path's own."""
        tiles = tiles or self.full_tile()
        arr, n = tiles_array(tiles)
        wc = abi.rt_work_counts()
        mode = abi.RT_COUNT_DEVICE if device else abi.RT_COUNT_REFERENCE
        abi.check(self.lib, self.lib.rt_count_work_ex(self.ctx, arr, n, int(sample_begin), int(sample_count),
                                                      mode, C.byref(wc)), self.ctx)
        return {k: int(getattr(wc, k)) for k, _ in abi.rt_work_counts._fields_}

    def close(self):
        if self.ctx:
            self.lib.rt_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def stripe_tiles(width: int, height: int, index: int, n_parts: int, stripe: int = 0, lib=None) -> list:
    """Context `index`'s tiles of the library's stripe deal (rt_stripe_tiles; stripe 0: the
    library's rt_stripe_rows), as (x0, y0, w, h) tuples."""
    lib = lib or abi.load_library()
    n = C.c_uint32()
    abi.check(lib, lib.rt_stripe_tiles(width, height, stripe, index, n_parts, None, 0, C.byref(n)))
    arr = (abi.rt_tile * max(n.value, 1))()
    abi.check(lib, lib.rt_stripe_tiles(width, height, stripe, index, n_parts, arr, n.value, C.byref(n)))
    return [(t.x0, t.y0, t.w, t.h) for t in arr[:n.value]]


class Frame:
    """One frame over several contexts (rt_frame_*): each renders its stripes on its device, one
    gather per frame assembles the frame on devices[0] (SURVEY.md §8e at the C ABI)."""

    def __init__(self, loaded: LoadedScheme, devices, stripe: int = 0, lib=None,
                 tree: "abi.rt_kd_tree | None" = None):
        self.lib = lib or abi.load_library()
        self.loaded = loaded
        self.devices = [int(d) for d in devices]
        self.ptr = C.c_void_p()
        devs = (C.c_int * len(self.devices))(*self.devices)
        st = self.lib.rt_frame_create(C.byref(loaded.desc), C.byref(loaded.cam), C.byref(loaded.info),
                                      C.byref(tree) if tree is not None else None, devs, len(self.devices),
                                      int(stripe), C.byref(self.ptr))
        abi.check(self.lib, st)

    def _check(self, st):
        if st != abi.RT_OK:
            msg = abi.load_library().rt_status_string(st).decode()
            raise abi.RtError(st, msg + " — " + (self.lib.rt_frame_last_error(self.ptr) or b"").decode())

    def render(self, sample_begin: int, sample_count: int):
        """Every context advances its stripes by [sample_begin, sample_begin + count) (enqueued)."""
        self._check(self.lib.rt_frame_render(self.ptr, int(sample_begin), int(sample_count)))

    def gather(self, want_host: bool = True, dev_ptr: int = 0) -> np.ndarray | None:
        """The frame-end gather; the frame (H, W, 4) f32 on the host when want_host."""
        w, h = int(self.loaded.info.width), int(self.loaded.info.height)
        out = np.empty((h, w, 4), dtype=np.float32) if want_host else None
        self._check(self.lib.rt_frame_gather(self.ptr, out.ctypes.data_as(abi.P_f) if want_host else None,
                                             C.c_void_p(dev_ptr or None)))
        return out

    def synchronize(self):
        self._check(self.lib.rt_frame_synchronize(self.ptr))

    def stats(self) -> dict:
        s = abi.rt_frame_stats()
        self._check(self.lib.rt_frame_get_stats(self.ptr, C.byref(s)))
        return {k: getattr(s, k) for k, _ in abi.rt_frame_stats._fields_}

    def part(self, index: int) -> dict:
        dev, ctx, nt = C.c_int(), C.c_void_p(), C.c_uint32()
        self._check(self.lib.rt_frame_part(self.ptr, index, C.byref(dev), C.byref(ctx), C.byref(nt)))
        return {"device": dev.value, "ctx": ctx, "n_tiles": nt.value}

    def close(self):
        if self.ptr:
            self.lib.rt_frame_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rgba_to_u8(rgba: np.ndarray, lib=None) -> np.ndarray:
    """rgb_f_to_u8 (draw_scene.rs:104-108) through the C++ host."""
    lib = lib or abi.load_library()
    rgba = np.ascontiguousarray(rgba, dtype=np.float32).reshape(-1, 4)
    out = np.empty(rgba.shape, dtype=np.uint8)
    abi.check(lib, lib.rt_rgba_to_u8(rgba.ctypes.data_as(abi.P_f), rgba.shape[0],
                                     out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out


def render_to_target(loaded: LoadedScheme, spp: int, batch: int, device: int = 0, update_hook=None,
                     lib=None) -> np.ndarray:
    """render_to_target_gpu (draw_scene.rs:17-47) via rt_render_to_target."""
    lib = lib or abi.load_library()
    w, h = int(loaded.info.width), int(loaded.info.height)
    target = np.zeros((h, w, 4), dtype=np.uint8)
    HOOK = C.CFUNCTYPE(None, C.c_void_p, C.c_uint32)
    cb = HOOK(lambda _u, done: update_hook(target, int(done))) if update_hook else None
    st = lib.rt_render_to_target(C.byref(loaded.desc), C.byref(loaded.cam), C.byref(loaded.info), int(spp),
                                 int(batch), int(device), target.ctypes.data_as(C.POINTER(C.c_uint8)),
                                 C.cast(cb, C.c_void_p) if cb else None, None)
    abi.check(lib, st)
    return target


def render_to_target_devices(loaded: LoadedScheme, spp: int, batch: int, devices, update_hook=None,
                             lib=None) -> np.ndarray:
    """render_to_target_gpu over several contexts (rt_render_to_target_devices)."""
    lib = lib or abi.load_library()
    w, h = int(loaded.info.width), int(loaded.info.height)
    target = np.zeros((h, w, 4), dtype=np.uint8)
    HOOK = C.CFUNCTYPE(None, C.c_void_p, C.c_uint32)
    cb = HOOK(lambda _u, done: update_hook(target, int(done))) if update_hook else None
    devs = (C.c_int * len(devices))(*[int(d) for d in devices])
    st = lib.rt_render_to_target_devices(C.byref(loaded.desc), C.byref(loaded.cam), C.byref(loaded.info), int(spp),
                                         int(batch), devs, len(devices), target.ctypes.data_as(C.POINTER(C.c_uint8)),
                                         C.cast(cb, C.c_void_p) if cb else None, None)
    abi.check(lib, st)
    return target
