"""`!Model` members: glTF 2.0 -> rt_mesh, as builder/pr/model.rs:19-207 does it.

- model transform T(translation) * S(uniform_scale) * R(euler) (model.rs:23-29), nalgebra f32
  products (C_ij = ((a_i0 b_0j + a_i1 b_1j) + a_i2 b_2j) + a_i3 b_3j);
- every scene's root nodes walked depth first, node matrices composed parent * node
  (model.rs:31-53); a node's TRS is turned into a matrix as the gltf crate does (T * R(q) * S);
- positions transformed by the node's world matrix, normals left untransformed (model.rs:85-90,121);
- textures are looked up as images[texture index] (model.rs:157 indexes images by the
  *texture* index, not texture.source — replicated), read with texCoord set `tex_coord`;
- texel values: image::to_rgb32f (u8 / 255).
Declared fallback: a texture whose image file is absent (spaceship_shuttle_r1's
metallicRoughness, .MISSING_LARGE_BLOBS) is treated as not present: the reference's
gltf::import would panic instead.
"""
from __future__ import annotations

import ctypes as C
import ctypes.util
from dataclasses import dataclass, field

import numpy as np

from . import abi
from .assets import open_store, to_rgb32f

F32 = np.float32
_libm = C.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.sinf.restype = C.c_float
_libm.sinf.argtypes = [C.c_float]
_libm.cosf.restype = C.c_float
_libm.cosf.argtypes = [C.c_float]

_COMP = {5120: np.int8, 5121: np.uint8, 5122: np.int16, 5123: np.uint16, 5125: np.uint32, 5126: np.float32}
_NCOMP = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4, "MAT2": 4, "MAT3": 9, "MAT4": 16}


def sinf(x) -> np.float32:  # glibc, what Rust's f32::sin calls
    return F32(_libm.sinf(float(x)))


def cosf(x) -> np.float32:
    return F32(_libm.cosf(float(x)))


def matmul4(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """f32 4x4 product in nalgebra's accumulation order (row-major arrays)."""
    c = np.zeros((4, 4), F32)
    for i in range(4):
        for j in range(4):
            s = F32(a[i, 0] * b[0, j])
            for k in range(1, 4):
                s = F32(s + F32(a[i, k] * b[k, j]))
            c[i, j] = s
    return c


def euler4(r, p, y) -> np.ndarray:
    """Matrix4::from_euler_angles (nalgebra Rotation3::from_euler_angles, to_homogeneous)."""
    sr, cr, sp, cp, sy, cy = sinf(r), cosf(r), sinf(p), cosf(p), sinf(y), cosf(y)
    m = np.eye(4, dtype=F32)
    m[0, 0] = cy * cp
    m[0, 1] = F32(F32(cy * sp) * sr) - F32(sy * cr)
    m[0, 2] = F32(F32(cy * sp) * cr) + F32(sy * sr)
    m[1, 0] = sy * cp
    m[1, 1] = F32(F32(sy * sp) * sr) + F32(cy * cr)
    m[1, 2] = F32(F32(sy * sp) * cr) - F32(cy * sr)
    m[2, 0] = -sp
    m[2, 1] = cp * sr
    m[2, 2] = cp * cr
    return m


def model_transform(model: dict) -> np.ndarray:
    t = [F32(float(v)) for v in model["translation"]]
    s = F32(float(model["uniform_scale"]))
    r, p, y = (F32(float(v)) for v in model["euler_angles"])
    T = np.eye(4, dtype=F32)
    T[0, 3], T[1, 3], T[2, 3] = t
    S = np.diag(np.array([s, s, s, 1.0], F32))
    return matmul4(matmul4(T, S), euler4(r, p, y))


def node_matrix(node: dict) -> np.ndarray:
    """gltf::scene::Transform::matrix() as a row-major f32 array."""
    if "matrix" in node:
        m = np.array([F32(float(v)) for v in node["matrix"]], F32).reshape(4, 4)  # column-major
        return m.T.copy()
    t = [F32(float(v)) for v in node.get("translation", [0, 0, 0])]
    qx, qy, qz, qw = (F32(float(v)) for v in node.get("rotation", [0, 0, 0, 1]))
    sx, sy, sz = (F32(float(v)) for v in node.get("scale", [1, 1, 1]))
    x2, y2, z2 = qx + qx, qy + qy, qz + qz
    xx2, xy2, xz2 = x2 * qx, x2 * qy, x2 * qz
    yy2, yz2, zz2 = y2 * qy, y2 * qz, z2 * qz
    sy2, sz2, sx2 = y2 * qw, z2 * qw, x2 * qw
    R = np.eye(4, dtype=F32)
    R[:3, :3] = np.array([[F32(1.0) - yy2 - zz2, xy2 - sz2, xz2 + sy2],
                          [xy2 + sz2, F32(1.0) - xx2 - zz2, yz2 - sx2],
                          [xz2 - sy2, yz2 + sx2, F32(1.0) - xx2 - yy2]], F32)
    T = np.eye(4, dtype=F32)
    T[0, 3], T[1, 3], T[2, 3] = t
    S = np.diag(np.array([sx, sy, sz, 1.0], F32))
    return matmul4(matmul4(T, R), S)


def read_accessor(doc: dict, buffers: list, idx: int, normalized_to_f32: bool = False) -> np.ndarray:
    acc = doc["accessors"][idx]
    if "sparse" in acc:
        raise NotImplementedError("sparse accessors")
    dt = np.dtype(_COMP[acc["componentType"]])
    n = _NCOMP[acc["type"]]
    count = acc["count"]
    if "bufferView" not in acc:
        out = np.zeros((count, n), dt)
    else:
        bv = doc["bufferViews"][acc["bufferView"]]
        buf = buffers[bv["buffer"]]
        off = bv.get("byteOffset", 0) + acc.get("byteOffset", 0)
        stride = bv.get("byteStride") or dt.itemsize * n
        raw = np.frombuffer(buf, dtype=np.uint8)
        view = np.lib.stride_tricks.as_strided(raw[off:], shape=(count, n * dt.itemsize), strides=(stride, 1))
        out = view.copy().view(dt).reshape(count, n)
    if normalized_to_f32 and dt != np.float32:
        # gltf::accessor::util Normalize: u8 / 255, u16 / 65535 in f32
        out = out.astype(F32) / F32(np.iinfo(dt).max)
    return out


@dataclass
class PrimData:
    poses: np.ndarray
    norms: np.ndarray
    indices: np.ndarray
    tangents: np.ndarray | None
    base_color_factor: np.ndarray
    base_tex: int = -1
    base_uv: np.ndarray | None = None
    normal_tex: int = -1
    normal_scale: float = 1.0
    normal_uv: np.ndarray | None = None
    mr_tex: int = -1
    mr_uv: np.ndarray | None = None
    metal: float = 1.0
    rough: float = 1.0


@dataclass
class MeshData:
    trans_mat: np.ndarray  # row-major 4x4 f32
    prims: list = field(default_factory=list)

    @property
    def n_tris(self) -> int:
        return sum(len(p.indices) // 3 for p in self.prims)

    def to_abi(self, keep: list) -> abi.rt_mesh:
        m = abi.rt_mesh()
        m.trans_mat[:] = [float(v) for v in self.trans_mat.T.reshape(-1)]  # column-major storage
        prims = []

        def ptr(a, ctype=C.c_float):
            if a is None:
                return None
            a = np.ascontiguousarray(a)
            keep.append(a)
            return a.ctypes.data_as(C.POINTER(ctype))

        for p in self.prims:
            r = abi.rt_mesh_prim()
            r.n_verts = len(p.poses)
            r.n_tris = len(p.indices) // 3
            r.poses = ptr(p.poses.astype(F32))
            r.norms = ptr(p.norms.astype(F32))
            r.indices = ptr(p.indices.astype(np.uint32), C.c_uint32)
            r.tangents = ptr(None if p.tangents is None else p.tangents.astype(F32))
            r.base_color_factor[:] = [float(v) for v in p.base_color_factor]
            r.base_color_tex = p.base_tex
            r.base_color_uv = ptr(p.base_uv)
            r.normal_tex = p.normal_tex
            r.normal_scale = float(p.normal_scale)
            r.normal_uv = ptr(p.normal_uv)
            r.metal_rough_tex = p.mr_tex
            r.metal_rough_uv = ptr(p.mr_uv)
            r.metal = float(p.metal)
            r.rough = float(p.rough)
            prims.append(r)
        arr = (abi.rt_mesh_prim * max(1, len(prims)))(*prims)
        keep.append(arr)
        m.n_prims = len(prims)
        m.prims = arr
        return m


def model_to_meshes(model: dict, assets_root: str, scene) -> list:
    """Model::to_meshes (model.rs:19-41); textures are appended to `scene` (SceneDesc)."""
    store = open_store(assets_root)
    doc, buffers, load_image = store.gltf(model["path"])
    tex_ids: dict[int, int] = {}

    def texture(tinfo):
        """(scene texture id, uv array) for a textureInfo, or (-1, None) when its image is absent."""
        if tinfo is None:
            return -1, None
        ti = tinfo["index"]
        if ti not in tex_ids:
            img = load_image(ti)  # images[texture.index()] (model.rs:157)
            tex_ids[ti] = -1 if img is None else scene.add_texture(to_rgb32f(img))
        if tex_ids[ti] < 0:
            return -1, None
        return tex_ids[ti], None

    meshes = []
    transform = model_transform(model)

    def generate_mesh(mesh: dict, trans: np.ndarray) -> MeshData:  # model.rs:56-134
        md = MeshData(trans_mat=trans)
        for prim in mesh["primitives"]:
            if prim.get("mode", 4) != 4:
                raise NotImplementedError("only triangle lists (mode 4)")
            attrs = prim["attributes"]
            idx = read_accessor(doc, buffers, prim["indices"]).astype(np.uint32).reshape(-1)
            pos = read_accessor(doc, buffers, attrs["POSITION"]).astype(F32)
            x, y, z = pos[:, 0], pos[:, 1], pos[:, 2]
            one = F32(1.0)
            poses = np.stack([((trans[i, 0] * x + trans[i, 1] * y) + trans[i, 2] * z) + trans[i, 3] * one
                              for i in range(3)], axis=1).astype(F32)
            norms = read_accessor(doc, buffers, attrs["NORMAL"]).astype(F32)
            tans = read_accessor(doc, buffers, attrs["TANGENT"])[:, :3].astype(F32) if "TANGENT" in attrs else None
            mat = doc["materials"][prim["material"]] if "material" in prim else {}
            pbr = mat.get("pbrMetallicRoughness", {})
            pd = PrimData(poses=poses, norms=norms, indices=idx, tangents=tans,
                          base_color_factor=np.array([F32(float(v)) for v in pbr.get("baseColorFactor", [1, 1, 1, 1])[:3]], F32))

            def coords(tinfo):
                return read_accessor(doc, buffers, attrs[f"TEXCOORD_{tinfo.get('texCoord', 0)}"],
                                     normalized_to_f32=True).astype(F32)

            bt = pbr.get("baseColorTexture")
            if bt is not None:
                tid, _ = texture(bt)
                if tid >= 0:
                    pd.base_tex, pd.base_uv = tid, coords(bt)
            nt = mat.get("normalTexture")
            if nt is not None:
                tid, _ = texture(nt)
                if tid >= 0:
                    pd.normal_tex, pd.normal_uv = tid, coords(nt)
                    pd.normal_scale = float(F32(float(nt.get("scale", 1.0))))
            mt = pbr.get("metallicRoughnessTexture")
            if mt is not None:
                tid, _ = texture(mt)
                if tid >= 0:
                    pd.mr_tex, pd.mr_uv = tid, coords(mt)
            pd.metal = float(F32(float(pbr.get("metallicFactor", 1.0))))
            pd.rough = float(F32(float(pbr.get("roughnessFactor", 1.0))))
            md.prims.append(pd)
        return md

    def explore(ni: int, parent: np.ndarray):  # model.rs:43-53
        node = doc["nodes"][ni]
        trans = matmul4(parent, node_matrix(node))
        if "mesh" in node:
            meshes.append(generate_mesh(doc["meshes"][node["mesh"]], trans))
        for c in node.get("children", []):
            explore(c, trans)

    for sc in doc.get("scenes", []):
        for ni in sc.get("nodes", []):
            explore(ni, transform)
    return meshes
