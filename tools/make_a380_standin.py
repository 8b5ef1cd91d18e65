"""Synthetic stand-in for the a380 geometry.

The reference snapshot holds a380/scene.gltf (node tree, 32 mesh primitives, materials, 21
textures) but not its binary buffer scene.bin (listed in .MISSING_LARGE_BLOBS).  This tool
writes a deterministic replacement buffer of the declared byteLength into assets_pack/a380.npz
as "buf:scene.gltf:0", laid out exactly as the glTF's accessors and bufferViews declare, so the
unchanged glTF reader (rt_amd/gltf.py) loads it:

  * every primitive keeps its declared vertex count (312,143 in total) and index count
    (127,749 triangles), its material and its textures;
  * its vertices lie on an ellipsoid fitted to the accessor's POSITION min/max box (the long
    axis of the box is the ellipsoid's polar axis), with outward normals and (u, v) texture
    coordinates from the surface parameters;
  * its triangles are the first n of the parameter grid's quads, split in two (repeated
    cyclically if the grid has fewer), so the surface is a closed, non-degenerate mesh.

The image is not comparable to the reference's a380 renders; the workload shape (primitive,
triangle and vertex counts, bounding boxes, texture set, camera, KD depth) is.  Run in this
container after tools/make_asset_packs.py:  python tools/make_a380_standin.py
"""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PACK = os.path.join(ROOT, "assets_pack", "a380.npz")
SEED = 0xA380


def surface(n_verts, n_tris, lo, hi, rng):
    cols = max(3, int(round(np.sqrt(n_verts))))
    rows = max(2, n_verts // cols)
    while rows * cols > n_verts:
        cols -= 1
    u = np.linspace(0.0, 1.0, cols, dtype=np.float64)
    v = np.linspace(0.0, 1.0, rows, dtype=np.float64)
    uu, vv = np.meshgrid(u, v)
    lo = np.asarray(lo, np.float64)
    hi = np.asarray(hi, np.float64)
    c = (lo + hi) / 2
    e = np.maximum((hi - lo) / 2, 1e-3)
    pole = int(np.argmax(e))            # polar axis = the box's longest side
    a1, a2 = [a for a in range(3) if a != pole]
    th = 2 * np.pi * uu
    ph = np.pi * (0.02 + 0.96 * vv)     # stay off the poles: no degenerate rows
    unit = np.zeros(uu.shape + (3,))
    unit[..., pole] = np.cos(ph)
    unit[..., a1] = np.cos(th) * np.sin(ph)
    unit[..., a2] = np.sin(th) * np.sin(ph)
    pos = c + e * unit
    nrm = unit / (e * e)
    nrm /= np.linalg.norm(nrm, axis=-1, keepdims=True)
    uv = np.stack([uu, vv], -1)
    pos = pos.reshape(-1, 3)
    nrm = nrm.reshape(-1, 3)
    uv = uv.reshape(-1, 2)
    extra = n_verts - pos.shape[0]      # leftover vertices: jittered copies (unreferenced)
    if extra:
        pick = rng.integers(0, pos.shape[0], extra)
        pos = np.concatenate([pos, pos[pick]])
        nrm = np.concatenate([nrm, nrm[pick]])
        uv = np.concatenate([uv, uv[pick]])
    quads = []
    for r in range(rows - 1):
        for q in range(cols - 1):
            a = r * cols + q
            quads.append((a, a + 1, a + cols))
            quads.append((a + 1, a + cols + 1, a + cols))
    tris = np.array(quads, np.uint32)
    reps = int(np.ceil(n_tris / len(tris)))
    tris = np.tile(tris, (reps, 1))[:n_tris]
    return pos.astype(np.float32), nrm.astype(np.float32), uv.astype(np.float32), tris


def main():
    g = json.loads(bytes(np.load(PACK)["gltf:scene.gltf"]).decode())
    buf = np.zeros(g["buffers"][0]["byteLength"], np.uint8)
    views = g["bufferViews"]
    rng = np.random.default_rng(SEED)

    def put(acc_i, arr, comps):
        acc = g["accessors"][acc_i]
        view = views[acc["bufferView"]]
        stride = view.get("byteStride", 0) or arr.dtype.itemsize * comps
        base = view.get("byteOffset", 0) + acc.get("byteOffset", 0)
        assert acc["count"] == arr.shape[0], (acc_i, acc["count"], arr.shape)
        raw = np.ascontiguousarray(arr).view(np.uint8).reshape(arr.shape[0], -1)
        for k in range(arr.shape[0]):
            buf[base + k * stride: base + k * stride + raw.shape[1]] = raw[k]

    n_tri = n_vert = 0
    for m in g["meshes"]:
        for p in m["primitives"]:
            at = p["attributes"]
            pa = g["accessors"][at["POSITION"]]
            ia = g["accessors"][p["indices"]]
            assert ia["componentType"] == 5125, "u32 indices"
            pos, nrm, uv, tris = surface(pa["count"], ia["count"] // 3, pa["min"], pa["max"], rng)
            put(at["POSITION"], pos, 3)
            put(at["NORMAL"], nrm, 3)
            put(at["TEXCOORD_0"], uv, 2)
            put(p["indices"], tris.reshape(-1, 1), 1)
            n_tri += ia["count"] // 3
            n_vert += pa["count"]
    d = dict(np.load(PACK))
    d["buf:scene.gltf:0"] = buf
    np.savez_compressed(PACK, **d)
    print(f"a380 stand-in: {n_tri} triangles, {n_vert} vertices, {buf.size} bytes -> {PACK}")


if __name__ == "__main__":
    main()
