"""Asset access for scene loading: real files (glTF + .bin + PNG/JPEG) or a packed store.

The GPU box receives only this repository, so the benchmark scenes' assets travel as packs
(`assets_pack/<dir>.npz`, written by tools/make_asset_packs.py from the reference's asset
files): the glTF JSON, its binary buffers and every image already decoded to 8-bit channels.
Both stores return the same arrays, so a scene loads identically from either.

Image decoding follows gltf::import + image::DynamicImage (builder/pr/model.rs:151-207,
pr/distant_cube_map.rs:19-23): 8-bit L / RGB / RGBA; palette images expand to RGB(A);
16-bit and luma-alpha images are rejected (the reference panics on LA8 / R16 in model.rs:202).
"""
from __future__ import annotations

import io
import json
import os

import numpy as np


def _png_bit_depth(raw: bytes):
    if raw[:8] == b"\x89PNG\r\n\x1a\n" and raw[12:16] == b"IHDR":
        return raw[24], raw[25]
    return None


def decode_image(raw: bytes) -> np.ndarray:
    """-> uint8 array (H, W, C), C in {1, 3, 4}: the channels the reference keeps before
    to_rgb32f."""
    from PIL import Image

    bd = _png_bit_depth(raw)
    if bd and bd[0] == 16:
        raise NotImplementedError("16-bit PNG textures are not supported by this loader")
    with Image.open(io.BytesIO(raw)) as im:
        mode = im.mode
        if mode == "P":
            im = im.convert("RGBA" if "transparency" in im.info else "RGB")
        elif mode == "1":
            im = im.convert("L")
        elif mode == "LA":
            raise ValueError("luma-alpha textures make the reference panic (model.rs:202)")
        elif mode not in ("L", "RGB", "RGBA"):
            im = im.convert("RGB")
        arr = np.asarray(im, dtype=np.uint8)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    return np.ascontiguousarray(arr)


def to_rgb32f(img_u8: np.ndarray) -> np.ndarray:
    """image::DynamicImage::to_rgb32f: luma replicated, alpha dropped, c / 255 in f32."""
    if img_u8.shape[2] == 1:
        img_u8 = np.repeat(img_u8, 3, axis=2)
    rgb = img_u8[:, :, :3].astype(np.float32)
    return np.ascontiguousarray(rgb / np.float32(255.0), dtype=np.float32)


class FileStore:
    """Reads assets from a directory holding the reference's `assets/` contents."""

    def __init__(self, root: str):
        self.root = root

    def path(self, rel: str) -> str:
        parts = [p for p in rel.replace("\\", "/").split("/") if p not in ("", ".", "..")]
        if parts and parts[0] == "assets":
            parts = parts[1:]
        return os.path.join(self.root, *parts)

    def read_bytes(self, rel: str) -> bytes | None:
        p = self.path(rel)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            return f.read()

    def image(self, rel: str) -> np.ndarray | None:
        raw = self.read_bytes(rel)
        return None if raw is None else decode_image(raw)

    def gltf(self, rel: str):
        """-> (json dict, [buffer bytes], image_loader(i) -> uint8 array | None)."""
        p = self.path(rel)
        with open(p) as f:
            doc = json.load(f)
        base = os.path.dirname(p)
        buffers = []
        for b in doc.get("buffers", []):
            with open(os.path.join(base, b["uri"]), "rb") as f:
                buffers.append(f.read())

        def image(i):
            uri = doc["images"][i].get("uri")
            full = os.path.join(base, uri) if uri else None
            if not full or not os.path.exists(full):
                return None
            with open(full, "rb") as f:
                return decode_image(f.read())

        return doc, buffers, image


class PackStore:
    """Reads assets from assets_pack/*.npz (see tools/make_asset_packs.py)."""

    def __init__(self, root: str):
        self.root = root
        self._open = {}

    def _pack(self, top: str):
        if top not in self._open:
            p = os.path.join(self.root, top + ".npz")
            self._open[top] = np.load(p, allow_pickle=False) if os.path.exists(p) else None
        return self._open[top]

    @staticmethod
    def _split(rel: str):
        parts = [p for p in rel.replace("\\", "/").split("/") if p not in ("", ".", "..")]
        if parts and parts[0] == "assets":
            parts = parts[1:]
        return parts[0], "/".join(parts[1:])

    @staticmethod
    def _image(pk, name):
        if pk is None:
            return None
        if "img:" + name in pk.files:
            return pk["img:" + name]
        if "jpg:" + name in pk.files:
            return decode_image(bytes(pk["jpg:" + name]))
        return None

    def image(self, rel: str) -> np.ndarray | None:
        top, name = self._split(rel)
        return self._image(self._pack(top), name)

    def gltf(self, rel: str):
        top, name = self._split(rel)
        pk = self._pack(top)
        if pk is None or ("gltf:" + name) not in pk.files:
            raise FileNotFoundError(rel)
        doc = json.loads(bytes(pk["gltf:" + name]).decode())
        buffers = [bytes(pk[f"buf:{name}:{i}"]) for i in range(len(doc.get("buffers", [])))]
        base = os.path.dirname(name)

        def image(i):
            uri = doc["images"][i].get("uri")
            if not uri:
                return None
            return self._image(pk, base + "/" + uri if base else uri)

        return doc, buffers, image


def open_store(assets_root: str | None):
    """A FileStore when `assets_root` holds real asset directories, else the packed store."""
    if assets_root is None:
        return None
    if os.path.isdir(assets_root) and any(os.path.isdir(os.path.join(assets_root, d)) for d in os.listdir(assets_root)):
        return FileStore(assets_root)
    return PackStore(assets_root)
