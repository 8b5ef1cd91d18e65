"""Prices an exact culling of a leaf's triangle tests by cluster boxes ("Cluster
boxes"): primary rays of a scene, traversed as the reference does (kdtree.rs:66-104), and per leaf
visit the triangle tests made against the tests left if the leaf's triangles were grouped in
clusters of C (leaf order, or Morton order of centroids with SORT=1) and a cluster were skipped
whenever the ray segment [0, exit + EPS] misses its box grown by a pad:
  - "loose": 1e-3 of the cluster's extent (no exactness argument: what culling could gain);
  - "rigorous": the float error bound of Moller-Trumbore (triangle/generic.rs:102-137) in the
    form the kernel computes it, so that a skipped cluster provably holds no accepted hit; the
    bound grows like 1/|det|, and |det| is bounded below by the cluster's normal cone against the
    ray (or the reference's EPS floor when the cone is wide).
`viol` counts leaf visits where a pad missed an accepted hit (0 expected for both).
Usage: python tools/cluster_cull.py [scene] [grid]   (env SORT=0|1|2: leaf / Morton / normal bins, PAD=loose|rigorous)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gpu-ray_trace-rust_amd"))
import bench  # noqa: E402
from rt_amd import render  # noqa: E402

SCENE = sys.argv[1] if len(sys.argv) > 1 else "spaceship_r1"
GRID = int(sys.argv[2]) if len(sys.argv) > 2 else 20
SORT = int(os.environ.get("SORT", "0"))
PAD = os.environ.get("PAD", "rigorous")
SIZES = (4, 8, 16, 32)
EPS, HIT_MIN, U = np.float32(1e-4), np.float32(2e-3), 2.0 ** -24

_, L = bench.load(SCENE)
n_elems = L.desc.n_elems
tris = [np.asarray(p.poses, np.float32).reshape(-1, 3)[np.asarray(p.indices, np.uint32).reshape(-1, 3)]
        for m in L.scene.meshes for p in m.prims]
T = np.concatenate(tris) if tris else np.zeros((0, 3, 3), np.float32)
V0, E1, E2 = T[:, 0], T[:, 1] - T[:, 0], T[:, 2] - T[:, 0]
NRM = np.cross(E1.astype(np.float64), E2.astype(np.float64))
kd = render.KdTree(L.desc, L.info.kd_tree_depth)
nodes, refs, bounds = kd.nodes, kd.refs, kd.bounds
TLO, THI = T.min(1), T.max(1)
st = {"rays": 0, "leaf_visits": 0, "tri_tests": 0, "viol": 0, **{f"c{c}": 0 for c in SIZES}}
pads = []


def mt(o, d, idx):
    e1, e2, v0 = E1[idx], E2[idx], V0[idx]
    p = np.cross(d, e2)
    det = np.einsum("ij,ij->i", e1, p)
    ok = ~(np.abs(det) < EPS)
    inv = np.float32(1) / np.where(ok, det, np.float32(1))
    s = o - v0
    u = inv * np.einsum("ij,ij->i", s, p)
    q = np.cross(s, e1)
    v = inv * (q @ d)
    t = inv * np.einsum("ij,ij->i", e2, q)
    return ok & (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= EPS), t


def seg_box(o, d, lo, hi, tmax):
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / np.where(np.abs(d) < 1e-30, 1e-30, d)
        ta, tb = (lo - o) * inv, (hi - o) * inv
    tn, tf = np.minimum(ta, tb).max(), np.maximum(ta, tb).min()
    return tn <= tf and tf >= 0 and tn <= tmax


def pad(o, d, sl, lo, hi):
    if PAD == "loose":
        return 1e-3 * float((hi - lo).max()) + 1e-6
    c, h = (lo + hi) / 2, (hi - lo) / 2
    s = np.linalg.norm(o - c) + np.linalg.norm(h)
    dd = float(np.abs(d).sum())
    nn = np.linalg.norm(NRM[sl], axis=1)
    en = np.maximum(np.linalg.norm(E1[sl], axis=1), np.linalg.norm(E2[sl], axis=1))
    cb = 0.0
    if nn.min() > 0:
        nu = NRM[sl] / nn[:, None]
        ax = (nu * np.sign(nu @ nu[0])[:, None]).sum(0)
        ax /= np.linalg.norm(ax)
        cosa = np.abs(nu @ ax).min()
        dn = d / np.linalg.norm(d)
        cphi = abs(dn @ ax)
        cb = cphi * cosa - np.sqrt(max(0.0, 1 - cphi ** 2)) * np.sqrt(max(0.0, 1 - cosa ** 2))
    # per triangle |det_i| >= max(EPS, |d| |n_i| cb); delta_i = E_i (dU + dV),
    # dU <= (7u |d| E_i^2 + 8u S |d| E_i) / |det_i| + 2u; the cluster's pad is the max
    det_i = np.maximum(1e-4, 0.99 * np.linalg.norm(d) * nn * cb)
    di = U * (14 * en ** 3 * dd + 15.5 * s * dd * en ** 2) / det_i + 4 * U * en
    return 1.25 * float(di.max()) + 8 * U * float(np.abs(np.concatenate([lo, hi])).max())


def morton(tr):
    cen = T[tr].mean(1)
    lo, hi = cen.min(0), cen.max(0)
    q = ((cen - lo) / np.maximum(hi - lo, 1e-9) * 1023).astype(np.int64)

    def spread(x):
        r = np.zeros_like(x)
        for b in range(10):
            r |= ((x >> b) & 1) << (3 * b)
        return r

    return tr[np.argsort(spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2), kind="stable")]


def by_normal(tr):
    """Grouped by normal direction (sign-free: the axis of largest |n| made positive, then
    binned 8 x 8 on the other two components), Morton order of centroids within a bin."""
    n = NRM[tr] / np.maximum(np.linalg.norm(NRM[tr], axis=1), 1e-30)[:, None]
    k = np.abs(n).argmax(1)
    n = n * np.sign(n[np.arange(len(n)), k])[:, None]
    oth = np.stack([n[np.arange(len(n)), (k + 1) % 3], n[np.arange(len(n)), (k + 2) % 3]], 1)
    b = np.clip(((oth + 1) * 4).astype(np.int64), 0, 7)
    key = k * 64 + b[:, 0] * 8 + b[:, 1]
    m = morton(tr)
    rank = np.empty(len(tr), np.int64)
    rank[np.searchsorted(np.sort(tr), m)] = np.arange(len(tr))  # Morton rank of each ref
    pos = rank[np.searchsorted(np.sort(tr), tr)]
    return tr[np.lexsort((pos, key))]


def leaf(o, d, lrefs, exit_t):
    tr = lrefs[lrefs >= n_elems] - n_elems
    if len(tr) == 0:
        return None
    if SORT == 1:
        tr = morton(tr)
    elif SORT == 2:
        tr = by_normal(tr)
    st["tri_tests"] += len(tr)
    h, t = mt(o, d, tr)
    rel = h & (t >= HIT_MIN) & (t <= exit_t + EPS)
    tmax = exit_t + EPS
    for size in SIZES:
        n, left = len(tr), 0
        nc = (n + size - 1) // size
        for c in range(nc):
            sl = tr[c * size:(c + 1) * size]
            lo, hi = TLO[sl].min(0), THI[sl].max(0)
            p = pad(o, d, sl, lo, hi)
            if size == 8:
                pads.append(p)
            hit = seg_box(o, d, lo - p, hi + p, tmax * (1 + 1e-6) + p)
            left += len(sl) if hit else 0
            if not hit and rel[c * size:(c + 1) * size].any():
                st["viol"] += 1
        st[f"c{size}"] += left + (nc if n > size else 0)
    ok = h & (t >= HIT_MIN)
    return float(t[ok].min()) if ok.any() else None


def trace(o, d):
    tn, tf = -np.inf, np.inf
    for a in range(3):
        dd = d[a] if abs(d[a]) > 1e-30 else 1e-30
        ta, tb = (bounds[2 * a] - o[a]) / dd, (bounds[2 * a + 1] - o[a]) / dd
        tn, tf = max(tn, min(ta, tb)), min(tf, max(ta, tb))
    if tn > tf or tf < 0:
        return
    stack = [(0, tn, tf)]
    while stack:
        ni, en, ex = stack.pop()
        while True:
            a, b = int(nodes[ni, 0]), int(nodes[ni, 1])
            if (b & 3) == 3:
                break
            ax = b & 3
            dd = d[ax] if abs(d[ax]) >= EPS else (-EPS if d[ax] < 0 else EPS)
            t = (np.uint32(a).view(np.float32) - o[ax]) / dd
            near, far = ((b >> 2), (b >> 2) + 1) if dd > 0 else ((b >> 2) + 1, (b >> 2))
            if t >= ex:
                ni = near
            elif t <= en:
                ni = far
            else:
                stack.append((far, t, ex))
                ni, ex = near, t
        st["leaf_visits"] += 1
        best = leaf(o, d, refs[(b >> 2):(b >> 2) + a], ex)
        if best is not None and best <= ex + EPS:
            return


cam = L.cam
w, h = int(L.info.width), int(L.info.height)
cd, co, up = (np.array(v, np.float32) for v in (cam.d, cam.o, cam.up))
right = np.cross(cd / np.linalg.norm(cd), up)
right /= np.linalg.norm(right)
for yy in np.linspace(0, h - 1, GRID).astype(int):
    for xx in np.linspace(0, w - 1, 2 * GRID).astype(int):
        d = cd + cam.screen_width / w * (xx - w / 2) * right + cam.screen_height / h * (yy - h / 2) * up
        st["rays"] += 1
        trace(co.copy(), (d / np.linalg.norm(d)).astype(np.float32))
r = st["rays"]
out = {"scene": SCENE, "pad": PAD, "order": ["leaf", "morton", "normal bins + morton"][SORT], "rays": r, "viol": st["viol"],
       "tri_tests_per_ray": round(st["tri_tests"] / r, 1), "leaf_visits_per_ray": round(st["leaf_visits"] / r, 2),
       **{f"tests_left_c{c}": round(st[f"c{c}"] / r, 1) for c in SIZES},
       "pad_c8_pctl_50_90_99": [round(float(x), 4) for x in np.percentile(pads, [50, 90, 99])] if pads else None,
       "scene_bounds": [float(x) for x in bounds]}
print(json.dumps(out))
