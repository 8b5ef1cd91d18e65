"""Prices skipping, in a leaf visit, the tests of primitives the ray's previous leaf also held
("Shared refs"): the same ray against the same triangle gives the same length, so
the leaf's first strict minimum (closest_hit.rs:6-30) can often be decided from its own other
refs plus the previous leaf's minimum key, which the cooperative search already carries
(RT_LEAF_REUSE).  Per leaf visit L after a leaf P:
  - S = refs(L) & refs(P) (both lists are ascending renderable indices), T = refs(L) - S;
  - m1 = first strict minimum over T, lP = P's minimum (over all of P);
  - every hit in S is >= lP (S is part of P), so: no hit in P -> L's minimum is m1; m1 < lP ->
    it is m1; P's minimum primitive in S -> it is min(m1, lP) (a tie m1 == lP falls back);
    otherwise S must be tested too (fallback).
Rays: the camera's primary rays on a grid and, from each primary hit, one secondary ray in a
random direction of the hit's outer hemisphere (the cooperative search's main traffic).
Checks each decided minimum against the full leaf test; counts tests, skips, fallbacks and the
distinct (L, P) pairs a per-pair membership mask would need.
Usage: python tools/shared_refs.py [scene] [grid]"""
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
GRID = int(sys.argv[2]) if len(sys.argv) > 2 else 16
EPS, HIT_MIN = np.float32(1e-4), np.float32(2e-3)

_, L = bench.load(SCENE)
n_elems = L.desc.n_elems
tris = [np.asarray(p.poses, np.float32).reshape(-1, 3)[np.asarray(p.indices, np.uint32).reshape(-1, 3)]
        for m in L.scene.meshes for p in m.prims]
T = np.concatenate(tris) if tris else np.zeros((0, 3, 3), np.float32)
V0, E1, E2 = T[:, 0], T[:, 1] - T[:, 0], T[:, 2] - T[:, 0]
NRM = np.cross(E1.astype(np.float64), E2.astype(np.float64))
SPH = []
for k, i in [(int(e.kind), int(e.index)) for e in L.desc.elems[:n_elems]]:
    if k == 0:
        s = L.desc.spheres[i]
        SPH.append((np.array(s.c[:], np.float32), np.float32(s.r)))
    else:
        SPH.append(None)
kd = render.KdTree(L.desc, L.info.kd_tree_depth)
nodes, refs, bounds = kd.nodes, kd.refs, kd.bounds
PARENT = np.full(len(nodes), -1, np.int64)
for i in range(len(nodes)):
    if (int(nodes[i, 1]) & 3) != 3:
        c = int(nodes[i, 1]) >> 2
        PARENT[c] = PARENT[c + 1] = i


def lca_up(a, b):
    """levels from leaf b up to the lowest common ancestor of leaves a and b."""
    anc = set()
    x = a
    while x >= 0:
        anc.add(x)
        x = PARENT[x]
    k, x = 0, b
    while x not in anc:
        x, k = PARENT[x], k + 1
    return k
# renumbering of the primitives by first appearance in the leaf lists (depth-first leaf order)
NEWID = np.full(int(refs.max()) + 1 if len(refs) else 1, -1, np.int64)
_n = 0
_stk = [0]
while _stk:
    _i = _stk.pop()
    _a, _b = int(nodes[_i, 0]), int(nodes[_i, 1])
    if (_b & 3) == 3:
        for _r in refs[(_b >> 2):(_b >> 2) + _a]:
            if NEWID[_r] < 0:
                NEWID[_r] = _n
                _n += 1
    else:
        _stk.append((_b >> 2) + 1)
        _stk.append(_b >> 2)
UP = {}
st = {"rays": 0, "leaf_visits": 0, "tests": 0, "reuse_tests": 0, "after_leaf": 0, "shared": 0, "decided_no_hit": 0,
      "decided_m1": 0, "decided_pmin_in_s": 0, "fallback": 0, "fallback_tests": 0, "mismatch": 0}
pairs = set()


def hits(o, d, rr):
    """lengths of every ref in rr (inf where no valid hit), the reference's tests in float32."""
    out = np.full(len(rr), np.inf, np.float32)
    tr = rr >= n_elems
    if tr.any():
        idx = rr[tr] - n_elems
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
        h = ok & (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= EPS) & (t >= HIT_MIN)
        out[np.where(tr)[0][h]] = t[h]
    for j in np.where(~tr)[0]:
        c, r = SPH[int(rr[j])]
        oc = o - c
        b = np.float32(np.dot(oc, d))
        disc = b * b - (np.float32(np.dot(oc, oc)) - r * r)
        if disc > 0:
            sq = np.sqrt(disc)
            l0, l1 = -b + sq, -b - sq
            ln = l1 if l1 > 0 else l0
            if l0 > 0 and ln >= HIT_MIN:
                out[j] = ln
    return out


def first_min(ls):
    if not np.isfinite(ls).any():
        return None
    j = int(np.argmin(ls))  # first index of the minimum
    return j, float(ls[j])


def trace(o, d):
    tn, tf = -np.inf, np.inf
    for a in range(3):
        dd = d[a] if abs(d[a]) > 1e-30 else 1e-30
        ta, tb = (bounds[2 * a] - o[a]) / dd, (bounds[2 * a + 1] - o[a]) / dd
        tn, tf = max(tn, min(ta, tb)), min(tf, max(ta, tb))
    if tn > tf or tf < 0:
        return None
    stack = [(0, tn, tf)]
    prev = None  # (leaf offset, refs, first-min (pos, l) or None)
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
        off, cnt = b >> 2, a
        rl = refs[off:off + cnt]
        leaf_node = ni
        st["leaf_visits"] += 1
        st["tests"] += cnt
        ls = hits(o, d, rl)
        fm = first_min(ls)
        if prev is not None and cnt:
            poff, prl, pfm, pnode = prev
            if poff == off:
                st["reuse_tests"] += cnt  # leaf-minimum reuse (identical lists) already skips these
            else:
                st["after_leaf"] += cnt
                sh = np.isin(rl, prl)
                ns = int(sh.sum())
                st["shared"] += ns
                k = lca_up(pnode, leaf_node)
                UP[k] = UP.get(k, 0) + ns
                for wsz in (64, 128, 256):
                    st[f"shared_in_window{wsz}"] = st.get(f"shared_in_window{wsz}", 0) + int((sh & ((rl.astype(np.int64) - int(prl[0])) < wsz)).sum())
                    nb = int(NEWID[prl].min())
                    st[f"shared_in_window{wsz}_renum"] = st.get(f"shared_in_window{wsz}_renum", 0) + int((sh & ((NEWID[rl] - nb) < wsz)).sum())
                if ns:
                    pairs.add((off, poff))
                    m1 = first_min(np.where(sh, np.inf, ls))
                    if pfm is None:
                        st["decided_no_hit"] += 1
                        dec = m1
                    elif m1 is not None and m1[1] < pfm[1]:
                        st["decided_m1"] += 1
                        dec = m1
                    elif (int(prl[pfm[0]]) in set(rl[sh].tolist())) and not (m1 is not None and m1[1] == pfm[1]):
                        st["decided_pmin_in_s"] += 1
                        jp = int(np.where(rl == prl[pfm[0]])[0][0])
                        dec = m1 if (m1 is not None and m1[1] < pfm[1]) else (jp, pfm[1])
                    else:
                        st["fallback"] += 1
                        st["fallback_tests"] += ns
                        dec = fm
                    if (dec is None) != (fm is None) or (dec is not None and (dec[0] != fm[0] or dec[1] != fm[1])):
                        st["mismatch"] += 1
        prev = (off, rl, fm, leaf_node)
        if fm is not None and fm[1] <= ex + EPS:
            return fm[1], int(rl[fm[0]])
    return None


cam = L.cam
w, h = int(L.info.width), int(L.info.height)
cd, co, up = (np.array(v, np.float32) for v in (cam.d, cam.o, cam.up))
right = np.cross(cd / np.linalg.norm(cd), up)
right /= np.linalg.norm(right)
rng = np.random.default_rng(7)
for yy in np.linspace(0, h - 1, GRID).astype(int):
    for xx in np.linspace(0, w - 1, 2 * GRID).astype(int):
        d = cd + cam.screen_width / w * (xx - w / 2) * right + cam.screen_height / h * (yy - h / 2) * up
        d = (d / np.linalg.norm(d)).astype(np.float32)
        st["rays"] += 1
        hit = trace(co.copy(), d)
        if hit is None or hit[1] < n_elems:
            continue
        n = NRM[hit[1] - n_elems]
        n = n / np.linalg.norm(n)
        if np.dot(n, d) > 0:
            n = -n
        pos = (co + d * np.float32(hit[0]) + n * 1e-4).astype(np.float32)
        v = rng.normal(size=3)
        v /= np.linalg.norm(v)
        if np.dot(v, n) < 0:
            v = -v
        st["rays"] += 1
        trace(pos, v.astype(np.float32))
tests = st["tests"]
skipped = st["shared"] - st["fallback_tests"]
out = {"scene": SCENE, **st, "shared_by_lca_levels": {k: UP[k] for k in sorted(UP)}, "distinct_leaf_pairs": len(pairs),
       "share_of_tests_skippable": round(skipped / max(tests - st["reuse_tests"], 1), 3),
       "fallback_per_shared_visit": round(st["fallback"] / max(st["decided_no_hit"] + st["decided_m1"]
                                                              + st["decided_pmin_in_s"] + st["fallback"], 1), 3)}
print(json.dumps(out))
