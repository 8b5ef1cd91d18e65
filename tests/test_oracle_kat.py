"""The reference's own unit tests, restated against the oracle, plus known-answer checks.

src/accel/aabb.rs:66-121 (slab test), src/ray/hit.rs:90-140 (RayLen ordering),
src/render/target.rs:17-46 (chunk_to_pix).  These are the only golden vectors the reference
holds for the hot path; they pin the oracle's slab test, NaN ordering and
pixel indexing.
"""
import ctypes as C
import math

import numpy as np
import pytest

INF, NAN = float("inf"), float("nan")
CUBE = [-1.0, 1.0, -1.0, 1.0, -1.0, 1.0]


def f32(*v):
    return np.array(v, dtype=np.float32)


def entry_exit(oracle, bounds, d, o):
    b, dd, oo = f32(*bounds), f32(*d), f32(*o)
    ma, xa = C.c_int(), C.c_int()
    en, ex = C.c_float(), C.c_float()
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    hit = oracle.lib().oracle_aabb_entry_exit(fp(b), fp(dd), fp(oo), C.byref(ma), C.byref(en), C.byref(xa),
                                              C.byref(ex))
    return ((ma.value, en.value), (xa.value, ex.value)) if hit else None


# ---- aabb.rs:71-91 test_straight_axes (the reference loops a in 1..3: y and z only)
@pytest.mark.parametrize("a", [1, 2])
def test_straight_axes(oracle, a):
    d = [0.0, 0.0, 0.0]
    d[a] = 1.0
    o = [-3.0 * x for x in d]
    assert entry_exit(oracle, CUBE, d, o) == ((a, 2.0), (a, 4.0))


# ---- aabb.rs:93-106 test_xy_hits_both
def test_xy_hits_both(oracle):
    got = entry_exit(oracle, CUBE, [2.1, 1.0, 0.0], [-2.0, 0.0, 0.0])
    assert got[0][0] == 0 and got[1] == (1, 1.0)
    assert got[0][1] == float(np.float32(1.0) / np.float32(2.1))  # 1.0/2.1 in f32


# ---- aabb.rs:108-121 test_parallel_x
def test_parallel_x(oracle):
    assert entry_exit(oracle, CUBE, [1.0, 0.1, 0.0], [0.0, 1.1, 0.0]) is None


# ---- hit.rs:94-140 RayLen ordering
@pytest.mark.parametrize("a,b,want", [
    (-1.0, 1.0, -1),          # test_less_than
    (1.0, -1.0, 1),           # test_greater_than
    (1.34324, 1.34324, 0),    # test_eq
    (NAN, NAN, 0),            # test_nan_eq
    (INF, INF, 0),            # test_inf_eq
    (NAN, INF, 1),            # test_nan_inf_lt (me > them)
    (INF, NAN, -1),           # test_nan_inf_lt (me < them)
])
def test_raylen_order(oracle, a, b, want):
    assert oracle.lib().oracle_raylen_cmp(a, b) == want


# ---- target.rs:23-46 test_renderer_chunk_to_pix (400 x 500)
def test_chunk_to_pix(oracle):
    w, h = 400, 500
    x, y = C.c_int32(), C.c_int32()
    for idx, want in [(0, (0, 0)), (w - 1, (w - 1, 0)), (h * w - 1, (w - 1, h - 1)), ((h - 1) * w, (0, h - 1))]:
        oracle.lib().oracle_chunk_to_pix(idx, w, C.byref(x), C.byref(y))
        assert (x.value, y.value) == want


# ---- beyond the reference's tests: hand-derived known answers
def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def test_sphere_known_answers(oracle):
    l = C.c_float()
    c, d = f32(0, 0, -5), f32(0, 0, -1)
    assert oracle.lib().oracle_sphere_intersect(_fp(c), 1.0, _fp(d), _fp(f32(0, 0, 0)), C.byref(l)) == 1
    assert l.value == 4.0                       # near root of (5 -/+ 1)
    # from inside: only the far root is positive (sphere.rs:95)
    assert oracle.lib().oracle_sphere_intersect(_fp(c), 1.0, _fp(d), _fp(f32(0, 0, -5)), C.byref(l)) == 1
    assert l.value == 1.0
    # tangent ray: disc == 0 is a miss (sphere.rs:90, strict >)
    assert oracle.lib().oracle_sphere_intersect(_fp(c), 1.0, _fp(d), _fp(f32(1, 0, 0)), C.byref(l)) == 0
    # behind the ray
    assert oracle.lib().oracle_sphere_intersect(_fp(c), 1.0, _fp(-d), _fp(f32(0, 0, 0)), C.byref(l)) == 0


def test_triangle_known_answers(oracle):
    v = f32(0, 0, -2, 1, 0, -2, 0, 1, -2)
    l, u, w = C.c_float(), C.c_float(), C.c_float()
    o, d = f32(0.25, 0.25, 0), f32(0, 0, -1)
    assert oracle.lib().oracle_triangle_intersect(_fp(v), _fp(d), _fp(o), C.byref(l), C.byref(u), C.byref(w)) == 1
    assert (l.value, u.value, w.value) == (2.0, 0.25, 0.25)
    # double sided (generic.rs: det sign is not tested)
    o2, d2 = f32(0.25, 0.25, -4), f32(0, 0, 1)
    assert oracle.lib().oracle_triangle_intersect(_fp(v), _fp(d2), _fp(o2), C.byref(l), C.byref(u), C.byref(w)) == 1
    assert l.value == 2.0
    # outside (u + v > 1) and parallel (|det| < EPS)
    o3 = f32(0.75, 0.75, 0)
    assert oracle.lib().oracle_triangle_intersect(_fp(v), _fp(d), _fp(o3), C.byref(l), C.byref(u), C.byref(w)) == 0
    d4 = f32(1, 0, 0)
    assert oracle.lib().oracle_triangle_intersect(_fp(v), _fp(d4), _fp(o), C.byref(l), C.byref(u), C.byref(w)) == 0
    # hit closer than EPS is rejected (generic.rs:129)
    o5 = f32(0.25, 0.25, -2.00005)
    assert oracle.lib().oracle_triangle_intersect(_fp(v), _fp(d), _fp(o5), C.byref(l), C.byref(u), C.byref(w)) == 0


def test_refract_fresnel_quirk(oracle):
    """interaction.rs:50 uses (1 + r0), so re can exceed the physical reflectance."""
    d, n = f32(0, -1, 0), f32(0, 1, 0)  # head-on, entering glass 1.0 -> 1.3
    out, p = f32(0, 0, 0), C.c_float()
    oracle.lib().oracle_refract(_fp(d), _fp(n), 1.0, 1.3, 0.999, _fp(out), C.byref(p))
    r0 = np.float32(((np.float32(1.0) - np.float32(1.3)) / (np.float32(1.0) + np.float32(1.3)))) ** 2
    # c = 1 - c1 = 0 -> re = r0; transmitted with p = 1 - re, straight through
    assert out.tolist() == [0.0, -1.0, 0.0]
    assert math.isclose(p.value, 1.0 - float(r0), rel_tol=1e-6)
    # grazing: c -> 1, re = r0 + (1 + r0) > 1, so the transmit branch would carry p < 0
    d2 = f32(1.0, -0.003, 0)
    d2 = d2 / np.sqrt(np.float32(d2 @ d2))
    oracle.lib().oracle_refract(_fp(d2.astype(np.float32)), _fp(n), 1.0, 1.3, 0.0, _fp(out), C.byref(p))
    assert p.value > 1.0  # reflected with p = re > 1


def test_rng_stream_contract(oracle):
    """rt_rng.h: 24-bit floats in [0, 1), independent of call order, keyed on (seed, pixel, sample)."""
    out = np.zeros(4096, np.float32)
    oracle.lib().oracle_rng_stream(0x5EED0001, 7, 3, 4096, _fp(out))
    assert out.min() >= 0.0 and out.max() < 1.0
    assert np.all((out * (1 << 24)) == np.floor(out * (1 << 24)))
    assert abs(out.mean() - 0.5) < 0.02
    again = np.zeros(4096, np.float32)
    oracle.lib().oracle_rng_stream(0x5EED0001, 7, 3, 4096, _fp(again))
    assert np.array_equal(out, again)
    other = np.zeros(4096, np.float32)
    oracle.lib().oracle_rng_stream(0x5EED0001, 8, 3, 4096, _fp(other))
    assert not np.array_equal(out, other)


def _mix64(z):
    m = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def test_rng_is_xoroshiro64star(oracle):
    """rt_rng.h's draws are the published xoroshiro64* (Blackman & Vigna 2018: out = s0 * 0x9E3779BB;
    s1 ^= s0; s0 = rotl(s0, 26) ^ s1 ^ (s1 << 9); s1 = rotl(s1, 13)) started at the SplitMix64 hash of
    (seed, pixel, sample), mapped to f32 as rand 0.8's Standard: (u32 >> 8) * 2^-24 — restated here
    in plain Python integers."""
    m32, m64 = (1 << 32) - 1, (1 << 64) - 1
    rotl = lambda x, k: ((x << k) | (x >> (32 - k))) & m32  # noqa: E731
    for seed, pixel, sample in ((0x5EED0001, 7, 3), (0, 0, 0), (2**64 - 1, 719_999, 2**40 + 5)):
        key = _mix64((seed + 0x9E3779B97F4A7C15 * (pixel + 1)) & m64)
        st = _mix64(key ^ sample) or 0x9E3779B97F4A7C15
        s0, s1 = st & m32, st >> 32
        want = []
        for _ in range(64):
            out = (s0 * 0x9E3779BB) & m32
            want.append(np.float32((out >> 8) * 2.0**-24))
            s1 ^= s0
            s0 = rotl(s0, 26) ^ s1 ^ ((s1 << 9) & m32)
            s1 = rotl(s1, 13)
        got = np.zeros(64, np.float32)
        oracle.lib().oracle_rng_stream(C.c_uint64(seed), pixel, C.c_uint64(sample), 64, _fp(got))
        assert np.array_equal(got, np.array(want, np.float32)), (seed, pixel, sample)


def test_rng_stream_statistics(oracle):
    """Uniformity and serial independence of the f32 draws over many (pixel, sample) streams: the
    mean and variance of U[0, 1), lag-1 correlation within a stream and correlation between the
    first draws of neighbouring samples, each within 5 sigma of its expectation."""
    n_streams, L = 4096, 32
    draws = np.zeros((n_streams, L), np.float32)
    for k in range(n_streams):
        oracle.lib().oracle_rng_stream(C.c_uint64(0x5EED0001), k % 64, C.c_uint64(k // 64), L,
                                       _fp(draws[k]))
    x = draws.astype(np.float64)
    n = x.size
    assert abs(x.mean() - 0.5) < 5 * np.sqrt(1 / 12 / n)
    assert abs(x.var() - 1 / 12) < 5 * np.sqrt(1 / 180 / n)
    lag = np.corrcoef(x[:, :-1].ravel(), x[:, 1:].ravel())[0, 1]
    assert abs(lag) < 5 / np.sqrt(n)
    first = x[:, 0].reshape(64, 64)  # [sample][pixel]
    across = np.corrcoef(first[:-1].ravel(), first[1:].ravel())[0, 1]
    assert abs(across) < 5 / np.sqrt(first.size)
