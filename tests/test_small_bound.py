"""The thresholds of the sphere-only kernel's in_return_leaf (trace.hip), on the CPU.

The shortcut compares approximate face distances q (v_rcp_f32 products, within 3 * 2^-23 |q| of
the traversal's quotients) against E' and L', which must fold the 2^-21 margin in:
E' = RN(L* (1 - 2^-17) - 2 EPS (1 + 2^-20)) <= E / (1 + 2^-21), where E = RN(RN(L* - 2 EPS) -
RN(L* 2^-18)) is the descent floor of closest_small, and L' = RN(L* + L* 2^-20) >= L* / (1 - 2^-21),
for every L* >= HIT_MIN = 20 EPS a hit can have.  numpy float32 arithmetic is IEEE round-to-nearest;
the fma is evaluated exactly in float64 (a product of two float32 is exact there) and rounded once
more, which can differ from a true fma only on exact float64 ties, far inside the margins here."""
import numpy as np

F = np.float32
EPS = F(1e-4)
HIT_MIN = EPS * F(20)


def _fma32(a, b, c):
    return (a.astype(np.float64) * np.float64(b) + np.float64(c)).astype(np.float32)


def _ls_values():
    rng = np.random.default_rng(6)
    near = (HIT_MIN * (1 + rng.random(500_000) * 20)).astype(np.float32)
    wide = (10 ** rng.uniform(np.log10(float(HIT_MIN)), 7, 1_000_000)).astype(np.float32)
    edge = np.nextafter(HIT_MIN, F(np.inf)) * np.arange(1, 20001, dtype=np.float32)
    ls = np.concatenate([near, wide, edge, [HIT_MIN]]).astype(np.float32)
    return ls[ls >= HIT_MIN]


def test_descent_floor_threshold_has_the_margin():
    ls = _ls_values()
    e = ((ls - F(2) * EPS).astype(np.float32) - (ls * F(2.0 ** -18)).astype(np.float32)).astype(np.float32)
    assert (e > 0).all()
    en = _fma32(ls, F(1 - 2.0 ** -17), F(-2 * float(EPS) * (1 + 2.0 ** -20)))
    assert (en.astype(np.float64) <= e.astype(np.float64) / (1 + 2.0 ** -21)).all()


def test_far_threshold_has_the_margin():
    ls = _ls_values()
    lf = _fma32(ls, F(2.0 ** -20), ls)
    assert (lf.astype(np.float64) >= ls.astype(np.float64) / (1 - 2.0 ** -21)).all()
