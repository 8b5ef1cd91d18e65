"""include/rt_libm.h — the device's sinf, cosf and powf(x, 5) — against the C library the
reference's f32::sin/cos/powf call on Linux (glibc), bit for bit.

CPU: lib/check_libm (gcc build of the same header) over every angle 2*pi*v the renderer forms
and 2^24 powf inputs; the exhaustive pass (every float in [-2 pi, 2 pi] and in [0, 1.001]) is
`check_libm full`, recorded in DESIGN.md §3.  GPU: lib/check_libm_gpu computes on gfx950 and
compares on the host."""
import json
import os
import subprocess

import pytest

from conftest import PKG

LIB = os.path.join(PKG, "lib")


def _run(exe, *args, timeout=300):
    path = os.path.join(LIB, exe)
    if not os.path.exists(path):
        pytest.fail(f"{path} is not built (make -C gpu-ray_trace-rust_amd)")
    p = subprocess.run([path, *args], capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout + p.stderr
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_libm_restatement_matches_glibc_cpu():
    r = _run("check_libm", "quick")
    assert r["angles_2pi_v"][:2] == [1 << 24, 0], r
    assert r["powf5_sample"][1] == 0, r


@pytest.mark.gpu
def test_libm_restatement_matches_glibc_on_gfx950(gpu_available):
    r = _run("check_libm_gpu", timeout=120)
    assert r["angles_2pi_v"][1] == 0 and r["hashed_pm2pi"][1] == 0 and r["powf5"][1] == 0, r


def test_libm_restatement_exhaustive_cpu():
    """Every float in [-2 pi, 2 pi] (sinf, cosf) and in [0, 1.001] / [-0.001, 0] (powf(x, 5)):
    4.2e9 inputs, bit for bit (about 10 s on 8 cores)."""
    r = _run("check_libm", "full", timeout=600)
    assert r["sincos_all_floats_pm2pi"][1] == 0 and r["powf5_all_floats"][1] == 0, r


def test_powf5_every_float_cpu():
    """powf(x, 5) on all 2^32 float bit patterns (negative, subnormal, zero, inf, NaN and the
    overflow / underflow range included), bit for bit against glibc (about 10 s on 8 cores)."""
    r = _run("check_libm", "pow_all", timeout=900)
    assert r["powf5_every_float"] == [1 << 32, 0, "0x00000000"], r
    # the glibc algorithm alone is exact too, and the fast path (x^5 in double, round 4) serves
    # over 99% of its range [2^-25, 2]
    assert r["glibc_path_mismatches"] == 0, r
    assert r["fast_path_taken"] > 0.99 * r["fast_path_range"], r
