"""The shipped library's gfx950 code object, read on the CPU: every kernel the runtime can
launch has a real body.  A kernel the compiler reduced to `s_endpgm` (undefined behaviour, or a
branch that made the work unreachable) renders nothing and returns success; the GPU parity tests
catch that only for the scenes that reach it, so this checks every instantiation at build time.
Format: the .hip_fatbin section is a clang offload bundle ("__CLANG_OFFLOAD_BUNDLE__", entry
count, then offset / size / target triple per entry) holding an AMDGPU ELF per target."""
import os
import struct

import pytest

from conftest import PKG


def _sections(b):
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    names = secs[shstrndx][4]
    return {b[names + s[0]: b.index(b"\0", names + s[0])].decode(): s for s in secs}


def _gfx950_object(lib_path):
    b = open(lib_path, "rb").read()
    s = _sections(b)[".hip_fatbin"]
    fb = b[s[4]: s[4] + s[5]]
    assert fb.startswith(b"__CLANG_OFFLOAD_BUNDLE__")
    n, = struct.unpack_from("<Q", fb, 24)
    off = 32
    for _ in range(n):
        o, size, tl = struct.unpack_from("<QQQ", fb, off)
        triple = fb[off + 24: off + 24 + tl].decode()
        off += 24 + tl
        if triple.endswith("gfx950"):
            return fb[o: o + size]
    raise AssertionError("no gfx950 code object in the bundle")


def _kernel_sizes(elf):
    """{symbol: size in bytes} of the code object's functions (STT_FUNC)."""
    secs = _sections(elf)
    symtab, strtab = secs[".symtab"], secs[".strtab"]
    out = {}
    for i in range(symtab[5] // 24):
        name_off, info, _other, _shndx, _value, size = struct.unpack_from("<IBBHQQ", elf, symtab[4] + 24 * i)
        if info & 0xF == 2:  # STT_FUNC
            out[elf[strtab[4] + name_off: elf.index(b"\0", strtab[4] + name_off)].decode()] = size
    return out


def test_every_kernel_has_a_body():
    from rt_amd import abi

    sizes = _kernel_sizes(_gfx950_object(abi.LIB_PATH))
    queue = {k: v for k, v in sizes.items() if "queue_kernel" in k}
    # queue_kernel<GEN, DLS, RESTART, STARTS>: general and DLS, each with the stack and the
    # stackless traversal; sphere-only the same, each with batched and per-lane path starts
    # (round 6: the measured-slower LDS slab and pool kernels are gone)
    assert len(queue) == 8, sorted(queue)
    for name, size in sorted(sizes.items()):
        if "kernel" in name:
            assert size > 256, f"{name}: {size} B of code (an empty kernel is 4)"
    assert min(queue.values()) > 8192, queue


def test_u8_over_255_markstein_is_exact(tmp_path):
    """trace.hip u8_over_255: the texel decode of the 8-bit pool, q0 = k * r, q = fma(fma(-q0,
    255, k), r, q0) with r = RN(1 / 255), equals the IEEE k / 255.0f (image::to_rgb32f's value)
    for every k in 0..255, so the 8-bit pool renders the f32 pool's bits.  C fmaf is correctly
    rounded (glibc), as v_fma_f32 is."""
    import subprocess

    src = tmp_path / "u8.c"
    src.write_text(r'''
#include <math.h>
#include <stdio.h>
#include <string.h>
int main(void) {
    const float r = 0x1.010102p-8f;
    if (r != 1.0f / 255.0f) return 2;
    int bad = 0;
    for (unsigned k = 0; k < 256; ++k) {
        float a = (float)k, q0 = a * r;
        float q = fmaf(fmaf(-q0, 255.0f, a), r, q0);
        if (k == 0) q = a;  /* div_mk's zero case */
        float want = (float)k / 255.0f;
        if (memcmp(&q, &want, 4)) bad++;
    }
    printf("%d\n", bad);
    return bad != 0;
}
''')
    exe = tmp_path / "u8"
    subprocess.run(["gcc", "-O0", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "0", r.stdout


def test_shipped_library_has_no_device_printf():
    """The diagnostic instrumentation (csrc/kernel/diag.h: clock reads, counters, printf) is
    compiled only into `make diag`'s libraries.  A device printf makes the kernel take the
    hostcall buffer (metadata `hidden_hostcall_buffer`); the shipped code object must have none.
    When the diagnostic libraries are built, they are checked to carry it, so the probe can see
    a printf when there is one."""
    import os

    from rt_amd import abi

    assert b"hostcall" not in _gfx950_object(abi.LIB_PATH)
    assert b"printf" not in _gfx950_object(abi.LIB_PATH)
    diag = os.path.join(os.path.dirname(abi.LIB_PATH), "variants", "librt_diag_timing.so")
    if os.path.exists(diag):
        assert b"hostcall" in _gfx950_object(diag)


def test_in_return_leaf_quotient_bracket():
    """trace.hip in_return_leaf (round 4) compares the face distances through q = RN(n * RN(1 / d))
    and the bounds fma(|q|, 2^-21, q) (upper) / fma(-|q|, 2^-21, q) (lower) instead of the exact
    quotient RN(n / d) the traversal computes: the exact quotient must lie inside the bracket for
    every n and every clamped direction d (|d| in [EPS, 1]).  Checked on 2^24 random pairs spread
    over the exponents the scenes reach (|n| in [2^-40, 2^60]) plus powers of two and ties."""
    import numpy as np

    rng = np.random.default_rng(7)
    N = 1 << 24
    n = (rng.uniform(1, 2, N) * 2.0 ** rng.integers(-40, 60, N)).astype(np.float32)
    n *= np.where(rng.integers(0, 2, N) == 1, 1, -1).astype(np.float32)
    d = (rng.uniform(1, 2, N) * 2.0 ** rng.integers(-14, 0, N)).astype(np.float32)  # [2^-14, 1) >= EPS
    d = np.clip(d, np.float32(1e-4), np.float32(1.0)) * np.where(rng.integers(0, 2, N) == 1, 1, -1).astype(np.float32)
    n[:64] = np.float32(2.0) ** np.arange(-32, 32, dtype=np.float32)
    d[:64] = np.float32(1e-4)
    rc = (np.float32(1.0) / d).astype(np.float32)
    q = (n * rc).astype(np.float32)
    t = (n / d).astype(np.float32)  # the traversal's quotient (correctly rounded)
    # fmaf(|q|, 2^-21, +-q): exact in double (24 + 21 bits), then one rounding to float
    aq = np.abs(q).astype(np.float64) * 2.0 ** -21
    up = (q.astype(np.float64) + aq).astype(np.float32)
    lo = (q.astype(np.float64) - aq).astype(np.float32)
    assert np.all(t <= up) and np.all(t >= lo)


@pytest.mark.gpu
def test_exact_arithmetic_identities_on_gfx950(gpu_available):
    """lib/check_exact_ops (tools/check_exact_ops.hip) on the GPU: rcp_exact over every normal
    |b| in [2^-60, 2^60], the Markstein quotient on 4.3e9 random pairs and 2.1e9 normalize-shaped
    ones, sincosf == (sinf, cosf) on every angle a draw forms, and both square roots — the
    v_sqrt_f32 fix-up and the kernel's sqrt_rn (x * rsq(x) with one FMA correction) — on every
    float in [2^-80, FLT_MAX]: 0 mismatches against the IEEE operations."""
    import json
    import subprocess

    exe = os.path.join(PKG, "lib", "check_exact_ops")
    if not os.path.exists(exe):
        pytest.fail("lib/check_exact_ops not built (make -C gpu-ray_trace-rust_amd)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("rcp_exact_all_normal_2^-60_2^60", "markstein_div_random_pairs", "normalize_quotients",
              "sincosf_vs_sinf_cosf", "sqrt_fix_2^-80_to_inf", "sqrt_rn_rsq_2^-80_to_max"):
        assert d[k]["tested"] > 0 and d[k]["bad"] == 0, (k, d[k])
    assert d["sqrt_rn_rsq_2^-80_to_max"]["tested"] == (0x7F7FFFFF - (47 << 23) + 1), d
    assert r.returncode == 0, r.stdout[-500:]
