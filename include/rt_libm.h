/*
 * rt_libm.h — sinf, cosf and powf with the results of the C library the reference calls.
 *
 * The reference's transcendentals are Rust's f32 methods: `thet.cos()` / `thet.sin()`
 * (src/material/interaction.rs:22-23, src/ray/generate.rs:58-59) and `c.powf(5.0)`
 * (interaction.rs:50, src/elements/mesh/triangle.rs:204).  On Linux these lower to glibc's
 * sinf, cosf and powf.  glibc 2.35 (the version of this image) implements them with the
 * double-precision algorithms of ARM's optimized-routines (sysdeps/ieee754/flt-32: s_sinf.c,
 * s_cosf.c, sincosf.h, sincosf_data.c, e_powf.c, e_powf_log2_data.c, e_exp2f_data.c); on x86-64
 * CPUs with FMA, glibc's ifunc selects the builds of those files compiled with -mfma, where GCC
 * contracts every single-use product feeding an add into an FMA.  This header restates those
 * fast paths — same tables, same operation order, the same contractions as explicit fma() — so
 * the device computes glibc's float results bit for bit instead of ocml's (which differ by an
 * ulp on some inputs).  Only the ranges the renderer reaches are restated:
 *   - sinf/cosf for |x| < 120 (the renderer's angles are 2*pi*v, v in [0, 1));
 *   - powf(x, 5) for every finite x (the Schlick terms; x in [-eps, 1 + eps]), with a fast path
 *     (x^5 in double, exact where it cannot differ from glibc's rounding: rt_powf5_fast).
 * Outside its range rt_sincosf reports failure (the renderer's angles never leave it).
 * The tables are the values of glibc's __sincosf_table, __powf_log2_data and __exp2f_data.
 *
 * Checked against the C library by tests/test_libm.py (every angle 2*pi*v the RNG can draw,
 * every float in [0, 2*pi] and in [0, 1] for powf(x, 5): tools/check_libm.c) and on the GPU by
 * tools/check_libm_gpu.hip.  Plain C: compiled unchanged by gcc and by hipcc for gfx950 (device
 * functions there).
 *
 * Licence of the restated algorithms and tables: the sinf / cosf / powf code and its data tables
 * come from ARM's optimized-routines, "Copyright (c) 2017-2018, Arm Limited.", distributed with
 * glibc under the GNU Lesser General Public License v2.1 or later (glibc 2.35,
 * sysdeps/ieee754/flt-32) and by Arm under the MIT License (optimized-routines, math/).  The
 * tables below are those published values; the notice above is kept with them.
 */
#ifndef RT_LIBM_H
#define RT_LIBM_H

#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#define RT_LIBM_FN static inline __device__
#define RT_LIBM_TABLE static __constant__ const
#else
#define RT_LIBM_FN static inline
#define RT_LIBM_TABLE static const
#endif

RT_LIBM_FN uint32_t rt_libm_asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
RT_LIBM_FN float rt_libm_asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
RT_LIBM_FN uint64_t rt_libm_asuint64(double f) { uint64_t u; memcpy(&u, &f, 8); return u; }
RT_LIBM_FN double rt_libm_asdouble(uint64_t u) { double f; memcpy(&f, &u, 8); return f; }

/* ------------------------------------------------------------------ sinf / cosf (sincosf.h) */
/* __sincosf_table[0]: cosine coefficients c0..c4, sine coefficients s1..s3 (|x| <= pi/4) */
#define RT_SC_HPI_INV 0x1.45f306dc9c883p+23 /* 2/pi * 2^24 (no fast round-to-int intrinsics) */
#define RT_SC_HPI 0x1.921fb54442d18p+0      /* pi/2 */
#define RT_SC_C0 0x1p0
#define RT_SC_C1 (-0x1.ffffffd0c621cp-2)
#define RT_SC_C2 0x1.55553e1068f19p-5
#define RT_SC_C3 (-0x1.6c087e89a359dp-10)
#define RT_SC_C4 0x1.99343027bf8c3p-16
#define RT_SC_S1 (-0x1.555545995a603p-3)
#define RT_SC_S2 0x1.1107605230bc4p-7
#define RT_SC_S3 (-0x1.994eb3774cf24p-13)

/* abstop12: the top 12 bits of |x| (sign cleared) */
RT_LIBM_FN uint32_t rt_libm_abstop12(float x) { return (rt_libm_asuint(x) >> 20) & 0x7ffu; }

/* sinf_poly (sincosf.h) split into its two polynomials.  The sine polynomial is odd and the
 * cosine one even, exactly: every step is a product or an FMA whose rounding commutes with
 * negation.  So sinf_poly(x * sign, x2, p, n) with p = __sincosf_table[n >> 1 & 1] (table 1 is
 * table 0 with the cosine coefficients negated) is +-rt_sin_poly(x) or +-rt_cos_poly(x2), and
 * one evaluation of each serves both sinf and cosf. */
RT_LIBM_FN double rt_sin_poly(double x, double x2) {
    const double x3 = x * x2;
    const double s1 = fma(x2, RT_SC_S3, RT_SC_S2);
    const double x7 = x3 * x2;
    const double s = fma(x3, RT_SC_S1, x);
    return fma(x7, s1, s);
}
RT_LIBM_FN double rt_cos_poly(double x2) {
    const double x4 = x2 * x2;
    const double c2 = fma(x2, RT_SC_C4, RT_SC_C3);
    const double c1 = fma(x2, RT_SC_C1, RT_SC_C0);
    const double x6 = x4 * x2;
    const double c = fma(x4, RT_SC_C2, c1);
    return fma(x6, c2, c);
}

/* reduce_fast: x mod pi/2 in [-pi/4, pi/4] and the quadrant n, accurate for |x| <= 120 */
RT_LIBM_FN double rt_sincos_reduce(double x, int* np) {
    const double r = x * RT_SC_HPI_INV;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fma(-(double)n, RT_SC_HPI, x);
}

/* sinf(y) and cosf(y), each equal to its own glibc call.  Returns 0 (outputs unset) for
 * |y| >= 120 or non-finite y, where glibc takes its slow path.  Branch-free below that:
 * for |y| < pi/4 glibc skips the reduction, which then gives n = 0 and x = y anyway, and for
 * |y| < 2^-12 it returns (y, 1). */
RT_LIBM_FN int rt_sincosf(float y, float* sinp, float* cosp) {
    const uint32_t t = rt_libm_abstop12(y);
    if (t >= rt_libm_abstop12(120.0f)) return 0;
    int n;
    const double x = rt_sincos_reduce((double)y, &n);
    const double x2 = x * x;
    const float sp = (float)rt_sin_poly(x, x2);  /* sin of the reduced argument */
    const float cp = (float)rt_cos_poly(x2);     /* cos of the reduced argument */
    /* quadrant n: sin y = {sp, cp, -sp, -cp}[n & 3], cos y = {cp, -sp, -cp, sp}[n & 3] */
    float s = (n & 1) ? cp : sp, c = (n & 1) ? sp : cp;
    s = (n & 2) ? -s : s;
    c = ((n + 1) & 2) ? -c : c;
    const int tiny = t < rt_libm_abstop12(0x1p-12f);
    *sinp = tiny ? y : s;
    *cosp = tiny ? 1.0f : c;
    return 1;
}

/* ------------------------------------------------------------------ powf (e_powf.c) */
/* __powf_log2_data: 16 subintervals {1/c, log2(c)} and the log2(1+r) polynomial */
#define RT_POWF_OFF 0x3f330000u
RT_LIBM_TABLE double rt_powf_log2_tab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4}, {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2}, {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2},
};
#define RT_POWF_A0 0x1.27616c9496e0bp-2
#define RT_POWF_A1 (-0x1.71969a075c67ap-2)
#define RT_POWF_A2 0x1.ec70a6ca7baddp-2
#define RT_POWF_A3 (-0x1.7154748bef6c8p-1)
#define RT_POWF_A4 0x1.71547652ab82bp+0
/* __exp2f_data: 2^(i/32) with i<<47 subtracted from the bits, and the 2^r polynomial */
RT_LIBM_TABLE uint64_t rt_exp2f_tab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
};
#define RT_EXP2F_SHIFT 0x1.8p+47 /* 0x1.8p52 / 32 */
#define RT_EXP2F_C0 0x1.c6af84b912394p-5
#define RT_EXP2F_C1 0x1.ebfce50fac4f3p-3
#define RT_EXP2F_C2 0x1.62e42ff0c52d6p-1

/* powf(x, 5.0f), as glibc computes it for y = 5 (an odd integer).  Every finite x. */
RT_LIBM_FN float rt_powf5_glibc(float x) {
    uint32_t ix = rt_libm_asuint(x);
    uint64_t sign_bias = 0;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        /* zero, subnormal, negative, inf or nan x */
        if (2u * ix - 1u >= 2u * 0x7f800000u - 1u) {       /* zeroinfnan(x) */
            float x2 = x * x;
            if (ix & 0x80000000u) x2 = -x2;                  /* y odd */
            return x2;                                       /* y > 0 */
        }
        if (ix & 0x80000000u) {                              /* finite x < 0, y odd */
            sign_bias = 0x800ull << 5;
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {                              /* subnormal: normalise */
            ix = rt_libm_asuint(rt_libm_asfloat(ix) * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    /* log2_inline */
    const uint32_t tmp = ix - RT_POWF_OFF;
    const int i = (int)((tmp >> (23 - 4)) % 16u);
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;
    const double invc = rt_powf_log2_tab[i][0], logc = rt_powf_log2_tab[i][1];
    const double z = (double)rt_libm_asfloat(iz);
    const double r = fma(z, invc, -1.0);
    const double y0 = logc + (double)k;
    const double r2 = r * r;
    double y = fma(RT_POWF_A0, r, RT_POWF_A1);
    const double p = fma(RT_POWF_A2, r, RT_POWF_A3);
    const double r4 = r2 * r2;
    double q = fma(RT_POWF_A4, r, y0);
    q = fma(p, r2, q);
    y = fma(y, r4, q);
    const double ylogx = 5.0 * y;
    /* |y log2 x| >= 126: overflow / underflow limits (x^5 of a float stays below 2^640) */
    if (((rt_libm_asuint64(ylogx) >> 47) & 0xffffu) >= (rt_libm_asuint64(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return sign_bias ? -__builtin_inff() : __builtin_inff();
        if (ylogx <= -150.0) return sign_bias ? -0.0f : 0.0f;
    }
    /* exp2_inline */
    double kd = ylogx + RT_EXP2F_SHIFT;
    const uint64_t ki = rt_libm_asuint64(kd);
    kd -= RT_EXP2F_SHIFT;
    const double rr = ylogx - kd;
    uint64_t t = rt_exp2f_tab[ki % 32u];
    t += (ki + sign_bias) << (52 - 5);
    const double s = rt_libm_asdouble(t);
    const double zz = fma(RT_EXP2F_C0, rr, RT_EXP2F_C1);
    const double rr2 = rr * rr;
    double yy = fma(RT_EXP2F_C2, rr, 1.0);
    yy = fma(zz, rr2, yy);
    yy = yy * s;
    return (float)yy;
}

/* The fast path (round 4).  For x in [2^-25, 2], x^5 in double — x * x exact (48 bits), then two
 * rounded products, within 2^-52 of x^5 — rounds to the correctly rounded float x^5 for every
 * such x (exhaustive, tools/check_libm.c pow_all).  glibc's powf rounds its own double value yy,
 * which lies within 2^-32.83 (relative) of x^5 over that range (exhaustive), so it
 * returns the same float unless x^5 is that close to a midpoint between two floats.  The 29
 * double-fraction bits the float drops say how far x5 lies from the midpoint: when they are more
 * than 2^21 + 4 double ulps away from it (2^21 covers 2^-32 of a value in [2^e, 2^(e + 1))), both
 * x^5 and yy are on x5's side, and the float of x5 is glibc's result.  Otherwise (0.8% of the
 * floats in the range) and outside the range the caller takes glibc's algorithm.  Returns 0 then. */
#define RT_POW5_GUARD ((1 << 21) + 4)
#ifndef RT_LIBM_POW5_FAST
#define RT_LIBM_POW5_FAST 1  /* 0: glibc's algorithm for every x (A/B builds only) */
#endif
RT_LIBM_FN int rt_powf5_fast(float x, float* out) {
    const double x2 = (double)x * (double)x, x4 = x2 * x2, x5 = x4 * (double)x;
    const int32_t low = (int32_t)(rt_libm_asuint64(x5) & 0x1fffffffu) - 0x10000000;
    *out = (float)x5;
    return (x >= 0x1p-25f && x <= 2.0f) && (low > RT_POW5_GUARD || low < -RT_POW5_GUARD);
}

/* glibc's powf(x, 5.0f), bit for bit, for every float x (tools/check_libm.c pow_all). */
RT_LIBM_FN float rt_powf5(float x) {
    float f;
    if (RT_LIBM_POW5_FAST && __builtin_expect(rt_powf5_fast(x, &f), 1)) return f;
    return rt_powf5_glibc(x);
}

#endif /* RT_LIBM_H */
