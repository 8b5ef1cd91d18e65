/* Checks include/rt_libm.h against the C library's sinf, cosf and powf (glibc: the functions
 * the reference's f32::sin/cos/powf call on Linux), bit for bit.
 *
 *   check_libm quick   every angle 2*pi*v the renderer can form (v = j * 2^-24, j < 2^24),
 *                      powf(x, 5) on 2^24 hashed x in [0, 1.001] and the special inputs
 *   check_libm full    additionally every float in [-2*pi, 2*pi] (sinf, cosf) and every float
 *                      in [0, 1.001] and [-0.001, 0] (powf(x, 5))
 *   check_libm pow_all powf(x, 5) on every one of the 2^32 float bit patterns (about 15 s
 *                      on 8 threads; run once per change of rt_powf5, recorded in DESIGN.md §3)
 *
 * Prints one JSON line; exit status 1 on any mismatch.
 * Build: gcc -O2 -mfma -ffp-contract=off -fopenmp -Iinclude tools/check_libm.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "rt_libm.h"

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float flt(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static int same(float a, float b) { return bits(a) == bits(b) || (isnan(a) && isnan(b)); }

typedef struct { unsigned long long tested, bad; uint32_t first; } stat_t;

static void check_angle(float th, unsigned long long* bad, uint32_t* first) {
    float s, c;
    if (!rt_sincosf(th, &s, &c)) return;
    /* volatile: keep the library calls (gcc would otherwise fold sinf + cosf into sincosf) */
    volatile float tv = th;
    const float gs = sinf(tv), gc = cosf(tv);
    if (!same(s, gs) || !same(c, gc)) {
        if (*bad == 0) *first = bits(th);
        ++*bad;
    }
}

static void check_pow(float x, unsigned long long* bad, uint32_t* first) {
    volatile float xv = x, y = 5.0f;
    const float g = powf(xv, y);
    if (!same(rt_powf5(x), g)) {
        if (*bad == 0) *first = bits(x);
        ++*bad;
    }
}

static uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

int main(int argc, char** argv) {
    if (argc > 1 && strcmp(argv[1], "pow_all") == 0) {
        /* rt_powf5 (fast path + glibc's algorithm) and each part alone against glibc's powf */
        unsigned long long bad = 0, fast = 0, fast_range = 0, glibc_bad = 0; uint32_t first = 0;
#pragma omp parallel for reduction(+ : bad, fast, fast_range, glibc_bad) schedule(dynamic, 1 << 20)
        for (int64_t u = 0; u < (int64_t)1 << 32; ++u) {
            unsigned long long b = 0; uint32_t f = 0;
            const float x = flt((uint32_t)u);
            check_pow(x, &b, &f);
            float ff;
            if (x >= 0x1p-25f && x <= 2.0f) ++fast_range;
            if (rt_powf5_fast(x, &ff)) ++fast;
            volatile float xv = x, y = 5.0f;
            if (!same(rt_powf5_glibc(x), powf(xv, y))) ++glibc_bad;
            if (b) { bad += b;
#pragma omp critical
                if (!first) first = f; }
        }
        printf("{\"powf5_every_float\": [%llu, %llu, \"0x%08x\"], \"glibc_path_mismatches\": %llu, "
               "\"fast_path_taken\": %llu, \"fast_path_range\": %llu}\n",
               1ull << 32, bad, first, glibc_bad, fast, fast_range);
        return (bad || glibc_bad) ? 1 : 0;
    }
    const int full = argc > 1 && strcmp(argv[1], "full") == 0;
    const float PI = 3.14159265358979323846f;
    stat_t ang = {0, 0, 0}, rng = {0, 0, 0}, pw = {0, 0, 0}, pwr = {0, 0, 0};

    /* the renderer's angles: thet = 2.0f * PI * v, v = (u32 >> 8) * 2^-24 (rt_rng.h) */
    {
        unsigned long long bad = 0; uint32_t first = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
        for (int64_t j = 0; j < (1 << 24); ++j) {
            const float v = (float)j * (1.0f / 16777216.0f);
            const float th = 2.0f * PI * v;
            unsigned long long b = 0; uint32_t f = 0;
            check_angle(th, &b, &f);
            if (b) { bad += b;
#pragma omp critical
                if (!first) first = f; }
        }
        ang.tested = 1ull << 24; ang.bad = bad; ang.first = first;
    }
    /* powf(x, 5): hashed x in [0, 1.001], then the specials */
    {
        unsigned long long bad = 0; uint32_t first = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
        for (int64_t j = 0; j < (1 << 24); ++j) {
            const float x = (float)(hash((uint32_t)j) >> 8) * (1.001f / 16777216.0f);
            unsigned long long b = 0; uint32_t f = 0;
            check_pow(x, &b, &f);
            if (b) { bad += b;
#pragma omp critical
                if (!first) first = f; }
        }
        const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, 1e-30f, -1e-30f, 1e-40f, -1e-40f, 0x1p-149f,
                            2.0f, 1e10f, 3e38f, -3e38f, INFINITY, -INFINITY, NAN, 1.0000001f,
                            0.99999994f, -1.1920929e-7f, 0x1p-30f, 0x1.5p-30f, 0x1p-29f};
        for (unsigned i = 0; i < sizeof sp / sizeof sp[0]; ++i) check_pow(sp[i], &bad, &first);
        pw.tested = (1ull << 24) + sizeof sp / sizeof sp[0]; pw.bad = bad; pw.first = first;
    }
    if (full) {
        /* every float in [-2 pi, 2 pi] */
        const uint32_t top = bits(2.0f * PI);
        unsigned long long bad = 0, n = 0; uint32_t first = 0;
#pragma omp parallel for reduction(+ : bad, n) schedule(dynamic, 1 << 20)
        for (int64_t u = 0; u <= (int64_t)top; ++u) {
            unsigned long long b = 0; uint32_t f = 0;
            check_angle(flt((uint32_t)u), &b, &f);
            check_angle(-flt((uint32_t)u), &b, &f);
            n += 2;
            if (b) { bad += b;
#pragma omp critical
                if (!first) first = f; }
        }
        rng.tested = n; rng.bad = bad; rng.first = first;
        /* every float in [0, 1.001] and [-0.001, 0] */
        const uint32_t ptop = bits(1.001f), ntop = bits(0.001f);
        unsigned long long pbad = 0, pn = 0; uint32_t pfirst = 0;
#pragma omp parallel for reduction(+ : pbad, pn) schedule(dynamic, 1 << 20)
        for (int64_t u = 0; u <= (int64_t)ptop; ++u) {
            unsigned long long b = 0; uint32_t f = 0;
            check_pow(flt((uint32_t)u), &b, &f);
            ++pn;
            if (u <= (int64_t)ntop) { check_pow(-flt((uint32_t)u), &b, &f); ++pn; }
            if (b) { pbad += b;
#pragma omp critical
                if (!pfirst) pfirst = f; }
        }
        pwr.tested = pn; pwr.bad = pbad; pwr.first = pfirst;
    }
    printf("{\"angles_2pi_v\": [%llu, %llu, \"0x%08x\"], \"powf5_sample\": [%llu, %llu, \"0x%08x\"]",
           ang.tested, ang.bad, ang.first, pw.tested, pw.bad, pw.first);
    if (full)
        printf(", \"sincos_all_floats_pm2pi\": [%llu, %llu, \"0x%08x\"], \"powf5_all_floats\": [%llu, %llu, \"0x%08x\"]",
               rng.tested, rng.bad, rng.first, pwr.tested, pwr.bad, pwr.first);
    printf(", \"format\": \"[tested, mismatches, first mismatching input bits]\"}\n");
    return (ang.bad | pw.bad | rng.bad | pwr.bad) ? 1 : 0;
}
