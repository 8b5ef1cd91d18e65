/*
 * rt_rng.h — the random-stream contract shared by the device path and its CPU oracle.
 *
 * The reference draws from `rand::thread_rng()` (rand 0.8.5 ThreadRng = ChaCha12, OS-seeded,
 * one per rayon worker; src/lib.rs:22-27), so its images are not reproducible by design and
 * depend on thread scheduling.  This build replaces it with a keyed definition: every
 * (seed, pixel, absolute sample) owns its own stream, and draw k of a sample is a pure function
 * of (seed, pixel, sample, k).  Draw order within a sample follows the CPU path (SURVEY.md
 * Appendix B).  f32 draws keep rand 0.8's `Standard` mapping for f32: (u32 >> 8) * 2^-24,
 * uniform on [0, 1) with 24 significant bits.
 *
 * Generator: pcg32 (O'Neill 2014, "PCG-XSH-RR 64/32"): a 64-bit LCG state
 * (x <- x * 6364136223846793005 + 1442695040888963407 mod 2^64, period 2^64) with the XSH-RR
 * output permutation of the state before the step.  A stream's start state is a bijective
 * 64-bit hash (the SplitMix64 finalizer, Steele et al. 2014) of the seed, the pixel and the
 * sample, so distinct samples of one pixel start at distinct states.  With n streams of L draws
 * at random places on the one 2^64 cycle, a stream shares draws with about 2 n L / 2^64 others:
 * 5.5e-8 for spaceship_r1 at 4096^2 x 1000 spp (n = 1.7e10 streams, L ~ 30), i.e. ~470 pairs in
 * all, against ~240 overlapping streams for EVERY stream with round 1's 32-bit state.
 *
 * Plain C; compiled unchanged by gcc (oracle) and hipcc (gfx950 device code).
 */
#ifndef RT_RNG_H
#define RT_RNG_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RT_RNG_FN static inline __host__ __device__
#else
#define RT_RNG_FN static inline
#endif

#define RT_RNG_MUL 6364136223846793005ull
#define RT_RNG_INC 1442695040888963407ull

typedef uint64_t rt_rng_state;

/* SplitMix64's finalizer: a bijection of 64-bit words with full avalanche. */
RT_RNG_FN uint64_t rt_rng_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

/* Initial state of the stream of (seed, pixel = y*W + x, absolute sample index): for a fixed
 * seed and pixel, sample -> state is a bijection (mix64 of a bijection of the sample), and the
 * pixel enters through the first mix, so no two (pixel, sample) pairs share a start unless the
 * 64-bit hashes collide. */
RT_RNG_FN uint64_t rt_rng_pixel_key(uint64_t seed, uint32_t pixel) {
    return rt_rng_mix64(seed + 0x9e3779b97f4a7c15ull * ((uint64_t)pixel + 1u));
}
RT_RNG_FN rt_rng_state rt_rng_init_key(uint64_t key, uint64_t sample) { return rt_rng_mix64(key ^ sample); }
RT_RNG_FN rt_rng_state rt_rng_init(uint64_t seed, uint32_t pixel, uint64_t sample) {
    return rt_rng_init_key(rt_rng_pixel_key(seed, pixel), sample);
}

/* Next u32 of the stream (XSH-RR of the current state); advances *state. */
RT_RNG_FN uint32_t rt_rng_next_u32(rt_rng_state* state) {
    const uint64_t x = *state;
    *state = x * RT_RNG_MUL + RT_RNG_INC;
    const uint32_t xs = (uint32_t)(((x >> 18u) ^ x) >> 27u);
    const uint32_t rot = (uint32_t)(x >> 59u);
    return (xs >> rot) | (xs << ((32u - rot) & 31u));
}

/* rand 0.8 Standard f32: (u32 >> 8) * 2^-24 in [0, 1). */
RT_RNG_FN float rt_rng_next_f32(rt_rng_state* state) {
    return (float)(rt_rng_next_u32(state) >> 8) * (1.0f / 16777216.0f);
}

#endif /* RT_RNG_H */
