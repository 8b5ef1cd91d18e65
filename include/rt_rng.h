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
 * Generator: xoroshiro64* (Blackman & Vigna 2018, "Scrambled linear pseudorandom number
 * generators"): a 64-bit xorshift-rotate state of two 32-bit words (period 2^64 - 1), output the
 * first word times 0x9E3779BB.  Its lowest output bits are weak; the f32 draws use the top 24.
 * It replaced pcg32 (a 64-bit LCG with XSH-RR output) in round 4: one 32-bit multiply per draw
 * instead of a 64 x 64-bit multiply-add, for the same state size and period.  A
 * stream's start state is a bijective 64-bit hash (the SplitMix64 finalizer, Steele et al. 2014)
 * of the seed, the pixel and the sample, so distinct samples of one pixel start at distinct
 * states (but for the all-zero hash, a fixed point of the generator, which is replaced by a
 * constant that one other input also hashes to).  With n
 * streams of L draws at random places on the one 2^64 - 1 cycle, a stream shares draws with
 * about 2 n L / 2^64 others: 5.5e-8 for spaceship_r1 at 4096^2 x 1000 spp (n = 1.7e10 streams,
 * L ~ 30), i.e. ~470 pairs in all.
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
RT_RNG_FN rt_rng_state rt_rng_init_key(uint64_t key, uint64_t sample) {
    const uint64_t z = rt_rng_mix64(key ^ sample);
    return z ? z : 0x9e3779b97f4a7c15ull;  /* mix64(0) = 0 is xoroshiro's fixed point */
}
RT_RNG_FN rt_rng_state rt_rng_init(uint64_t seed, uint32_t pixel, uint64_t sample) {
    return rt_rng_init_key(rt_rng_pixel_key(seed, pixel), sample);
}

/* Next u32 of the stream (xoroshiro64*: state = s1 << 32 | s0); advances *state. */
RT_RNG_FN uint32_t rt_rng_rotl32(uint32_t x, uint32_t k) { return (x << k) | (x >> (32u - k)); }
RT_RNG_FN uint32_t rt_rng_next_u32(rt_rng_state* state) {
    const uint32_t s0 = (uint32_t)*state, s1 = (uint32_t)(*state >> 32) ^ s0;
    const uint32_t out = s0 * 0x9E3779BBu;
    const uint32_t n0 = rt_rng_rotl32(s0, 26) ^ s1 ^ (s1 << 9), n1 = rt_rng_rotl32(s1, 13);
    *state = ((uint64_t)n1 << 32) | n0;
    return out;
}

/* rand 0.8 Standard f32: (u32 >> 8) * 2^-24 in [0, 1). */
RT_RNG_FN float rt_rng_next_f32(rt_rng_state* state) {
    return (float)(rt_rng_next_u32(state) >> 8) * (1.0f / 16777216.0f);
}

#endif /* RT_RNG_H */
