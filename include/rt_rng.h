/*
 * rt_rng.h — the random-stream contract shared by the device path and its CPU oracle.
 *
 * The reference draws from `rand::thread_rng()` (rand 0.8.5 ThreadRng = ChaCha12, OS-seeded,
 * one per rayon worker; src/lib.rs:22-27), so its images are not reproducible by design and
 * depend on thread scheduling.  This build replaces it with a counter-based definition:
 * every (seed, pixel, absolute sample) owns an independent stream, and draw k of a sample is a
 * pure function of (seed, pixel, sample, k).  Draw order within a sample follows the CPU path
 * (SURVEY.md Appendix B).  f32 draws keep rand 0.8's `Standard` mapping for f32:
 * (u32 >> 8) * 2^-24, uniform on [0, 1) with 24 significant bits.
 *
 * Generator: PCG-RXS-M-XS-32 output permutation over a 32-bit LCG (O'Neill 2014), the stream
 * start obtained by hashing the key through the same permutation.  Plain C; compiled
 * unchanged by gcc (oracle) and hipcc (gfx950 device code).
 */
#ifndef RT_RNG_H
#define RT_RNG_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RT_RNG_FN static inline __host__ __device__
#else
#define RT_RNG_FN static inline
#endif

#define RT_RNG_MUL 747796405u
#define RT_RNG_INC 2891336453u

RT_RNG_FN uint32_t rt_rng_permute(uint32_t state) {
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}

RT_RNG_FN uint32_t rt_rng_hash(uint32_t v) {
    return rt_rng_permute(v * RT_RNG_MUL + RT_RNG_INC);
}

/* Initial LCG state of the stream of (seed, pixel = y*W + x, absolute sample index). */
RT_RNG_FN uint32_t rt_rng_init(uint64_t seed, uint32_t pixel, uint64_t sample) {
    uint32_t h = rt_rng_hash((uint32_t)(sample >> 32));
    h = rt_rng_hash((uint32_t)sample ^ h);
    h = rt_rng_hash(pixel ^ h);
    h = rt_rng_hash((uint32_t)(seed >> 32) ^ h);
    h = rt_rng_hash((uint32_t)seed ^ h);
    return h;
}

/* Next u32 of the stream; advances *state. */
RT_RNG_FN uint32_t rt_rng_next_u32(uint32_t* state) {
    *state = *state * RT_RNG_MUL + RT_RNG_INC;
    return rt_rng_permute(*state);
}

/* rand 0.8 Standard f32: (u32 >> 8) * 2^-24 in [0, 1). */
RT_RNG_FN float rt_rng_next_f32(uint32_t* state) {
    return (float)(rt_rng_next_u32(state) >> 8) * (1.0f / 16777216.0f);
}

#endif /* RT_RNG_H */
