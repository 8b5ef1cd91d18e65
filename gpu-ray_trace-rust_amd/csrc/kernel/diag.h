// diag.h — diagnostic instrumentation of the queue kernels, kept out of the shipped library.
//
// The product build (make) defines neither switch: every DIAG_* / TM_* / VC macro below expands
// to nothing, so the shipped code object holds no clock reads, no instrumentation atomics and no
// printf (tests/test_device_code.py checks the last).  `make diag` builds
// lib/variants/librt_diag_timing.so (-DRT_TIMING=1) and lib/variants/librt_diag_vmem.so
// (-DRT_VMEM_COUNT=1) for the tools that read their printed lines:
//   RT_TIMING      wave-clock split of the queue kernels, summed over waves and printed by the
//                  last wave of each launch (tools/gpu_timing.sh);
//   RT_VMEM_COUNT  vector-memory load instructions of the general queue kernel by class, counted
//                  once per wave execution of each load site (tools/vmem_classes.py).  Classes:
//                  0 descent nodes, 1 pop nodes, 2 pass refs, 3 pass triangles, 4 leading spheres,
//                  5 winner re-test, 6 path-start pixel table, 7 mesh shading records, 8 textures,
//                  9 sphere / free-triangle shading, 10 packet leaf visits (scalar loads: no
//                  VMEM), 11 cooperative passes, 12 cooperative rounds, 13 radiance stores
//                  (writes), 14 path starts, 15-21 leaf sharing per round.  VL(class, address,
//                  bytes) beside a load counts, per wave execution, the distinct 128-B lines, 64-B
//                  sectors and lane addresses the load's active lanes touch (the requests that
//                  load can send towards L2), and its lanes: which class pulls lines it does
//                  not use (tools/vmem_classes.py).
// Included by trace.hip after the kernel helpers it calls (wave_incl_scan).
#pragma once

#ifndef RT_TIMING
#define RT_TIMING 0
#endif
#ifndef RT_VMEM_COUNT
#define RT_VMEM_COUNT 0
#endif
#ifndef RT_REGION_COUNT
#define RT_REGION_COUNT 0
#endif

namespace rtd {

#if RT_TIMING
__device__ unsigned long long g_tm[16];
__device__ unsigned int g_tm_waves;
__device__ __forceinline__ unsigned long long tm_now() {  // ordered stamp (cdna guide §7)
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define TM_NOW() ::rtd::tm_now()
#define TM_ADD(i, v) do { const unsigned long long tm_v_ = (unsigned long long)(v); \
                          if (__lane_id() == 0) atomicAdd(&::rtd::g_tm[i], tm_v_); } while (0)
#define TM_VAR(decl) decl
#else
#define TM_ADD(i, v) do { } while (0)
#define TM_VAR(decl)
#endif

#if RT_VMEM_COUNT
__device__ unsigned long long g_vc[24];
__device__ unsigned int g_vc_waves;
#define VC(i, n) do { if (__lane_id() == (uint32_t)__builtin_amdgcn_readfirstlane((int)__lane_id())) \
                           atomicAdd(&::rtd::g_vc[i], (unsigned long long)(n)); } while (0)
// VL: per class, {active lanes, distinct 128-B lines, distinct 64-B sectors, bytes the distinct
// lane addresses ask for (distinct addresses x the access's bytes)}
__device__ unsigned long long g_vl[16][4];
__device__ __forceinline__ uint32_t vl_distinct(uint64_t key, uint64_t mask) {
    uint32_t n = 0;
    while (mask) {
        const uint32_t ld = (uint32_t)__ffsll((unsigned long long)mask) - 1u;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, (int)ld);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(key >> 32), (int)ld);
        mask &= ~__ballot(key == (((uint64_t)hi << 32) | lo));
        ++n;
    }
    return n;
}
__device__ __forceinline__ void vl_count(uint32_t cls, uint64_t addr, uint32_t nbytes, bool act) {
    const uint64_t m = __ballot(act);
    if (!m) return;
    const uint32_t lanes = (uint32_t)__popcll(m);
    const uint32_t lines = vl_distinct(act ? addr >> 7 : ~0ull, m);
    const uint32_t secs = vl_distinct(act ? addr >> 6 : ~0ull, m);
    const uint32_t addrs = vl_distinct(act ? addr : ~0ull, m);
    if (__lane_id() == (uint32_t)__builtin_amdgcn_readfirstlane((int)__lane_id())) {
        atomicAdd(&g_vl[cls][0], (unsigned long long)lanes);
        atomicAdd(&g_vl[cls][1], (unsigned long long)lines);
        atomicAdd(&g_vl[cls][2], (unsigned long long)secs);
        atomicAdd(&g_vl[cls][3], (unsigned long long)addrs * nbytes);
    }
}
#define VL(cls, ptr, nbytes, act) ::rtd::vl_count((cls), (uint64_t)(uintptr_t)(ptr), (nbytes), (act))
#else
#define VC(i, n) do { } while (0)
#define VL(cls, ptr, nbytes, act) do { } while (0)
#endif

// RT_REGION_COUNT: wave-level executions of the sphere-only kernel's code regions (the first
// active lane adds 1: one count per wave-instruction stream through the region) and, for RC_LANES,
// the active lanes there — the dynamic side of the walled instruction accounting
// (tools/walled_accounting.py: counts x the region's VALU instructions per execution in the
// shipped ISA, reconciled with SQ_INSTS_VALU).  Regions: RC_* below.
enum {
    RC_ITER = 0,      // queue loop iterations with a path on some lane (= wave-segments)
    RC_ITER_LANES,    // ... lanes with a path in them
    RC_REGEN,         // path-start step taken (batched starts)
    RC_BATCH,         // a batch of 64 camera rays made (make_start)
    RC_ROOTS,         // closest_small: the roots of one sphere (some lane's ray line meets it)
    RC_SLAB,          // closest_small: root slab test + in_return_leaf (some lane hit a sphere)
    RC_FALLBACK,      // closest_small: the exact traversal below E (some lane not in the returning leaf)
    RC_FB_NODES,      // ... its descent steps
    RC_FB_LEAVES,     // ... its leaves
    RC_SHADE_HIT,     // shade past the miss test (some lane hit)
    RC_SEED,          // DiffSpec seed draw
    RC_RR,            // Russian roulette draw (depth > assured_depth)
    RC_SPEC,          // mirror continue
    RC_DIELECTRIC,    // refraction continue
    RC_DIFF,          // diffuse continue
    RC_ATTEN_DIV,     // attenuated colour by division (p != 1)
    RC_STORE,         // radiance stores (paths ending)
    RC_CUBE,          // cube-map emission
    RC_POW_SLOW,      // powf(x, 5) through glibc's path (the fast double-product check failed)
    RC_ROOTS_USEFUL,  // closest_small: roots executions where some lane's length becomes the running best
    RC_ROOTS_FRONT,   // ... where some lane meets the sphere ahead of its origin (not both roots behind it)
    RC_N = 24
};
#if RT_REGION_COUNT
__device__ unsigned long long g_rc[RC_N];
__device__ unsigned int g_rc_waves;
#define RC(i) do { if (__lane_id() == (uint32_t)__builtin_amdgcn_readfirstlane((int)__lane_id())) \
                        atomicAdd(&::rtd::g_rc[i], 1ull); } while (0)
#define RC_LANES(i) do { const uint32_t n_ = (uint32_t)__popcll(__ballot(1)); \
                         if (__lane_id() == (uint32_t)__builtin_amdgcn_readfirstlane((int)__lane_id())) \
                             atomicAdd(&::rtd::g_rc[i], (unsigned long long)n_); } while (0)
#else
#define RC(i) do { } while (0)
#define RC_LANES(i) do { } while (0)
#endif

#if RT_TIMING || RT_VMEM_COUNT
// One cooperative round, before its passes: how many lanes share a leaf.  RT_TIMING counts the
// rounds, the lanes with a leaf and the lanes at the first such lane's leaf; RT_VMEM_COUNT the
// pairs at leaves held by 2+ / 3+ / 4+ / 8+ lanes.
__device__ __forceinline__ void diag_round_sharing(uint32_t off, uint32_t cnt) {
#if RT_TIMING
    TM_ADD(9, 1);
    TM_ADD(10, __popcll(__ballot(cnt > 0)));
    {
        const uint64_t hv = __ballot(cnt > 0);
        const uint32_t f = hv ? (uint32_t)__ffsll((unsigned long long)hv) - 1u : 0u;
        const uint32_t fo = (uint32_t)__builtin_amdgcn_readlane((int)off, (int)f);
        TM_ADD(11, hv ? __popcll(__ballot(cnt > 0 && off == fo)) : 0);
    }
#endif
#if RT_VMEM_COUNT
    uint64_t pending = __ballot(cnt > 0);
    while (pending) {
        const uint32_t ld = (uint32_t)__ffsll((unsigned long long)pending) - 1u;
        const uint32_t o = __builtin_amdgcn_readlane(off, ld), n = __builtin_amdgcn_readlane(cnt, ld);
        const uint64_t same = __ballot(off == o && cnt > 0) & pending;
        pending &= ~same;
        const uint32_t g = (uint32_t)__popcll(same);
        VC(15, n * g);
        if (g >= 2) VC(16, n * g);
        if (g >= 3) VC(17, n * g);
        if (g >= 4) VC(18, n * g);
        if (g >= 8) VC(19, n * g);
        VC(20, n * ((g + 3u) / 4u));
        VC(21, 1);
    }
#endif
}
#define DIAG_ROUND_SHARING(off, cnt) ::rtd::diag_round_sharing(off, cnt)
#else
#define DIAG_ROUND_SHARING(off, cnt) do { } while (0)
#endif

// The last wave of a launch prints the launch's totals and clears them for the next launch.
#if RT_TIMING || RT_VMEM_COUNT || RT_REGION_COUNT
template <bool GEN>
__device__ __forceinline__ void diag_wave_exit() {
#if RT_REGION_COUNT
    if (__lane_id() == 0 && atomicAdd(&g_rc_waves, 1u) == gridDim.x * (blockDim.x / 64) - 1u) {
        __threadfence();
        for (int i = 0; i < RC_N; ++i) printf("RT_RC %d %llu\n", i, g_rc[i]);
        for (int i = 0; i < RC_N; ++i) g_rc[i] = 0;
        g_rc_waves = 0;
    }
#endif
#if RT_VMEM_COUNT
    if (GEN && __lane_id() == 0 && atomicAdd(&g_vc_waves, 1u) == gridDim.x * (blockDim.x / 64) - 1u) {
        __threadfence();
        for (int i = 0; i < 24; ++i) printf("RT_VC %d %llu\n", i, g_vc[i]);
        for (int i = 0; i < 24; ++i) g_vc[i] = 0;
        for (int i = 0; i < 16; ++i)
            printf("RT_VL %d %llu %llu %llu %llu\n", i, g_vl[i][0], g_vl[i][1], g_vl[i][2], g_vl[i][3]);
        for (int i = 0; i < 16; ++i) g_vl[i][0] = g_vl[i][1] = g_vl[i][2] = g_vl[i][3] = 0;
        g_vc_waves = 0;
    }
#endif
#if RT_TIMING
    if (__lane_id() == 0 && atomicAdd(&g_tm_waves, 1u) == gridDim.x * (blockDim.x / 64) - 1u) {
        __threadfence();
        printf("RT_TIMING packet %llu coop %llu wave %llu | pk_leaves %llu pk_lanes %llu pk_refs %llu | "
               "pk_rays %llu handed %llu coop_rays %llu | coop_rounds %llu coop_lanes %llu first_group %llu | "
               "passes_time %llu passes %llu\n",
               g_tm[0], g_tm[1], g_tm[2], g_tm[3], g_tm[4], g_tm[5], g_tm[6], g_tm[7], g_tm[8], g_tm[9],
               g_tm[10], g_tm[11], g_tm[12], g_tm[13]);
        for (int i = 0; i < 16; ++i) g_tm[i] = 0;
        g_tm_waves = 0;
    }
#endif
}
#define DIAG_WAVE_EXIT(GEN) ::rtd::diag_wave_exit<GEN>()
#else
#define DIAG_WAVE_EXIT(GEN) do { } while (0)
#endif

}  // namespace rtd
