// trace.hip — the gfx950 path-tracing kernels behind rt_render (include/rt_abi.h).
//
// Product schedule (queue_kernel): a persistent grid of exactly the resident lanes traces
// (pixel, sample) items until the launch's items run out.  A wave claims a run of consecutive
// items with one atomic and deals them to its idle lanes; a lane whose path ends writes the
// sample's radiance to radiance[sample][pixel] and takes the next item, so no lane waits for a
// slow pixel.  fold_kernel then applies the reference's per-pixel running mean
// (draw_scene.rs:81-83) in sample order.  Per item the lane runs the reference CPU path
// (render_to_target_cpu -> radiance, draw_scene.rs:73-84, radiance.rs:20-72) as a loop:
// camera ray (generate.rs:24-66) -> KD traversal (kdtree.rs:58-104) with the leaf test of
// closest_hit.rs:6-30 -> hit_info / Russian roulette / continue_ray of the hit element
// (sphere.rs, triangle/generic.rs, mesh/triangle.rs, distant_cube_map.rs, material/*.rs).
//
// Two instantiations: GEN = false for sphere-only scenes (walled.yml: spheres and materials in
// LDS, the exact brute-force bound closest_small), GEN = true for triangles and meshes: a wave's
// camera rays of one direction octant walk the tree as a packet, with wave-uniform nodes and
// triangles in scalar registers (closest_packet), and every other search tests the lanes' KD
// leaves cooperatively, all (ray, ref) pairs of the wave spread over its 64 lanes
// (stack_search_coop).  Both are bit-identical to the reference's per-ray stack traversal.
// The queue hands out a launch's pixels in 8 x 8 blocks (LaunchArgs::pix_q).  trace_kernel (one lane
// per pixel, running mean in registers) is the direct schedule kept as the tests' second path
// and, with COUNT, the work counter behind the roofline's algorithmic bytes.
//
// Float order matches the oracle operation for operation (compiled with -ffp-contract=off,
// correctly rounded div/sqrt, and glibc's sinf/cosf/powf restated in include/rt_libm.h); the
// only intended difference is the accumulation order of the bounce estimator (forward
// L += T*e instead of the reference's recursion) — DESIGN.md §Numerics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/rt_abi.h"
#include "../../../include/rt_rng.h"
#include "../../../include/rt_libm.h"
#include "device_scene.h"
#include "diag.h"  // instrumentation of the diagnostic builds only (make diag); empty here

// Tuning constants (round 5: compile-time switches folded into constants; each value is the
// measured best of its A/B).  LDS_SPHERES lives in device_scene.h (the host
// shares it).

namespace rtd {

constexpr int RT_REGEN_MIN = 12;  // sphere-only queue kernel: start new paths once this many lanes are idle or none is busy (walled +1.4%; 6: 0, 16: +1.2%)
constexpr int RT_REGEN_MIN_BATCH = 1;  // the sphere-only kernel with batched starts (RT_START_BATCH): a start costs a few LDS reads, so idle lanes start at once (walled +6.5%; 4: +4.8%, 8: +3.5%); lens cameras, which keep per-lane starts, use it too
constexpr int RT_REGEN_MIN_GEN = 16;  // the same for the general queue kernel: camera rays start in batches that form packets (closest_packet; a380 +2.6%)
constexpr int RT_MIN_WAVES = 7;  // __launch_bounds__ min waves per SIMD: 7 -> <=72 VGPRs (measured best; 6: -3%, 8: -2.3%)
constexpr int RT_MIN_WAVES_GEN = 8;  // general (triangle / mesh) kernels: 8 -> <=64 VGPRs; latency-bound, +2..7% over 7 (spills outside the pass loop)
constexpr int RT_OWNER_LOOP = 8;  // cooperative pass: owners of a pass found by a readlane loop when at most this many leaves end in it (0: binary search)
constexpr int RT_PAIR_FETCH = 1;  // cooperative descent: a node's two children loaded together, before its decision (a380 +3%, biplane +3%)
constexpr int RT_PIX_KEY = 1;  // queue kernels: the pixel's stream key from the queue-order table (one SplitMix64 round per path start, not two)
constexpr int RT_START_BATCH = 1;  // sphere-only queue kernel: camera rays made 64 at a time, at full wave width, and handed out from LDS
constexpr int RT_PACKET = 1;  // general queue kernel: camera rays of a wave traced as one packet (closest_packet)
constexpr int RT_LEAF_REUSE = 1;  // cooperative search: a leaf whose ref list is the previous leaf's reuses its minimum
constexpr int RT_PACKET_MIN = 40;  // fewest camera rays of one direction octant that form a packet

constexpr float EPS = 1e-4f;            // src/lib.rs:20
constexpr float HIT_MIN = EPS * 20.0f;  // closest_hit.rs:16
constexpr float PI = 3.14159265358979323846f;
constexpr float RR_THRES = 0.4f;        // radiance.rs:77
// The reference has no depth cap (radiance.rs:44); past assured_depth a path survives a bounce
// with p = 0.4, so a cap of 1024 bounces changes an estimate with probability < 0.4^1000.
// It only guarantees that a corrupted scene cannot hang the GPU.
constexpr int MAX_BOUNCES = 1024;

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 mk(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator-(V3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 operator*(float s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ V3 operator/(V3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ V3 cmul(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
// ---------------------------------------------------------------- exact fast arithmetic
// Correctly rounded reciprocal and quotient in 3 + 3 instructions instead of hipcc's ~10-instruction
// IEEE sequence (div_scale / rcp / fma chain / div_fmas / div_fixup):
//   rcp_exact(b) = fma(fma(-b, y, 1), y, y), y = v_rcp_f32(b): equal to 1.0f / b for EVERY normal
//     |b| in [2^-60, 2^60] (exhaustive, tools/check_exact_ops.hip);
//   div_mk(a, b, r) = fma(fma(-a*r, b, a), r, a*r) with r = rcp_exact(b): equal to a / b
//     (Markstein; 4.3e9 random pairs + 2.1e9 normalize-shaped pairs, same tool) when a is 0 or
//     also in that range — the zero case keeps a's sign explicitly.
// Operands outside the range take the IEEE division (a divergent branch no lane normally takes).
__device__ __forceinline__ bool mk_range(float x) {
    const uint32_t e = (__float_as_uint(x) >> 23) & 0xffu;
    return e >= 67u && e <= 186u;  // [2^-60, 2^60): the range the checks cover
}
__device__ __forceinline__ bool mk_num(float x) { return (__float_as_uint(x) << 1) == 0u || mk_range(x); }
__device__ __forceinline__ float rcp_exact(float b) {
    const float y = __builtin_amdgcn_rcpf(b);
    return fmaf(fmaf(-b, y, 1.0f), y, y);
}
__device__ __forceinline__ float div_mk(float a, float b, float r) {
    const float q0 = a * r;
    const float q = fmaf(fmaf(-q0, b, a), r, q0);
    return (__float_as_uint(a) << 1) == 0u ? a : q;
}
// The Markstein quotient without div_mk's zero test: exact for nonzero a in range; a = +-0
// gives +0 (callers that need the sign of a zero restore it, or only compare the result).
__device__ __forceinline__ float div_mk_nz(float a, float b, float r) {
    const float q0 = a * r;
    return fmaf(fmaf(-q0, b, a), r, q0);
}
// 1.0f / b for a b the caller knows is not below 2^-60 in magnitude (or whose reciprocal it
// discards otherwise): one compare guards the top of the exact range.
__device__ __forceinline__ float recip_big(float b) {
    float r = rcp_exact(b);
    if (__builtin_expect(!(fabsf(b) < 0x1p60f), 0)) r = 1.0f / b;
    return r;
}
// 1.0f / b, bit for bit
__device__ __forceinline__ float recip(float b) {
    float r = rcp_exact(b);
    if (__builtin_expect(!mk_range(b), 0)) r = 1.0f / b;
    return r;
}
// (a.x / b, a.y / b, a.z / b), bit for bit
__device__ __forceinline__ V3 div3(V3 a, float b) {
    const float r = rcp_exact(b);
    V3 q = mk(div_mk(a.x, b, r), div_mk(a.y, b, r), div_mk(a.z, b, r));
    if (__builtin_expect(!(mk_range(b) && mk_num(a.x) && mk_num(a.y) && mk_num(a.z)), 0)) q = a / b;
    return q;
}
// sqrtf(x), bit for bit, for every x in [2^-80, FLT_MAX] (exhaustive, tools/check_exact_ops.hip):
// Markstein's correction of s = x * rsq(x) with one rounding, s + (x - s^2) * rsq(x) / 2 — five
// instructions instead of hipcc's IEEE sequence.  DOMAIN: [2^-80, FLT_MAX] only — at +-0 and +inf
// it returns NaN, below 2^-80 it is inexact.  A caller whose argument may leave that range goes
// through sqrt_nonneg / sqrt_draw (the guarded forms below), as every current caller does.
__device__ __forceinline__ float sqrt_rn_normal(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    return fmaf(fmaf(-s, s, x), 0.5f * y, s);
}
// sqrtf(x) for x >= -0 (an fmaxf(y, 0), a dot(a, a), a uniform draw): one compare sends ±0,
// (0, 2^-80), +inf and NaN to sqrtf — a divergent branch no lane normally takes.
__device__ __forceinline__ float sqrt_nonneg(float x) {
    float s = sqrt_rn_normal(x);
    if (__builtin_expect(__float_as_uint(x) - (47u << 23) >= 0x7f800000u - (47u << 23), 0)) s = sqrtf(x);
    return s;
}
// sqrtf of a uniform draw u or of 1 - u: 0 or in [2^-24, 1] (rt_rng.h's (x >> 8) * 2^-24,
// u <= 1 - 2^-24), inside sqrt_rn_normal's exact range but for 0.
__device__ __forceinline__ float sqrt_draw(float x) {
    return x == 0.0f ? x : sqrt_rn_normal(x);
}
// nalgebra normalize: a / |a| per component.  div3's guard, specialised: |a_i| < 2^60 follows
// from |a| < 2^60 (|a_i| >= 2^60 makes fl(a.a) >= 2^120), so each numerator only needs to be
// nonzero with |a_i| >= 2^-60.  A NaN numerator makes |a| NaN, which fails mk_range.
__device__ __forceinline__ V3 normalize(V3 a) {
    float n = sqrt_nonneg(dot(a, a));
    const float r = rcp_exact(n);
    // Common case: every |a_i| >= 2^-60 (one v_min3 and one compare), so no numerator is zero
    // and div_mk's zero test is not needed either.  A zero or tiny component, or n out of range,
    // takes the IEEE division (a divergent branch that lanes rarely take).
    V3 q = mk(div_mk_nz(a.x, n, r), div_mk_nz(a.y, n, r), div_mk_nz(a.z, n, r));
    const float amin = fminf(fminf(fabsf(a.x), fabsf(a.y)), fabsf(a.z));
    if (__builtin_expect(!(mk_range(n) && amin >= 0x1p-60f), 0)) q = a / n;
    return q;
}
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float comp(V3 v, uint32_t a) {
    float r = __builtin_unpredictable(a == 1u) ? v.y : v.x;
    return __builtin_unpredictable(a == 2u) ? v.z : r;
}
__device__ __forceinline__ V3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ V3 xyz(float4 v) { return mk(v.x, v.y, v.z); }

// RayLen ordering (hit.rs:50-76): NaN sorts above everything.
__device__ __forceinline__ bool raylen_less(float a, float b) {
    if (__builtin_isnan(a)) return false;
    if (__builtin_isnan(b)) return true;
    return a < b;
}

struct Ray {
    V3 d, o;
};

struct Hit {
    uint32_t ref;   // device ref (kind | index); 0xffffffff = cube map
    float l;
    float bu, bv;   // triangle barycentrics
};
constexpr uint32_t REF_CUBE = 0xffffffffu;

template <bool COUNT>
struct Ctr {
    uint32_t nodes = 0, leaf_refs = 0, sph = 0, tri = 0, segments = 0, hits = 0, mesh_hits = 0;
};

// Workgroup-shared copies (LDS) of the sphere-only kernel's scene data: every sphere, its
// {c, fl(r * r)} and its material (the host launches that kernel only when they all fit).
// The LDS copies are file-scope __shared__ arrays referenced directly, so loads from them are
// ds_read (a pointer that may be LDS or global would become a slower FLAT load).
__shared__ float4 g_lds_csq[LDS_SPHERES];  // {c, fl(r * r)}: sphere.rs:92's r*r, computed once
__shared__ float4 g_lds_lo[LDS_SPHERES];   // {fl(c - r), r}: the box's low faces (sphere.rs:106-114)
__shared__ float4 g_lds_hi[LDS_SPHERES];   // {fl(c + r), 0}: its high faces
__shared__ DevMat g_lds_mat[LDS_SPHERES];
__device__ __forceinline__ uint2 fetch_node(const DevScene& sc, uint32_t i) { return sc.nodes[i]; }
// GEN == false (sphere-only kernel): spheres come from LDS.  The general kernel reads them from
// global memory.
template <bool GEN>
__device__ __forceinline__ float4 fetch_sphere(const DevScene& sc, uint32_t i) {
    if (!GEN) {
        const float4 q = g_lds_csq[i];
        return make_float4(q.x, q.y, q.z, g_lds_lo[i].w);
    }
    return sc.sph[i];
}

__device__ __forceinline__ void fill_lds_spheres(const DevScene& sc) {
    const uint32_t n = sc.n_spheres < (uint32_t)LDS_SPHERES ? sc.n_spheres : (uint32_t)LDS_SPHERES;
    for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {
        const float4 v = sc.sph[i];
        g_lds_csq[i] = make_float4(v.x, v.y, v.z, v.w * v.w);
        g_lds_lo[i] = make_float4(v.x - v.w, v.y - v.w, v.z - v.w, v.w);
        g_lds_hi[i] = make_float4(v.x + v.w, v.y + v.w, v.z + v.w, 0.f);
        g_lds_mat[i] = sc.sph_mat[i];
    }
}

// ---------------------------------------------------------------- primitives
// Sphere::intersect (sphere.rs:83-105) in two steps: the discriminant (sphere_disc, with
// rr = fl(r * r)), then the roots (sphere_roots), so the brute-force loop can skip the second
// step for a sphere no lane of the wave meets.  Branch-free: the root is taken of thing2 as is,
// and used only when thing2 > 0.  thing >= 0 gives l1 = RN(offset - thing) <=
// l0 = RN(offset + thing), so p1 implies p0, filter(>0).reduce(min) is `p1 ? l1 : l0`, and a
// hit is disc && p0 (a miss's *l is never used).
struct SphDisc {
    float dir, thing2;
};
__device__ __forceinline__ SphDisc sphere_disc(float4 s, float rr, const Ray& r) {
    const V3 oc = r.o - xyz(s);
    const float dir = dot(r.d, oc);
    const float consts = dot(oc, oc) - rr;
    return SphDisc{dir, dir * dir - consts};
}
// L0 = false drops the l0 > 0 test, for callers that then require !(l < HIT_MIN): with disc,
// and finite dir and thing2 (scene coordinates below 2^58, DevScene::small_ok), l is finite, and
// l >= HIT_MIN > 0 implies l0 > 0 (l = l1 > 0 gives l0 >= l1; otherwise l = l0).
template <bool L0 = true>
__device__ __forceinline__ bool sphere_roots(SphDisc q, float* l) {
    const bool disc = q.thing2 > 0.0f;
    const float offset = -q.dir;
    // thing2 <= 0 (or NaN) gives a NaN or 0 here, but then disc is false and *l is never used
    // sqrt_nonneg's tiny-input guard as one float compare beside disc (lanes without disc
    // never use the root, so only disc lanes with thing2 < 2^-80 need sqrtf)
    float thing = sqrt_rn_normal(q.thing2);
    if (__builtin_expect(disc && q.thing2 < 0x1p-80f, 0)) thing = sqrtf(q.thing2);
    const float l0 = offset + thing, l1 = offset - thing;
    *l = l1 > 0.0f ? l1 : l0;  // sphere.rs:95
    return disc && (!L0 || l0 > 0.0f);
}
__device__ __forceinline__ bool sphere_hit(float4 s, const Ray& r, float* l) {
    return sphere_roots(sphere_disc(s, s.w * s.w, r), l);
}

// Triangle::intersect, Möller–Trumbore (triangle/generic.rs:102-137), from the vertex v0 and
// the edges e1 = v1 - v0, e2 = v2 - v0 the host computed (DevScene::prim4)
__device__ __forceinline__ bool tri_hit(V3 v0, V3 e1, V3 e2, const Ray& r, float* l, float* bu,
                                        float* bv) {
    V3 ray_x_e2 = cross(r.d, e2);
    float det = dot(e1, ray_x_e2);
    if (fabsf(det) < EPS) return false;
    float inv_det = recip_big(det);  // |det| >= EPS here
    V3 rhs = r.o - v0;
    float u = inv_det * dot(rhs, ray_x_e2);
    if (u < 0.0f || u > 1.0f) return false;
    V3 rhs_x_e1 = cross(rhs, e1);
    float v = inv_det * dot(r.d, rhs_x_e1);
    if (v < 0.0f || (u + v) > 1.0f) return false;
    float t = inv_det * dot(e2, rhs_x_e1);
    if (t < EPS) return false;
    *l = t;
    *bu = u;
    *bv = v;
    return true;
}

// closest_ray_hit over one leaf (closest_hit.rs:6-30): first strict RayLen minimum among
// hits not shorter than 20*EPS.
// Device data of a leaf ref: a sphere's float4 {c, r} or a triangle's three vertices.
__device__ __forceinline__ const float4* prim_data(const DevScene& sc, uint32_t ref) {
    const uint32_t kind = ref >> REF_KIND_SHIFT, idx = ref & REF_INDEX_MASK;
    (void)kind;
    return sc.prim4 + 3 * (size_t)idx;
}
// One ref of a general leaf with its primitive's data (loaded ahead of the test).
struct LeafSlot {
    uint32_t ref;
    float4 a0, a1, a2;
    __device__ __forceinline__ void load(const DevScene& sc) {
        const float4* p = prim_data(sc, ref);
        a0 = p[0];
        a1 = p[1];
        a2 = p[2];
    }
};
// One ref of closest_ray_hit (closest_hit.rs:6-30) in the general kernel.
template <bool COUNT>
__device__ __forceinline__ void leaf_step(const LeafSlot& sl, const Ray& r, Hit* best, bool& found,
                                          Ctr<COUNT>& c) {
    const uint32_t ref = sl.ref;
    const float4 a0 = sl.a0, a1 = sl.a1, a2 = sl.a2;
    float l = 0.f, bu = 0.f, bv = 0.f;
    bool h;
    if (__builtin_expect((ref >> REF_KIND_SHIFT) == K_SPHERE, 0)) {
        if (COUNT) c.sph++;
        h = sphere_hit(a0, r, &l);
    } else {
        if (COUNT) c.tri++;
        h = tri_hit(xyz(a0), xyz(a1), xyz(a2), r, &l, &bu, &bv);
    }
    const bool above = !raylen_less(l, HIT_MIN);  // RayLen order: NaN sorts above everything
    const bool closer = raylen_less(l, best->l);
    const bool take = h & above & (!found | closer);
    best->ref = take ? ref : best->ref;
    best->l = take ? l : best->l;
    best->bu = take ? bu : best->bu;
    best->bv = take ? bv : best->bv;
    found = found || take;
}

template <bool COUNT, bool GEN, bool SMALL = false>
__device__ __forceinline__ bool leaf_closest(const DevScene& sc, uint32_t off,
                                             uint32_t cnt, const Ray& r, Hit* best, Ctr<COUNT>& c,
                                             uint32_t imin = 0, float lmin = 0.f) {
    if (SMALL) {
        // If the leaf holds the globally closest sphere, that sphere is its candidate: no other
        // leaf sphere is closer, and on a tie the lowest renderable index wins both globally and
        // in leaf order.  Only otherwise are the leaf's spheres re-tested.
        bool has_min = false;
        for (uint32_t j = 0; j < cnt; ++j) has_min |= (sc.refs[off + j] & REF_INDEX_MASK) == imin;
        if (has_min) {
            best->ref = (K_SPHERE << REF_KIND_SHIFT) | imin;
            best->l = lmin;
            best->bu = best->bv = 0.f;
            return true;
        }
    }
    bool found = false;
    if (GEN && !SMALL) {
        // Two refs per step: both refs and both primitives' data are loaded before either is
        // tested, so a lane keeps two dependent load chains in flight.  A sphere reads its float4
        // and the two padding float4s after it (the array is padded); a step past the leaf's end
        // re-reads its last ref and skips the test.
        for (uint32_t j = 0; j < cnt; j += 2) {
            LeafSlot s0, s1;
            s0.ref = sc.refs[off + j];
            s1.ref = sc.refs[off + (j + 1 < cnt ? j + 1 : cnt - 1)];
            s0.load(sc);
            s1.load(sc);
            leaf_step<COUNT>(s0, r, best, found, c);
            if (j + 1 < cnt) leaf_step<COUNT>(s1, r, best, found, c);
        }
        return found;
    }
    for (uint32_t j = 0; j < cnt; ++j) {
        uint32_t ref = sc.refs[off + j];
        uint32_t kind = ref >> REF_KIND_SHIFT, idx = ref & REF_INDEX_MASK;
        float l = 0.f, bu = 0.f, bv = 0.f;
        bool h;
        if (!GEN || kind == K_SPHERE) {
            if (COUNT) c.sph++;
            h = sphere_hit(fetch_sphere<GEN>(sc, idx), r, &l);
        } else {
            if (COUNT) c.tri++;
            const float4* v = sc.prim4 + 3 * (size_t)idx;
            h = tri_hit(xyz(v[0]), xyz(v[1]), xyz(v[2]), r, &l, &bu, &bv);
        }
        // spheres never produce a NaN length: plain compares; triangles keep RayLen's order
        const bool above = GEN ? !raylen_less(l, HIT_MIN) : !(l < HIT_MIN);
        const bool closer = GEN ? raylen_less(l, best->l) : (l < best->l);
        const bool take = h & above & (!found | closer);
        best->ref = take ? ref : best->ref;
        best->l = take ? l : best->l;
        best->bu = take ? bu : best->bu;
        best->bv = take ? bv : best->bv;
        found = found || take;
    }
    return found;
}

// Per-ray traversal constants: the EPS-clamped direction of kdtree.rs:75-77 / aabb.rs:28-30
// and its correctly rounded reciprocal 1.0 / d (aabb.rs:31 computes exactly this value).
// Named scalars, not arrays: an indexed array would be lowered to scratch memory.
struct RayAx {
    float dx, dy, dz, rx, ry, rz;
};
__device__ __forceinline__ float clamp_eps(float d) { return fabsf(d) < EPS ? (d < 0.0f ? -EPS : EPS) : d; }
__device__ __forceinline__ RayAx ray_axes(const Ray& r) {
    RayAx x;
    x.dx = clamp_eps(r.d.x);
    x.dy = clamp_eps(r.d.y);
    x.dz = clamp_eps(r.d.z);
    x.rx = recip_big(x.dx);  // clamped: |d| >= EPS (or NaN, which recip_big sends to 1 / d)
    x.ry = recip_big(x.dy);
    x.rz = recip_big(x.dz);
    return x;
}
// Branch-free pick by axis a in {0,1,2}.
__device__ __forceinline__ float sel3(float v0, float v1, float v2, uint32_t a) {
    float r = __builtin_unpredictable(a == 1u) ? v1 : v0;
    return __builtin_unpredictable(a == 2u) ? v2 : r;
}

// n / d, correctly rounded.  FAST: q0 = n*rcp, r = fma(-q0, d, n) (exact), q = fma(r, rcp, q0).
// With rcp = RN(1/d) this is RN(n/d) whenever nothing under/overflows (Markstein's theorem; also
// checked on 2e9 random f32 pairs, tools/check_fastdiv.c): 3 instructions instead of 11.  Here
// |d| is in [1e-4, 1] and FAST is only used when every split and ray-origin component is 0 or in
// [2^-70, 2^60] (origin_fast_ok, DevScene::fastdiv), so |n| = |split - o| is 0 or in
// [2^-93, 2^61]: no intermediate under/overflows.
template <bool FAST>
__device__ __forceinline__ float div_exact(float n, float d, float rcp) {
    if (FAST) {
        const float q0 = n * rcp;
        const float res = fmaf(-q0, d, n);
        return fmaf(res, rcp, q0);
    }
    (void)rcp;
    return n / d;
}
__device__ __forceinline__ bool fast_range(float x) {
    const uint32_t b = __float_as_uint(x) & 0x7fffffffu;
    return b == 0u || (b >= (57u << 23) && b < (188u << 23));  // 0 or [2^-70, 2^61)
}
__device__ __forceinline__ bool origin_fast_ok(V3 o) {
    return fast_range(o.x) && fast_range(o.y) && fast_range(o.z);
}

// Split distance of branch `nd` along the ray (kdtree.rs:75-78): (split - o_a) / d_a with the
// clamped d, bit-identical however often it is recomputed.
template <bool FAST>
__device__ __forceinline__ float split_t(uint2 nd, const RayAx& ax, const Ray& r, float* d_out) {
    const uint32_t a = nd.y & 3u;
    const float d = sel3(ax.dx, ax.dy, ax.dz, a);
    *d_out = d;
    return div_exact<FAST>(__uint_as_float(nd.x) - sel3(r.o.x, r.o.y, r.o.z, a), d, sel3(ax.rx, ax.ry, ax.rz, a));
}

// Aabb::get_entry_exit (aabb.rs:22-62): slab test with the clamped direction, f = 1.0 / d.
__device__ __forceinline__ bool entry_exit(const float* b, const RayAx& ax, const Ray& r, float* entry,
                                           float* exit_t) {
    float vp = 0.f, wp = 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float f = a == 0 ? ax.rx : (a == 1 ? ax.ry : ax.rz);
        const float o = a == 0 ? r.o.x : (a == 1 ? r.o.y : r.o.z);
        const float lo = (b[2 * a] - o) * f;
        const float hi = (b[2 * a + 1] - o) * f;
        const float v = fminf(lo, hi), w = fmaxf(lo, hi);
        if (a == 0) {
            vp = v;
            wp = w;
        } else {
            if (vp < v) vp = v;
            if (wp > w) wp = w;
        }
    }
    if (wp < 0.0f || vp > wp) return false;
    *entry = vp;
    *exit_t = wp;
    return true;
}

// KdTree::stack_search (kdtree.rs:66-104) from the root interval [root_entry, root_exit].
//
// Stack: the reference pushes (far child, t, exit) (kdtree.rs:85).  Here an entry is only the
// 4-byte index of the branch that pushed it: far child and t follow from that node and the ray
// (split_t), and an entry's exit is the t of the entry below it (or the root exit), because
// every push also sets exit = t.  The t of the top entry is cached in a register; popping
// recomputes the t of the new top.  4 bytes per entry keep the LDS stack small enough that
// LDS never limits the waves per SIMD.
//
// The descent step is branch-free: the current branch is always written to slot sp (above the
// stack top when nothing is pushed; a branch at depth D has sp <= D < stack_depth) and sp only
// advances on a push, so the three reference cases (near / far / push both) are selects.
template <bool COUNT, bool GEN, bool FAST, bool SMALL = false, bool RESTART = false>
__device__ __forceinline__ bool stack_search(const DevScene& sc, const Ray& r, const RayAx& ax,
                                             float root_entry, float root_exit, Hit* best, uint32_t* st,
                                             Ctr<COUNT>& c, uint32_t imin = 0, float lmin = 0.f) {
    float entry = root_entry, exit_t = root_exit, top_t = root_exit;
    uint32_t node = 0, restart = 0;
    int sp = 0;
    for (;;) {
        uint2 nd = fetch_node(sc, node);
        bool pushed = false;
        while ((nd.y & 3u) != RT_KD_LEAF) {
            if (COUNT) c.nodes++;
            if (!GEN && SMALL) RC(RC_FB_NODES);
            float d;
            const float t = split_t<FAST>(nd, ax, r, &d);
            const bool pos = d > 0.0f;          // near = low when d > 0 (kdtree.rs:79)
            const bool go_near = t >= exit_t;   // kdtree.rs:80
            const bool go_far = !go_near && t <= entry;  // kdtree.rs:82
            const bool push = !go_near && !go_far;       // kdtree.rs:84-87
            if (!RESTART) {
                st[sp * BLOCK] = node;
                sp += push ? 1 : 0;
                top_t = push ? t : top_t;
            }
            exit_t = push ? t : exit_t;
            node = (nd.y >> 2) + (go_far == pos ? 1u : 0u);
            if (RESTART) {  // stackless: see stack_search_coop
                pushed = pushed || push;
                restart = pushed ? restart : node;
            }
            nd = fetch_node(sc, node);
        }
        if (COUNT) { c.nodes++; c.leaf_refs += nd.x & LEAF_COUNT_MASK; }
        if (!GEN && SMALL) RC(RC_FB_LEAVES);
        if (leaf_closest<COUNT, GEN, SMALL>(sc, nd.y >> 2, nd.x & LEAF_COUNT_MASK, r, best, c, imin, lmin) &&
            best->l <= exit_t + EPS)
            return true;
        if (RESTART) {
            if (!pushed) return false;
            entry = exit_t;
            exit_t = root_exit;
            node = restart;
            continue;
        }
        if (sp == 0) return false;
        --sp;
        const uint2 pn = fetch_node(sc, st[sp * BLOCK]);
        float d;
        (void)split_t<FAST>(pn, ax, r, &d);
        node = (pn.y >> 2) + (d > 0.0f ? 1u : 0u);  // the far child
        entry = top_t;
        if (sp) {
            top_t = split_t<FAST>(fetch_node(sc, st[(sp - 1) * BLOCK]), ax, r, &d);
            exit_t = top_t;
        } else {
            exit_t = root_exit;
        }
    }
}

// Whether the closest sphere S (hit at L*, first minimum) is in the leaf the reference's
// traversal returns from, decided without the traversal.  The visited leaves' intervals
// [e_i, x_i] are contiguous and cover [root_entry, root_exit]; leaves with fl(x + EPS) < L*
// cannot return (their best hit is >= L*), so the returning leaf is the first leaf k with
// fl(x_k + EPS) >= L* if it holds S — whose candidate is then S at L* (leaf_closest's pmin
// argument).  Such a leaf exists when fl(root_exit + EPS) >= L*; it has x_k > E (the descent
// floor) and e_k <= L* (e_k = root_entry <= L*, or e_k = x_{k-1} < L*).  Below a branch (split
// s on axis a, t_s = RN(RN(s - o_a) / d_a), monotone in s), leaves of the near child have
// x <= t_s and leaves of the far child e >= t_s (kdtree.rs:79-87: intervals only shrink).  The
// build puts S in the low child iff lo_a <= s and in the high child iff hi_a >= s
// (kdtree.rs:119-127, lo/hi = fl(c -+ r), sphere.rs:106-114).  With d_a > 0: leaf k below the
// low (near) child without S needs t(lo_a) >= t_s >= x_k > E; below the high (far) child,
// t(hi_a) <= t_s <= e_k <= L*.  So t(near face) <= E and t(far face) > L* on every axis
// (faces swap for d_a < 0) put S in leaf k whatever the tree.  t(face) is the traversal's
// own arithmetic: the Markstein quotient with the ray's exact reciprocal, used only when
// equal to the division (face - o in mk range); otherwise the traversal runs.
//
// The face distances are only compared, so the quotients need not be computed exactly: with
// y = v_rcp_f32(d) (within 2 ulp of 1 / d; d clamped, |d| >= EPS) and q = RN(n * y), q lies within
// 2.5 * 2^-23 |q| of n / d, and the traversal's RN(n / d) within 3 * 2^-23 |q| < 2^-21 |q| of q.
// The bound is folded into the two thresholds once per ray: t(near) <= E follows from
// q <= E' <= E / (1 + 2^-21) (q <= 0 gives t <= 0 < E), and t(far) > L* from q > L' =
// RN(L* + L* 2^-20) >= L* / (1 - 2^-21).  E' = RN(L* (1 - 2^-17) - 2 EPS (1 + 2^-20)), one fma
// below E = RN(RN(L* - 2 EPS) - RN(L* 2^-18)) by more than the 2^-21 margin for every L* >=
// HIT_MIN (its coefficients undercut E's by 2^-18 L* and 2^-20 2 EPS, which exceed the roundings;
// tests/test_small_bound.py).  A true result is therefore true for the exact quotients; a
// marginal case just falls back to the traversal.  (|n| < 2^59 (small_ok) and |y| <= 1 / EPS: no
// overflow.  A product that underflows has |q| < 2^-100 and an exact quotient as tiny: both are
// below E's floor ~1.7e-3 and L* >= HIT_MIN, so the comparisons agree.  Only a ray with a hit
// gets here, so o and d are finite: dot(d, o - c) involves every component.)
//
// With r >= 0 (small_ok) the near face's quotient is the smaller of the two faces' on every axis
// and the far face's the larger (RN is monotone in the face and the sign of y orders them), so
// the test is min over axes of the far quotients > L' and max over axes of the near ones <= E'.
//
// The root slab test (aabb.rs:22-62) needs no arithmetic of its own when this holds: the scene
// box contains S's box (runtime.hip checks it for small_ok), so on every axis the box's far face
// is at least as far along the ray as S's and its near face at most as far (RN is monotone in
// the face), and the slab's products RN(RN(face - o) * RN(1 / d)) lie within 2^-23 of the exact
// quotients.  With the bounds above, every far product exceeds L* and every near one is below
// E < L*: entry <= L* <= exit, the slab test passes and fl(exit + EPS) >= L*, which is what the
// shortcut needs.  Lanes that fail it compute the exact slab and take the traversal.
// lo / hi: S's box faces fl(c -+ r) (g_lds_lo / g_lds_hi).
__device__ __forceinline__ bool in_return_leaf(float4 lo, float4 hi, const Ray& r, float ls) {
    const float en = fmaf(ls, 1.0f - 0x1p-17f, -2.0f * EPS * (1.0f + 0x1p-20f));  // E'
    const float lf = fmaf(ls, 0x1p-20f, ls);                                      // L'
    // the EPS-clamped direction of the traversal (kdtree.rs:75-77): d itself unless some lane of
    // the wave has a component below EPS (~2% of a wave's segments)
    V3 dc = r.d;
    if (__builtin_expect(__ballot(fminf(fminf(fabsf(dc.x), fabsf(dc.y)), fabsf(dc.z)) < EPS) != 0, 0))
        dc = mk(clamp_eps(dc.x), clamp_eps(dc.y), clamp_eps(dc.z));
    const float yx = __builtin_amdgcn_rcpf(dc.x), yy = __builtin_amdgcn_rcpf(dc.y), yz = __builtin_amdgcn_rcpf(dc.z);
    const float lx = (lo.x - r.o.x) * yx, hx = (hi.x - r.o.x) * yx;
    const float ly = (lo.y - r.o.y) * yy, hy = (hi.y - r.o.y) * yy;
    const float lz = (lo.z - r.o.z) * yz, hz = (hi.z - r.o.z) * yz;
    const float vp = fmaxf(fmaxf(fminf(lx, hx), fminf(ly, hy)), fminf(lz, hz));
    const float wp = fminf(fminf(fmaxf(lx, hx), fmaxf(ly, hy)), fmaxf(lz, hz));
    return vp <= en && wp > lf;
}

// KdTree::closest_ray_hit (kdtree.rs:58-64): root slab test, stack search, then the
// unconditional renderables.  The Markstein division is used for the whole wave unless some
// lane's origin (or the scene's splits) could underflow it.
// Small sphere scenes (<= 32 spheres, all in LDS): an exact shortcut of the same traversal.
// The reference returns the first leaf, front to back, whose best hit l satisfies
// l <= exit + EPS (kdtree.rs:96).  With L* the closest valid hit over all spheres, a leaf
// with fl(exit + EPS) < L* can never return.  Descending from entry E, where
// fl(E + EPS) < L* holds for every value <= E, skips exactly such leaves (a near child whose
// interval ends at or before E is not entered) and leaves every other leaf's interval, order
// and exit untouched — so the returned sphere and distance are the reference's.  Most rays
// need no descent at all (in_return_leaf).  The instrumented kernel counts the reference's work with the plain traversal and the device's
// work (count_device) through this function.
template <bool COUNT, bool RESTART = false>
__device__ __forceinline__ bool closest_small(const DevScene& sc, const Ray& r, Hit* best,
                                              uint32_t* st, Ctr<COUNT>& c) {
    uint32_t imin = 0;
    bool any = false;
    float ls = __builtin_inff();
    if (COUNT) c.sph += sc.n_spheres;
    // Spheres in pairs: the two discriminants are independent, so their arithmetic interleaves
    // (the per-sphere skip branch keeps the compiler from overlapping consecutive iterations).
    auto take = [&](const SphDisc& q, uint32_t i) {
        if (__builtin_expect(__ballot(q.thing2 > 0.0f) == 0, 0)) return;  // v false on every lane
        RC(RC_ROOTS);
        float l;
        const bool v = sphere_roots<false>(q, &l) & !(l < HIT_MIN);
        any |= v;
        const bool better = v & (l < ls);  // first minimum in renderable order (closest_hit.rs:25)
#if RT_REGION_COUNT
        if (__ballot(better)) RC(RC_ROOTS_USEFUL);
        if (__ballot(q.thing2 > 0.0f && !(q.dir > 0.0f && q.dir * q.dir > q.thing2))) RC(RC_ROOTS_FRONT);
#endif
        imin = better ? i : imin;
        ls = better ? l : ls;
    };
    uint32_t i = 0;
    for (; i + 1 < sc.n_spheres; i += 2) {
        const float4 sa = g_lds_csq[i], sb = g_lds_csq[i + 1];
        const SphDisc qa = sphere_disc(sa, sa.w, r), qb = sphere_disc(sb, sb.w, r);
        take(qa, i);
        take(qb, i + 1);
    }
    if (i < sc.n_spheres) {
        const float4 sa = g_lds_csq[i];
        take(sphere_disc(sa, sa.w, r), i);
    }
    if (any) {
        RC(RC_SLAB);
        // (COUNT here means the device-work count: closest_small never runs for the reference's)
        if (in_return_leaf(g_lds_lo[imin], g_lds_hi[imin], r, ls)) {
            best->ref = (K_SPHERE << REF_KIND_SHIFT) | imin;
            best->l = ls;
            best->bu = best->bv = 0.f;
            return true;
        }
        RC(RC_FALLBACK);
        float root_entry, root_exit;
        const RayAx ax = ray_axes(r);
        if (entry_exit(sc.bounds, ax, r, &root_entry, &root_exit)) {
            // fl(x + EPS) < L* for all x <= E: margin 2 EPS + 2^-18 L* (>> rounding of L*)
            const float e = (ls - 2.0f * EPS) - ls * 0x1p-18f;
            const float entry = fmaxf(root_entry, e);
            bool found;
            const bool fast = sc.fastdiv && origin_fast_ok(r.o);
            if (__builtin_expect(__ballot(!fast) == 0, 1))
                found = stack_search<COUNT, false, true, true, RESTART>(sc, r, ax, entry, root_exit, best, st, c, imin, ls);
            else
                found = stack_search<COUNT, false, false, true, RESTART>(sc, r, ax, entry, root_exit, best, st, c, imin, ls);
            if (found) return true;
        }
    }
    if (sc.has_cube) {
        best->ref = REF_CUBE;
        best->l = __builtin_inff();
        return true;
    }
    return false;
}

template <bool COUNT, bool GEN, bool RESTART = false>
__device__ __forceinline__ bool closest(const DevScene& sc, const Ray& r, Hit* best,
                                        uint32_t* st, Ctr<COUNT>& c) {
    if (!GEN && (!COUNT || sc.count_device) && sc.n_spheres <= 32u && sc.small_ok)
        return closest_small<COUNT, RESTART>(sc, r, best, st, c);
    float root_entry, root_exit;
    const RayAx ax = ray_axes(r);
    if (sc.n_nodes && entry_exit(sc.bounds, ax, r, &root_entry, &root_exit)) {
        bool found;
        const bool fast = sc.fastdiv && origin_fast_ok(r.o);
        if (__builtin_expect(__ballot(!fast) == 0, 1))
            found = stack_search<COUNT, GEN, true, false, RESTART>(sc, r, ax, root_entry, root_exit, best, st, c);
        else
            found = stack_search<COUNT, GEN, false, false, RESTART>(sc, r, ax, root_entry, root_exit, best, st, c);
        if (found) return true;
    }
    // unconditional renderables: every cube map hits at +inf, the first one wins
    if (sc.has_cube) {
        best->ref = REF_CUBE;
        best->l = __builtin_inff();
        return true;
    }
    return false;
}

// The scene arrays the packet traversal reads, as __restrict__ kernel arguments: loads from
// them that are wave-uniform then compile to scalar loads (s_load), which take the scalar
// memory path beside the vector-memory pipeline (TA/TD) that bounds the cooperative passes.
struct PkScene {
    const uint2* nodes;
    const uint32_t* refs;
    const float4* prim4;
};

// ------------------------------------------------------------ cooperative leaf tests (meshes)
// With one lane per ray, a wave tests leaf refs for as long as its *longest* leaf: mesh leaves
// average ~23 refs and the longest of 64 is ~4x that, so 3/4 of the lanes idle (biplane: 24%
// VALU lane utilisation).  Here every lane of the wave reaches its next leaf, then the wave
// tests all their (ray, ref) pairs as one list, 64 at a time: a pair's owner comes from a
// binary search over the wave's inclusive prefix of leaf sizes, and the owner's ray and leaf
// are read with cross-lane shuffles.  Each owner's leaf minimum is an LDS atomicMin on
// (bits(l) << 32 | position in the leaf): positive floats order like their bit patterns, so this
// is the first strict minimum in leaf order (closest_hit.rs:25), exactly; NaN lengths never
// win (see leaf_closest).  The owner then re-tests the winning ref for its barycentrics.
__shared__ unsigned long long g_coop_key[BLOCK];

// Inclusive prefix maximum over the 64 lanes (the DPP pattern of wave_incl_scan with max).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}

// Inclusive prefix sum over the 64 lanes.  DPP (GFX9): row_shr 1/2/4/8 with bound control
// (lanes shifted in from outside the 16-lane row read 0) scans each row; row_bcast:15 adds row
// r's total to row r+1 for rows 1 and 3, row_bcast:31 adds rows 0-1's total to rows 2-3.  No
// LDS, no per-lane address registers (the ds_bpermute form kept six of them live).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
    (void)lane;
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return v;
}

// Owner of item w of a wave-wide list: the number of lanes whose inclusive end (incl) is <= w.
__device__ __forceinline__ uint32_t list_owner(uint32_t incl, uint32_t w) {
    uint32_t owner = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1) {
        const uint32_t e = __shfl(incl, owner + step - 1);
        owner += e <= w ? step : 0u;
    }
    return owner;
}

// Owner of item w (= base + lane) of a pass.  owner(w) = #lanes with incl <= w: lanes below o_lo
// end at or before the pass's first item and lanes from o_hi on after its last one (incl is
// non-decreasing), so when few leaves end inside the pass only the lanes in between are compared,
// by readlane (scalar operands, no LDS round trip); otherwise the binary search of list_owner.
// Every lane of the wave calls this with the same base.
__device__ __forceinline__ uint32_t pass_owner(uint32_t incl, uint32_t total, uint32_t base, uint32_t w) {
    if (RT_OWNER_LOOP > 0) {
        const uint32_t last = min(base + 63u, total - 1u);
        const uint32_t o_lo = (uint32_t)__popcll(__ballot(incl <= base));
        const uint32_t o_hi = (uint32_t)__popcll(__ballot(incl <= last));
        if (o_hi - o_lo <= (uint32_t)RT_OWNER_LOOP) {
            uint32_t owner = o_lo;
            for (uint32_t k = o_lo; k < o_hi; ++k)
                owner += w >= (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)k) ? 1u : 0u;
            return owner;
        }
    }
    return list_owner(incl, w);
}

// Every lane of the wave must call this (all active); lanes without a leaf pass cnt = 0.
// Returns the lane's leaf minimum as (bits(l) << 32 | index into sc.refs), ~0 for none; one
// leaf's refs are contiguous, so the index orders like the position in the leaf.  `key0` is
// the lane's minimum over refs it tested itself (the leaf's leading spheres).
__device__ __forceinline__ unsigned long long coop_leaf(const DevScene& sc, const Ray& r, uint32_t off,
                                                        uint32_t cnt, uint32_t lane, unsigned long long key0) {
    const uint32_t incl = wave_incl_scan(cnt, lane);
    const uint32_t total = __shfl(incl, 63);
    const uint32_t wbase = threadIdx.x & ~63u;
    unsigned long long* const keys = g_coop_key;
    __hip_atomic_store(&keys[threadIdx.x], key0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    // item w of a lane's leaf is sc.refs[w + delta]
    const uint32_t delta = off - (incl - cnt);
    for (uint32_t base = 0; base < total; base += 64) {
        VC(11, 1);
        const uint32_t w = base + lane;
        const uint32_t owner = pass_owner(incl, total, base, w);
        const uint32_t idx = w + __shfl(delta, owner);
        Ray ro;
        ro.o = mk(__shfl(r.o.x, owner), __shfl(r.o.y, owner), __shfl(r.o.z, owner));
        ro.d = mk(__shfl(r.d.x, owner), __shfl(r.d.y, owner), __shfl(r.d.z, owner));
        if (w < total) {
            // the primitive's three float4 are loaded before the kind is known (a sphere's are
            // {c, r} and padding): one round trip to L2 after the ref, not two
            VC(2, 1);
            VL(2, sc.refs + idx, 4, true);
            const uint32_t ref = sc.refs[idx];
            VC(3, 3);
            const float4* pd = prim_data(sc, ref);
            VL(3, pd, 16, true);
            VL(3, pd + 1, 16, true);
            VL(3, pd + 2, 16, true);
            const float4 a0 = pd[0], a1 = pd[1], a2 = pd[2];
            float l = 0.f, bu, bv;
            bool h;
            if (__builtin_expect((ref >> REF_KIND_SHIFT) == K_SPHERE, 0)) h = sphere_hit(a0, ro, &l);
            else h = tri_hit(xyz(a0), xyz(a1), xyz(a2), ro, &l, &bu, &bv);
            if (h && l >= HIT_MIN)  // valid and not NaN
                atomicMin(&keys[wbase + owner], ((unsigned long long)__float_as_uint(l) << 32) | idx);
        }
    }
    return __hip_atomic_load(&keys[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// stack_search with cooperative leaves: the same per-lane traversal (kdtree.rs:66-104); lanes
// whose search has ended (or that had no ray) keep looping as helpers until the wave is done.
//
// RESTART (stackless, kd-restart with push-down): no stack.  After a leaf that does not return,
// the descent starts again with entry = that leaf's exit, from the deepest node the previous
// descent reached before its first push (every node above it went near with the full interval
// or far, and still does with the larger entry).  It reaches the reference's next leaf with the
// same interval, bit for bit: the deepest push has t = the new entry exactly (the same quotient
// of the same operands), so it now goes far — the reference's pop — while the shallower pushes,
// whose t is strictly larger, go near again with exit = their t, as their stack entries would
// have left it.  The remaining interval is empty exactly when the descent pushed nothing
// (exit == root exit), the reference's empty stack.
template <bool FAST, bool RESTART>
__device__ __forceinline__ bool stack_search_coop(const DevScene& sc, const Ray& r, const RayAx& ax,
                                                  bool active, float root_entry, float root_exit, Hit* best,
                                                  uint32_t* st) {
    float entry = root_entry, exit_t = root_exit, top_t = root_exit;
    uint32_t node = 0, restart = 0;
    int sp = 0;
    bool done = !active, found = false, pushed = false;
    const uint32_t lane = __lane_id();
    // RT_LEAF_REUSE: the previous leaf's list (its offset in sc.refs: the upload gives identical
    // lists one copy, so equal offsets mean equal lists) and its minimum key
    uint32_t prev_list = ~0u;
    unsigned long long prev_key = ~0ull;
    // After a leaf that does not return: the reference's pop (or the kd-restart); false when the
    // interval is exhausted (the reference's empty stack).
    // !RESTART: the pop after a leaf that does not return needs two nodes, the branch it returns to
    // (its b word: children and axis) and the branch below it (the new exit); both are loaded ahead
    // of the leaf's passes, so their trip to L1 / L2 overlaps the passes instead of following them
    // (A/B at 4-10 spp: a380 and biplane +4..7%, spaceship +-0; the bench configs +-0)
    uint32_t pop_b = 0;
    uint2 below = make_uint2(0u, 0u);
    auto advance = [&]() -> bool {
        if (RESTART ? !pushed : sp == 0) return false;
        if (RESTART) {
            entry = exit_t;
            exit_t = root_exit;
            node = restart;
        } else {
            --sp;
            // the popped branch's node and the one below it were loaded before the leaf's passes
            float d;
            (void)split_t<FAST>(make_uint2(0u, pop_b), ax, r, &d);
            node = (pop_b >> 2) + (d > 0.0f ? 1u : 0u);
            entry = top_t;
            if (sp) {
                top_t = split_t<FAST>(below, ax, r, &d);
                exit_t = top_t;
            } else {
                exit_t = root_exit;
            }
        }
        return true;
    };
    while (__ballot(!done) != 0) {
        uint32_t off = 0, cnt = 0, list = ~0u;
        unsigned long long key0 = ~0ull;
        VC(12, 1);
        if (!done) {
            uint2 nd = fetch_node(sc, node);
            pushed = false;
            VC(0, 1);
            VL(0, sc.nodes + node, 8, true);
            while ((nd.y & 3u) != RT_KD_LEAF) {
                VC(0, 1);
                // RT_PAIR_FETCH: both children (adjacent, 16 B: one global_load_dwordx4) are
                // loaded before this node's decision, so the next level's fetch overlaps the
                // decision's arithmetic
                const uint32_t cpair = nd.y >> 2;
                uint4 pair = make_uint4(0u, 0u, 0u, 0u);
                VL(0, sc.nodes + cpair, 16, true);
                if (RT_PAIR_FETCH) {
                    {
                        const uint2* pp = sc.nodes + cpair;
                        const uint2 c0 = pp[0], c1 = pp[1];
                        pair = make_uint4(c0.x, c0.y, c1.x, c1.y);
                    }
                }
                float d;
                const float t = split_t<FAST>(nd, ax, r, &d);
                const bool pos = d > 0.0f;
                const bool go_near = t >= exit_t;
                const bool go_far = !go_near && t <= entry;
                const bool push = !go_near && !go_far;
                if (!RESTART) {
                    st[sp * BLOCK] = node;
                    sp += push ? 1 : 0;
                    top_t = push ? t : top_t;
                }
                exit_t = push ? t : exit_t;
                node = (nd.y >> 2) + (go_far == pos ? 1u : 0u);
                if (RESTART) {
                    pushed = pushed || push;
                    restart = pushed ? restart : node;
                }
                if (RT_PAIR_FETCH) {
                    nd = node == cpair ? make_uint2(pair.x, pair.y) : make_uint2(pair.z, pair.w);
                } else {
                    nd = fetch_node(sc, node);
                }
            }
            off = nd.y >> 2;
            cnt = nd.x & LEAF_COUNT_MASK;
            list = off;
            if (RT_LEAF_REUSE && cnt && off == prev_list) {
                // The same ray against the same refs in the same order: every length, and so
                // the first strict minimum and its position, is the previous leaf's.  Only
                // the return test (this leaf's exit) differs.
                key0 = prev_key;
                cnt = 0;
            } else {
                // The leaf's leading spheres (a scene's lights span most leaves) are this
                // lane's own tests; the wave's passes then hold triangles only.
                const uint32_t lead = nd.x >> LEAF_LEAD_SHIFT;
                for (uint32_t j = 0; j < lead; ++j) {
                    VC(4, 2);
                    float l;
                    const uint32_t sref = sc.refs[off + j];
                    VL(4, prim_data(sc, sref), 16, true);
                    const float4 sph = prim_data(sc, sref)[0];
                    if (sphere_hit(sph, r, &l) && l >= HIT_MIN)
                        key0 = min(key0, ((unsigned long long)__float_as_uint(l) << 32) | (off + j));
                }
                off += lead;
                cnt -= lead;
            }
        }
        if (!RESTART && !done && sp > 0) {  // the pop after this leaf (if it does not return)
            VC(1, sp > 1 ? 2 : 1);
            VL(1, sc.nodes + st[(sp - 1) * BLOCK], 8, true);
            pop_b = fetch_node(sc, st[(sp - 1) * BLOCK]).y;
            if (sp > 1) below = fetch_node(sc, st[(sp - 2) * BLOCK]);
        }
        DIAG_ROUND_SHARING(off, cnt);
        TM_VAR(const unsigned long long tmc0 = TM_NOW());
        const unsigned long long key = coop_leaf(sc, r, off, cnt, lane, key0);
        TM_ADD(12, TM_NOW() - tmc0);
        TM_ADD(13, (__shfl(wave_incl_scan(cnt, lane), 63) + 63u) / 64u);
        if (!done) {
            if (RT_LEAF_REUSE) {
                prev_list = list;
                prev_key = key;
            }
            // The leaf returns its closest valid hit iff l <= exit + EPS; the key holds l's bits
            // (the re-test below computes the same l), so only a returning leaf re-tests its
            // winner for the barycentrics (biplane's light sphere, in every leaf, used to be
            // re-tested after every leaf).
            bool ret = key != ~0ull && __uint_as_float((uint32_t)(key >> 32)) <= exit_t + EPS;
            if (ret) {
                VC(5, 4);
                const uint32_t ref = sc.refs[(uint32_t)key];
                VL(5, sc.refs + (uint32_t)key, 4, true);
                VL(5, prim_data(sc, ref), 48, true);
                const float4* pd = prim_data(sc, ref);
                const float4 a0 = pd[0], a1 = pd[1], a2 = pd[2];
                float l = 0.f, bu = 0.f, bv = 0.f;
                if ((ref >> REF_KIND_SHIFT) == K_SPHERE) (void)sphere_hit(a0, r, &l);
                else (void)tri_hit(xyz(a0), xyz(a1), xyz(a2), r, &l, &bu, &bv);
                best->ref = ref;
                best->l = l;
                best->bu = bu;
                best->bv = bv;
                done = true;
                found = true;
            } else if (!advance()) {
                done = true;
            }
        }
    }
    return found;
}

// ------------------------------------------------------------ packet traversal (camera rays)

// Camera rays of one wave traced as a packet: lanes `pk` share the signs of their (EPS-clamped)
// directions, so every branch orders its children the same way for all of them.  The packet
// walks the tree from the root, the wave-uniform node fetched by a scalar load, each lane
// deciding near / far / both on its own interval exactly as kdtree.rs:79-87 does; where some
// lanes need the near child, the lanes that need only the far one are deferred.  At the leaf the
// lanes still active test its refs one at a time, the primitive in scalar registers (no
// per-lane gather; the next ref's primitive is loaded during the current test), keeping the
// first strict minimum (closest_hit.rs:25), and return it if l <= exit + EPS (kdtree.rs:96).
// A lane that does not return restarts from the root with entry = that leaf's exit (kd-restart
// with push-down, as in stack_search_coop); deferred lanes restart with their entry unchanged.
// Either way a lane's next leaf and its interval are those of the reference's stack traversal,
// bit for bit ("Packet traversal"), so each lane visits exactly its own leaves in
// its own order.  Called by every lane of the wave.
// A leaf visit costs the packet a descent and one test per ref at the whole wave's width, so
// once fewer than RT_PACKET_KEEP lanes reach the packet's next leaf the packet stops: its lanes
// still searching (`live`) continue in the cooperative search from interval [entry, root_exit],
// where the reference's stack traversal visits the same remaining leaves (kd-restart argument).
constexpr int RT_PACKET_KEEP = 40;
constexpr int RT_PACKET_SIDE = 1;  // 1: at a branch the packet follows the child more of its active lanes need (the others deferred)

template <bool FAST>
__device__ bool closest_packet(const PkScene& ps, const Ray& r, const RayAx& ax, bool pk, float& entry,
                               float root_exit, Hit* best, bool& live) {
    float exit_t = root_exit;
    bool found = false;
    live = pk;
    const uint32_t lead = (uint32_t)__ffsll((unsigned long long)__ballot(pk)) - 1u;
    // near child of a branch on axis a: low when the (shared) clamped d_a > 0
    const uint32_t pos_bits = (uint32_t)__builtin_amdgcn_readlane(
        (int)((ax.dx > 0.0f ? 1u : 0u) | (ax.dy > 0.0f ? 2u : 0u) | (ax.dz > 0.0f ? 4u : 0u)), (int)lead);
    // Restart node: the deepest node a descent reached before any live lane pushed or was
    // deferred.  Above it every live lane went near with its whole interval (t >= exit = root
    // exit) or far with t <= entry, and still does with a larger entry, so all of their
    // remaining intervals lie below it (the per-lane argument of stack_search_coop, for the
    // packet as a whole); it only moves down.
    uint32_t restart = 0;
    while (__ballot(live)) {
        bool act = live, pushed = false, clean = true;
        uint32_t node = restart;
        uint2 nd = ps.nodes[node];
        while ((nd.y & 3u) != RT_KD_LEAF) {
            float t = 0.f;
            bool go_far = false, push = false;
            if (act) {
                float d;
                t = split_t<FAST>(nd, ax, r, &d);
                const bool go_near = t >= exit_t;
                go_far = !go_near && t <= entry;
                push = !go_near && !go_far;
            }
            const bool pos = (pos_bits >> (nd.y & 3u)) & 1u;
            node = nd.y >> 2;
            const uint32_t n_near = (uint32_t)__popcll(__ballot(act && !go_far));
            const uint32_t n_far = (uint32_t)__popcll(__ballot(act && go_far));
            if (n_near && (!RT_PACKET_SIDE || n_near >= n_far)) {  // near child, with the lanes that need it
                clean = clean && __ballot(act && (go_far || push)) == 0;
                act = act && !go_far;
                exit_t = act && push ? t : exit_t;
                pushed = pushed || (act && push);
                node += pos ? 0u : 1u;
            } else {  // far child, with the lanes that need only it; the others are deferred
                clean = clean && n_near == 0;
                act = act && go_far;
                node += pos ? 1u : 0u;
            }
            restart = clean ? node : restart;
            nd = ps.nodes[node];
        }
        if (RT_PACKET_KEEP > 0 && __popcll(__ballot(act)) < RT_PACKET_KEEP) break;
        VC(10, 1);
        TM_ADD(3, 1);
        TM_ADD(4, __popcll(__ballot(act)));
        TM_ADD(5, nd.x & LEAF_COUNT_MASK);
        // the leaf: active lanes test every ref, first strict minimum
        const uint32_t off = nd.y >> 2, cnt = nd.x & LEAF_COUNT_MASK;
        bool lf = false;
        float ll = 0.f, lu = 0.f, lv = 0.f;
        uint32_t lref = 0;
        // software pipeline: during the test of ref j, the primitive of ref j + 1 and the ref
        // j + 2 are in flight (uploads carry zero padding past the end of refs).  An empty leaf
        // reads nothing (cnt is wave-uniform: the node is).
        uint32_t ref_n = 0, ref_nn = 0;
        const float4* pn = ps.prim4;
        float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0, b2 = b0;
        if (cnt) {
            ref_n = ps.refs[off];
            ref_nn = ps.refs[off + 1];
            pn = ps.prim4 + 3 * (size_t)(ref_n & REF_INDEX_MASK);
            b0 = pn[0];
            b1 = pn[1];
            b2 = pn[2];
        }
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t ref = ref_n;
            const float4 a0 = b0, a1 = b1, a2 = b2;
            if (j + 1 < cnt) {
                ref_n = ref_nn;
                ref_nn = ps.refs[off + j + 2];
                pn = ps.prim4 + 3 * (size_t)(ref_n & REF_INDEX_MASK);
                b0 = pn[0];
                b1 = pn[1];
                b2 = pn[2];
            }
            if (act) {
                float l = 0.f, bu = 0.f, bv = 0.f;
                bool h;
                if ((ref >> REF_KIND_SHIFT) == K_SPHERE) h = sphere_hit(a0, r, &l);
                else h = tri_hit(xyz(a0), xyz(a1), xyz(a2), r, &l, &bu, &bv);
                const bool take = h && l >= HIT_MIN && (!lf || l < ll);  // valid, not NaN, first minimum
                ll = take ? l : ll;
                lu = take ? bu : lu;
                lv = take ? bv : lv;
                lref = take ? ref : lref;
                lf = lf || take;
            }
        }
        if (act) {
            if (lf && ll <= exit_t + EPS) {
                best->ref = lref;
                best->l = ll;
                best->bu = lu;
                best->bv = lv;
                found = true;
                live = false;
            } else if (!pushed) {
                live = false;  // the interval is exhausted: the reference's empty stack
            } else {
                entry = exit_t;
            }
        }
        exit_t = root_exit;
    }
    return found;
}

// closest() for the general queue kernel: called by every lane of the wave; `active` lanes
// have a ray.
template <bool RESTART>
__device__ __forceinline__ bool closest_coop(const DevScene& sc, const Ray& r, Hit* best,
                                             uint32_t* st, bool active, bool camera = false,
                                             const PkScene* ps = nullptr) {
    float root_entry = 0.f, root_exit = 0.f;
    const RayAx ax = ray_axes(r);
    const bool in = active && sc.n_nodes && entry_exit(sc.bounds, ax, r, &root_entry, &root_exit);
    bool found = false;
    const bool fast = !in || (sc.fastdiv && origin_fast_ok(r.o));
    const bool all_fast = __ballot(!fast) == 0;
    bool pk = false, pk_live = false;
    TM_VAR(const unsigned long long tm0 = TM_NOW());
    if (RT_PACKET && ps && sc.packet) {
        // camera rays of the direction octant of the first one form the packet (NaN directions
        // never: d > 0 and d < 0 are both false); the other lanes take the cooperative search
        const uint32_t oct = (ax.dx > 0.0f ? 1u : 0u) | (ax.dy > 0.0f ? 2u : 0u) | (ax.dz > 0.0f ? 4u : 0u);
        const bool num = !__builtin_isnan(ax.dx) && !__builtin_isnan(ax.dy) && !__builtin_isnan(ax.dz);
        const bool cand = in && camera && num;
        const uint64_t cm = __ballot(cand);
        if (__popcll(cm) >= RT_PACKET_MIN) {
            const uint32_t lead = (uint32_t)__ffsll((unsigned long long)cm) - 1u;
            pk = cand && oct == (uint32_t)__builtin_amdgcn_readlane((int)oct, (int)lead);
            if (__popcll(__ballot(pk)) >= RT_PACKET_MIN) {
                found = all_fast ? closest_packet<true>(*ps, r, ax, pk, root_entry, root_exit, best, pk_live)
                                 : closest_packet<false>(*ps, r, ax, pk, root_entry, root_exit, best, pk_live);
            } else {
                pk = false;
            }
        }
    }
    const bool in_coop = in && (!pk || pk_live);
    TM_VAR(const unsigned long long tm1 = TM_NOW());
    TM_ADD(0, tm1 - tm0);
    TM_ADD(6, __popcll(__ballot(pk)));
    TM_ADD(7, __popcll(__ballot(pk && pk_live)));
    TM_ADD(8, __popcll(__ballot(in_coop)));
    if (__ballot(in_coop)) {
        if (__builtin_expect(all_fast, 1))
            found = stack_search_coop<true, RESTART>(sc, r, ax, in_coop, root_entry, root_exit, best, st) || found;
        else
            found = stack_search_coop<false, RESTART>(sc, r, ax, in_coop, root_entry, root_exit, best, st) || found;
    }
    TM_ADD(1, TM_NOW() - tm1);
    if (found) return true;
    if (active && sc.has_cube) {
        best->ref = REF_CUBE;
        best->l = __builtin_inff();
        return true;
    }
    return false;
}

// ---------------------------------------------------------------- materials (interaction.rs)
__device__ __forceinline__ float draw(rt_rng_state* rng) { return rt_rng_next_f32(rng); }

// Every continued direction of interaction.rs ends in a normalize, and so does the camera ray.
// The *_vec functions (and the mirror direction, computed inline) return the vector before it, and segment() normalizes once at its start:
// a wave whose lanes hit diffuse, mirror and glass spheres, or start new paths, runs one
// normalize at full width instead of one per branch at partial width.  Each lane still
// normalizes exactly the vector the reference does.
// dn = dot(d, n), shared by the callers' branches
__device__ __forceinline__ V3 diff_vec(V3 d, V3 n, float dn, rt_rng_state* rng) {  // :11-27
    V3 xd = normalize(d - n * dn);
    V3 yd = normalize(cross(n, xd));
    float u = draw(rng);
    float v = draw(rng);
    float r = sqrt_draw(u);
    float thet = 2.0f * PI * v;
    float sn, cs;
    (void)rt_sincosf(thet, &sn, &cs);  // glibc's sinf, cosf (rt_libm.h); thet in [0, 2 pi)
    float x = r * cs;
    float y = r * sn;
    // max(1 - u, 0) is 1 - u: u <= 1 - 2^-24
    return (xd * x + yd * y) + n * sqrt_draw(1.0f - u);
}
// over_in = n_out / n_in, over_out = n_in / n_out and r0 come precomputed (DevMat): the
// divisions n1 / n2 and (n1 - n2) / (n1 + n2) of :35,48 depend on the material only.
// Returns the reflected or transmitted vector, to be normalized by the caller.
// dn = dot(d, n) (= dot(n, d): products commute) and refl = d - 2n(d.n), the mirror direction
// of :6-9, come from the caller; the mirror about -n is the same vector bit for bit (each
// negation is exact).
// glibc's powf(x, 5) (include/rt_libm.h); the diagnostic region build counts the slow path.
__device__ __forceinline__ float pow5(float x) {
#if RT_REGION_COUNT
    float f;
    if (rt_powf5_fast(x, &f)) return f;
    RC(RC_POW_SLOW);
    return rt_powf5_glibc(x);
#else
    return rt_powf5(x);
#endif
}

__device__ __forceinline__ V3 refract_vec(V3 d, V3 n, float dn, V3 refl, float over_in, float over_out,
                                          float r0, float* p, rt_rng_state* rng) {  // :29-59
    float c_ = dn;
    bool into = c_ < 0.0f;
    float c1 = into ? -c_ : c_;
    V3 norm_refr = into ? n : -n;
    float n_over = into ? over_in : over_out;
    float c22 = 1.0f - n_over * n_over * (1.0f - c1 * c1);
    if (c22 < 0.0f) { *p = 1.0f; return refl; }
    V3 trns = n_over * d + norm_refr * (n_over * c1 - sqrt_nonneg(c22));  // c22 >= 0 here
    float c = 1.0f - (into ? c1 : dot(trns, n));
    float re = r0 + (1.0f + r0) * pow5(c);  // glibc's powf(c, 5)
    float u = draw(rng);
    if (u < re) { *p = re; return refl; }
    *p = 1.0f - re;
    return trns;
}

// k / 255.0f for an 8-bit k, bit for bit: the Markstein quotient with the exact reciprocal of
// 255 (div_mk; equal to the IEEE division for all 256 k, tests/test_device_code.py), k = 0 exact.
__device__ __forceinline__ float u8_over_255(uint32_t k) {
    const float r = 0x1.010102p-8f;  // RN(1 / 255)
    return div_mk((float)k, 255.0f, r);
}

// UVRgb32FImage::get_pixel (uv_image.rs:9-23): nearest texel, clamped, truncated; `as u32`
// maps NaN to 0.
__device__ __forceinline__ V3 get_pixel(const DevScene& sc, uint32_t off, uint32_t w, uint32_t h, float u,
                                        float v) {
    float width = (float)w, height = (float)h;
    float fx = fminf(fmaxf(u * width, 0.0f), width - 1.0f);
    float fy = fminf(fmaxf(v * height, 0.0f), height - 1.0f);
    uint32_t x = __builtin_isnan(fx) ? 0u : (uint32_t)truncf(fx);
    uint32_t y = __builtin_isnan(fy) ? 0u : (uint32_t)truncf(fy);
    const size_t i = (size_t)off + (size_t)y * w + x;
    VC(8, 1);
    VL(8, sc.texels8 ? (const void*)(sc.texels8 + i) : (const void*)(sc.texels + 3 * i), (sc.texels8 ? 4u : 12u), true);
    if (sc.texels8) {  // 4 B per texel instead of 12: each channel k / 255.0f, correctly rounded
        const uint32_t t = sc.texels8[i];
        return mk(u8_over_255(t & 0xffu), u8_over_255((t >> 8) & 0xffu), u8_over_255((t >> 16) & 0xffu));
    }
    return ld3(sc.texels + 3 * i);
}
__device__ __forceinline__ V3 tex_pixel(const DevScene& sc, int32_t t, float u, float v) {
    VC(8, 1);
    VL(8, sc.tex + t, 16, true);
    const DevTex tx = sc.tex[t];
    return get_pixel(sc, tx.off, tx.w, tx.h, u, v);
}

// DistantCubeMap::hit_info + sample_face + UVRgb32FImage::get_pixel
// (distant_cube_map.rs:27-69, uv_image.rs:9-23)
__device__ __forceinline__ V3 cube_emissive(const DevScene& sc, V3 rd) {
    int mi = 0;
    float mc = rd.x;
    if (fabsf(rd.y) > fabsf(mc)) { mi = 1; mc = rd.y; }
    if (fabsf(rd.z) > fabsf(mc)) { mi = 2; mc = rd.z; }
    if (!(mc < 0.0f) && !(mc > 0.0f)) return mk(0.f, 0.f, 0.f);
    V3 d = normalize(rd);
    bool neg = mc < 0.0f;
    float u, v, fact;
    int f;
    if (mi == 0) { u = d.z; v = d.y; fact = d.x; f = neg ? RT_FACE_NEG_X : RT_FACE_POS_X; }
    else if (mi == 1) { u = d.x; v = d.z; fact = d.y; f = neg ? RT_FACE_NEG_Y : RT_FACE_POS_Y; }
    else { u = d.x; v = d.y; fact = d.z; f = neg ? RT_FACE_NEG_Z : RT_FACE_POS_Z; }
    const DevFace fc = sc.face[f];
    float u1 = u * fc.us / fact, v1 = v * fc.vs / fact;
    return get_pixel(sc, fc.off, fc.w, fc.h, 0.5f * u1 + 0.5f, 0.5f * v1 + 0.5f);
}

// ---------------------------------------------------------------- camera (generate.rs:24-66)
// The pixel's base direction (cam_d + s_x right) + s_y up, before the lens and the jitter.
__device__ __forceinline__ V3 camera_base_dir(const DevScene& sc, int x, int y) {
    V3 up = ld3(sc.cam_up), right = ld3(sc.right);
    float s_x = sc.x_cf * ((float)x - sc.x_off);
    float s_y = sc.y_cf * ((float)y - sc.y_off);
    return (ld3(sc.cam_d) + s_x * right) + s_y * up;
}
__device__ __forceinline__ Ray camera_ray(const DevScene& sc, V3 d, rt_rng_state* rng) {
    V3 up = ld3(sc.cam_up), right = ld3(sc.right);
    Ray ray;
    if (sc.has_lens) {
        float a = sc.lens_r;
        float u = draw(rng);
        float v = draw(rng);
        float r = sqrt_draw(u);
        float thet = 2.0f * PI * v;
        float sn, cs;
        (void)rt_sincosf(thet, &sn, &cs);  // thet in [0, 2 pi)
        float lx = (r - 0.5f) * 2.0f * a * cs;
        float ly = (r - 0.5f) * 2.0f * a * sn;
        V3 off = right * lx + up * ly;
        ray.d = d - off;
        ray.o = off + ld3(sc.cam_o);
    } else {
        ray.d = d;
        ray.o = ld3(sc.cam_o);
    }
    float u = draw(rng) - 0.5f;
    float v = draw(rng) - 0.5f;
    ray.d = (ray.d + (right * u) * sc.x_cf) + (up * v) * sc.y_cf;
    return ray;  // d not yet normalized: segment() normalizes it (generate.rs:63)
}

// ---------------------------------------------------------------- one path segment (radiance.rs)
// State of the path a lane is tracing: the reference's recursion (radiance.rs:20-72) unrolled
// into L += T (x) e_k; T *= f_k.
struct Path {
    Ray ray;
    V3 L, T;
    int depth;
    rt_rng_state rng;
    // direct-light sampling (DLS kernels only): a DLS-eligible vertex waits for the next hit,
    // the second index establish_dls_contrib omits (radiance.rs:48-52)
    bool dls_on;
    uint32_t dls_ref;
    V3 dls_pos, dls_n, dls_T;
};
constexpr uint32_t REF_NONE = 0xfffffffeu;  // the continued ray hit nothing

// establish_dls_contrib (radiance.rs:89-120) for the vertex held in p.dls_*: every emissive
// sphere but the vertex's own element and `next` (the element the continued ray hit), seen
// along d = normalize(c - pos) with d.n > 0, whose brute-force shadow ray over all renderables
// returns that light as its first minimum, adds (d.n * emissive) * 1/(30 pi).  "First minimum
// is the light" = the light has a valid hit l and no renderable before it (renderable order)
// has a valid hit <= l, none after it one < l (closest_hit.rs:16-25; NaN never wins).
__device__ V3 dls_contrib(const DevScene& sc, const Path& p, uint32_t next) {
    const float NORMZE = 1.0f / (30.0f * PI);
    V3 acc = mk(0.f, 0.f, 0.f);
    for (uint32_t e = 0; e < sc.n_emit; ++e) {
        const uint2 em = sc.emit[e];
        const uint32_t eref = (K_SPHERE << REF_KIND_SHIFT) | em.x;
        if (eref == p.dls_ref || eref == next) continue;
        const float4 sp = sc.prim4[3 * (size_t)em.x];
        const V3 d = normalize(xyz(sp) - p.dls_pos);
        const float light_dot = dot(d, p.dls_n);
        if (!(light_dot > 0.0f)) continue;
        const Ray dr{d, p.dls_pos};
        float li;
        if (!sphere_hit(sp, dr, &li) || li < HIT_MIN) continue;
        bool occluded = false;
        for (uint32_t q = 0; q < sc.n_elem_refs && !occluded; ++q) {
            if (q == em.y) continue;
            const uint32_t ref = sc.elem_refs[q];
            const float4* pd = sc.prim4 + 3 * (size_t)(ref & REF_INDEX_MASK);
            float l = 0.f, bu, bv;
            const bool h = (ref >> REF_KIND_SHIFT) == K_SPHERE ? sphere_hit(pd[0], dr, &l)
                                                               : tri_hit(xyz(pd[0]), xyz(pd[1]), xyz(pd[2]), dr, &l, &bu, &bv);
            occluded = h && !(l < HIT_MIN) && (q < em.y ? l <= li : l < li);
        }
        if (occluded) continue;
        const V3 emi = ld3(sc.sph_mat[em.x].em);
        acc = acc + mk((light_dot * emi.x) * NORMZE, (light_dot * emi.y) * NORMZE, (light_dot * emi.z) * NORMZE);
    }
    return acc;
}

// tex_coord_from_bary (mesh/triangle.rs:228-237): sum from zero of coords[i_k] * b_k.
__device__ __forceinline__ void tex_coord(const float2* uv, const DevMeshTri& t, float b1, float b2, float* u,
                                          float* v) {
    float b0 = 1.0f - b2 - b1;
    VC(7, 3);
    VL(7, uv + t.v[0], 8, true);
    VL(7, uv + t.v[1], 8, true);
    VL(7, uv + t.v[2], 8, true);
    float2 c0 = uv[t.v[0]], c1 = uv[t.v[1]], c2 = uv[t.v[2]];
    float su = 0.0f, sv = 0.0f;
    su = su + c0.x * b0;
    sv = sv + c0.y * b0;
    su = su + c1.x * b1;
    sv = sv + c1.y * b1;
    su = su + c2.x * b2;
    sv = sv + c2.y * b2;
    *u = su;
    *v = sv;
}
__device__ __forceinline__ V3 mul3(const float* m, V3 v) {  // nalgebra gemv order
    return mk((m[0] * v.x + m[1] * v.y) + m[2] * v.z, (m[3] * v.x + m[4] * v.y) + m[5] * v.z,
              (m[6] * v.x + m[7] * v.y) + m[8] * v.z);
}

// Segment ending on a mesh triangle: MeshTriangle hit_info + continue_ray
// (triangle/generic.rs:59-92 with mesh/triangle.rs:136-225).  Draws: should_diff (1), RR (1 past
// assured_depth), diffuse (2), roughness scatter (3).  Triangles never emit.
template <bool COUNT>
__device__ __forceinline__ bool mesh_segment(const DevScene& sc, const Hit& h, uint32_t idx, Path& p,
                                          Ctr<COUNT>& c) {
    if (COUNT) c.mesh_hits++;
    VC(7, 6);  // the 64-B triangle record and the 32-B primitive record
    VL(7, sc.mtri + idx, 16, true);
    VL(7, reinterpret_cast<const char*>(sc.mtri + idx) + 16, 16, true);
    VL(7, reinterpret_cast<const char*>(sc.mtri + idx) + 32, 16, true);
    VL(7, reinterpret_cast<const char*>(sc.mtri + idx) + 48, 16, true);
    const DevMeshTri t = sc.mtri[idx];
    VL(7, sc.prims + t.prim, 32, true);
    const DevPrim pr = sc.prims[t.prim];
    const float b1 = h.bu, b2 = h.bv;
    V3 n;  // NormFromMesh::get_norm (:136-157)
    if (pr.normal_tex >= 0) {
        float u, v;
        tex_coord(sc.uv_norm, t, b1, b2, &u, &v);
        n = normalize(mul3(t.m, tex_pixel(sc, pr.normal_tex, u, v)));
    } else {
        V3 cum = mk(0.f, 0.f, 0.f);
        VC(7, 3);
        VL(7, sc.vnorm + t.v[0], 16, true);
        VL(7, sc.vnorm + t.v[1], 16, true);
        VL(7, sc.vnorm + t.v[2], 16, true);
        cum = cum + xyz(sc.vnorm[t.v[0]]);
        cum = cum + xyz(sc.vnorm[t.v[1]]);
        cum = cum + xyz(sc.vnorm[t.v[2]]);
        n = normalize(mul3(t.m, cum));
    }
    float metal = pr.metal, rough = pr.rough;  // divert_ray_seed (:190-207)
    if (pr.mr_tex >= 0) {
        float u, v;
        tex_coord(sc.uv_mr, t, b1, b2, &u, &v);
        V3 mr = tex_pixel(sc, pr.mr_tex, u, v);
        metal = mr.z * pr.metal;
        rough = mr.y * pr.rough;
    }
    const float r0 = 0.04f + (1.0f - 0.04f) * metal;
    const float reflectance = r0 + (1.0f - r0) * 1.0f * (1.0f - pow5(fabsf(dot(p.ray.d, n))));
    const bool should_diff = draw(&p.rng) < 1.0f - reflectance;  // DynDiffSpec::should_diff
    const V3 pos = (p.ray.d * h.l + p.ray.o) + n * EPS;
    if (sc.debug_single_ray) return true;
    bool atten = false;
    if (p.depth > sc.assured_depth) {
        if (!(draw(&p.rng) < RR_THRES)) return true;
        atten = true;
    }
    const float dn = dot(p.ray.d, n);
    V3 nd = normalize(should_diff ? diff_vec(p.ray.d, n, dn, &p.rng) : p.ray.d - (n * 2.0f) * dn);  // divert_new_ray
    const float su = draw(&p.rng), sv = draw(&p.rng), sw = draw(&p.rng);
    const V3 scatter = rough * normalize(mk(su, sv, sw));
    nd = nd + scatter;  // normalized at the start of the next segment
    V3 rgb = mk(pr.base_factor[0], pr.base_factor[1], pr.base_factor[2]);  // RgbFromMesh (:166-178)
    if (pr.base_tex >= 0) {
        float u, v;
        tex_coord(sc.uv_base, t, b1, b2, &u, &v);
        rgb = cmul(rgb, tex_pixel(sc, pr.base_tex, u, v));
    }
    rgb = rgb * 1.0f;
    if (atten) rgb = div3(rgb, RR_THRES);
    p.T = cmul(p.T, rgb);
    p.ray.d = nd;
    p.ray.o = pos;
    return ++p.depth >= MAX_BOUNCES;
}

// Traces one segment of `p`.  Returns true when the path has ended (miss, cube map, Russian
// roulette, debug_single_ray, bounce cap); p.L then holds the sample's radiance.
// Everything of a segment after its closest hit: hit_info, emission, Russian roulette and the
// continued ray.  Returns true when the path has ended.
template <bool COUNT, bool GEN, bool DLS>
__device__ __forceinline__ bool shade(const DevScene& sc, Path& p, Hit h, bool hit, Ctr<COUNT>& c) {
    if (DLS && p.dls_on) {  // the previous vertex's DLS term, now that its continued ray has hit
        p.L = p.L + cmul(p.dls_T, dls_contrib(sc, p, hit ? h.ref : REF_NONE));
        p.dls_on = false;
    }
    if (!hit) return true;  // miss: radiance 0
    if (COUNT) c.hits++;
    if (!GEN) RC(RC_SHADE_HIT);
    if (h.ref == REF_CUBE) {  // emissive only, no continue (distant_cube_map.rs:22,52-58)
        if (!GEN) RC(RC_CUBE);
        // (the reference still draws the RR uniform here; the stream ends with the path)
        p.L = p.L + cmul(p.T, cube_emissive(sc, p.ray.d));
        return true;
    }
    const uint32_t kind = h.ref >> REF_KIND_SHIFT, idx = h.ref & REF_INDEX_MASK;
    if (GEN && kind == K_MESH_TRI) return mesh_segment<COUNT>(sc, h, idx - sc.pool_mesh, p, c);
    V3 n, pos;
    const DevMat* m;
    if (GEN) VC(9, 6);
    if (!GEN || kind == K_SPHERE) {  // Sphere::hit_info (sphere.rs:64-80)
        float4 s = fetch_sphere<GEN>(sc, idx);
        V3 perfect = p.ray.o + p.ray.d * h.l;
        n = normalize(perfect - xyz(s));
        pos = perfect + n * EPS;
        m = GEN ? sc.sph_mat + idx : &g_lds_mat[idx];
    } else {  // FreeTriangle hit_info (generic.rs:78-92)
        n = xyz(sc.ftri_n[idx - sc.pool_ftri]);
        pos = (p.ray.d * h.l + p.ray.o) + n * EPS;
        m = sc.ftri_mat + (idx - sc.pool_ftri);
    }
    const uint32_t divert = m->divert;
    bool seed_diff = false;
    if (divert == RT_DIVERT_DIFFSPEC) {
        if (!GEN) RC(RC_SEED);
        seed_diff = draw(&p.rng) < m->diffp;  // generate_seed
    }
    p.L = p.L + cmul(p.T, ld3(m->em));  // triangles carry em = 0 (generic.rs:86)
    if (sc.debug_single_ray) return true;
    bool atten = false;  // russian_roulette_filter (radiance.rs:74-86)
    if (p.depth > sc.assured_depth) {
        if (!GEN) RC(RC_RR);
        if (!(draw(&p.rng) < RR_THRES)) return true;
        atten = true;
    }
    float prob = 1.0f;  // gen_new_ray (uniform_diff_spec.rs:44-68)
    // d.n and the mirror direction are shared by the three branches (computed once, full width)
    const float dn = dot(p.ray.d, n);
    const V3 refl = p.ray.d - (n * 2.0f) * dn;  // spec (interaction.rs:6-9)
    V3 nd;
    if (divert == RT_DIVERT_SPEC || (divert == RT_DIVERT_DIFFSPEC && !seed_diff)) {
        if (!GEN) RC(RC_SPEC);
        nd = refl;
    } else if (divert == RT_DIVERT_DIELECTRIC) {
        if (!GEN) RC(RC_DIELECTRIC);
        nd = refract_vec(p.ray.d, n, dn, refl, m->over_in, m->over_out, m->r0, &prob, &p.rng);
    } else {
        if (!GEN) RC(RC_DIFF);
        nd = diff_vec(p.ray.d, n, dn, &p.rng);
    }
    if (!GEN && atten && prob != 1.0f) RC(RC_ATTEN_DIV);
    V3 rgb = ld3(m->rgb) * prob;
    // rgb * 1 is rgb, so with p = 1 the attenuated colour is the host's rgb / 0.4
    if (atten) rgb = prob == 1.0f ? ld3(m->rgb_atten) : div3(rgb, RR_THRES);
    p.T = cmul(p.T, rgb);
    p.ray.d = nd;
    p.ray.o = pos;
    // should_dls: diffuse spheres (Diff, or DiffSpec seeded diffuse); triangles never
    if (DLS && kind == K_SPHERE && (divert == RT_DIVERT_DIFF || (divert == RT_DIVERT_DIFFSPEC && seed_diff))) {
        p.dls_on = true;
        p.dls_ref = h.ref;
        p.dls_pos = pos;
        p.dls_n = n;
        p.dls_T = p.T;
    }
    return ++p.depth >= MAX_BOUNCES;
}

template <bool COUNT, bool GEN, bool DLS = false, bool COOP = false, bool RESTART = false>
__device__ __forceinline__ bool segment(const DevScene& sc, Path& p, uint32_t* st,
                                        Ctr<COUNT>& c, bool active = true, const PkScene* ps = nullptr) {
    if (COUNT) c.segments++;
    // The ray's direction arrives un-normalized from camera_ray or shade: one normalize here
    // serves a wave's new paths and continued ones alike (each lane normalizes the same vector
    // the reference does, just later).
    p.ray.d = normalize(p.ray.d);
    Hit h;
    const bool hit = COOP ? closest_coop<RESTART>(sc, p.ray, &h, st, active, !DLS && p.depth == 0, ps)
                          : closest<COUNT, GEN, RESTART>(sc, p.ray, &h, st, c);
    if (COOP && !active) return false;
    return shade<COUNT, GEN, DLS>(sc, p, h, hit, c);
}

// key: the pixel's stream key, rt_rng_pixel_key(sc.seed, pixel) (rt_rng_init's first round)
__device__ __forceinline__ void start_path(const DevScene& sc, Path& p, V3 dir, uint64_t key, uint64_t s) {
    p.rng = rt_rng_init_key(key, s);
    p.ray = camera_ray(sc, dir, &p.rng);
    p.L = mk(0.f, 0.f, 0.f);
    p.T = mk(1.f, 1.f, 1.f);
    p.depth = 0;
    p.dls_on = false;
}

// One lane = one pixel for the launch's whole sample range, with path regeneration: when a
// path ends, the lane folds its radiance into the pixel's running mean and immediately starts
// the pixel's next sample, so a wave is not held back by its longest path of every sample
// (lanes only idle once their own sample budget is spent).  Samples of a pixel are still
// folded in sample order, exactly like draw_scene.rs:81-83.
// GEN = false: the scene holds spheres only (and possibly a cube map); triangle and mesh code
// is compiled out, which keeps the sphere kernel's register budget (walled.yml).
template <bool COUNT, bool GEN, bool DLS = false>
__global__ __launch_bounds__(BLOCK, RT_MIN_WAVES) void trace_kernel(LaunchArgs a) {
    extern __shared__ uint32_t dyn_lds[];  // traversal stack: [stack_depth][BLOCK] branch indices
    const DevScene& sc = a.sc;
    if (!GEN) {  // only the sphere-only kernel reads the LDS sphere tables
        fill_lds_spheres(sc);
        __syncthreads();
    }

    // workgroup -> tile -> block of 16 x (8/K) pixels, K lanes per pixel (adjacent lanes)
    const uint32_t K = a.lanes_per_pixel;
    uint32_t b = blockIdx.x, t = 0;
    while (t + 1 < a.n_tiles && a.tiles[t + 1].block_begin <= b) ++t;
    const DevTile tl = a.tiles[t];
    const uint32_t lb = b - tl.block_begin;
    const uint32_t lp = threadIdx.x / K, kk = threadIdx.x % K;
    const uint32_t lx = (lb % tl.bx) * BLOCK_W + (lp % BLOCK_W);
    const uint32_t ly = (lb / tl.bx) * (BLOCK_H / K) + (lp / BLOCK_W);
    if (lx >= tl.w || ly >= tl.h) return;
    const int x = (int)(tl.x0 + lx), y = (int)(tl.y0 + ly);
    const uint32_t pix = (uint32_t)y * sc.width + (uint32_t)x;
    const uint32_t o = tl.out_off + ly * tl.w + lx;

    uint32_t* st = dyn_lds + threadIdx.x;
    Ctr<COUNT> c;

    // this lane's samples: sample_begin + kk + K*j, j < n_mine
    const uint32_t n_mine = kk < a.sample_count ? (a.sample_count - kk + K - 1) / K : 0;
    V3 acc = mk(0.f, 0.f, 0.f);
    if (K == 1 && a.sample_begin > a.mean_base) acc = xyz(a.accum[pix]);
    uint32_t i = 0;
    Path p;
    const uint64_t pkey = rt_rng_pixel_key(sc.seed, pix);
    const V3 pdir = camera_base_dir(sc, x, y);
    if (n_mine) start_path(sc, p, pdir, pkey, a.sample_begin + kk);
    while (i < n_mine) {
        if (segment<COUNT, GEN, DLS>(sc, p, st, c)) {
            const uint32_t rel = kk + K * i;
            if (K == 1) {
                const float n = (float)(a.sample_begin - a.mean_base + rel);  // running mean, draw_scene.rs:81-83
                acc = mk((p.L.x + (acc.x * n)) / (n + 1.0f), (p.L.y + (acc.y * n)) / (n + 1.0f),
                         (p.L.z + (acc.z * n)) / (n + 1.0f));
            } else if (!COUNT) {
                float* r = a.radiance + 3 * ((size_t)rel * a.n_pix + o);
                r[0] = p.L.x;
                r[1] = p.L.y;
                r[2] = p.L.z;
            }
            if (++i < n_mine) start_path(sc, p, pdir, pkey, a.sample_begin + kk + K * i);
        }
    }
    if (COUNT) {
        atomicAdd(&a.counts->samples, (unsigned long long)n_mine);
        atomicAdd(&a.counts->segments, (unsigned long long)c.segments);
        atomicAdd(&a.counts->nodes, (unsigned long long)c.nodes);
        atomicAdd(&a.counts->leaf_refs, (unsigned long long)c.leaf_refs);
        atomicAdd(&a.counts->sphere_tests, (unsigned long long)c.sph);
        atomicAdd(&a.counts->tri_tests, (unsigned long long)c.tri);
        atomicAdd(&a.counts->hits, (unsigned long long)c.hits);
        atomicAdd(&a.counts->mesh_hits, (unsigned long long)c.mesh_hits);
        return;
    }
    if (K == 1) {
        const float4 ov = make_float4(acc.x, acc.y, acc.z, 1.0f);
        a.accum[pix] = ov;
        if (a.out) a.out[o] = ov;
    }
}

// (item / n_pix, item % n_pix) without a 32-bit division: q = mulhi(item, floor(2^32 / n_pix))
// is floor(item / n_pix) or one less (item < 2^32), and one compare fixes it.
__device__ __forceinline__ void split_item(const LaunchArgs& a, uint32_t item, uint32_t* j, uint32_t* o) {
    if (a.n_pix == 1u) { *j = item; *o = 0u; return; }
    uint32_t q = __umulhi(item, a.n_pix_magic);
    uint32_t r = item - q * a.n_pix;
    if (r >= a.n_pix) { ++q; r -= a.n_pix; }
    *j = q;
    *o = r;
}

// Tile holding launch pixel o (tiles are concatenated in out_off order).
__device__ __forceinline__ uint32_t tile_of(const LaunchArgs& a, uint32_t o) {
    uint32_t lo = 0, hi = a.n_tiles - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (a.tiles[mid].out_off <= o) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
// Frame coordinates of launch pixel o: one coalesced load from the host-built table, or (frames
// over 65535 pixels wide or high) a binary search over the tiles.
__device__ __forceinline__ void launch_pixel(const LaunchArgs& a, uint32_t o, int* x, int* y) {
    if (a.pix_xy) {
        const uint32_t v = a.pix_xy[o];
        *x = (int)(v & 0xffffu);
        *y = (int)(v >> 16);
        return;
    }
    const DevTile tl = a.tiles[tile_of(a, o)];
    const uint32_t lo = o - tl.out_off;
    *x = (int)(tl.x0 + lo % tl.w);
    *y = (int)(tl.y0 + lo / tl.w);
}

// Queue schedule: the grid is sized to the resident lanes, and every lane keeps tracing
// (pixel, sample) items until the launch's items are exhausted, so a wave is never held back
// by its slowest pixel (mesh scenes, where a sky pixel costs a fraction of an airplane pixel).
// A wave claims a run of consecutive items per atomic and hands them to its idle lanes in lane
// order; consecutive items are neighbouring pixels of one sample.  The run length adapts to
// what is left — about remaining / (RT_QDIV * waves), in multiples of 64, from RT_QMIN(_SPH) to RT_QMAX —
// so the single counter is hit rarely while most items remain (a cheap scene otherwise
// saturates it) and balance is fine-grained at the end of the launch.  Each item's radiance goes
// to radiance[j][o]; fold_kernel then applies the running mean in sample order, so the image is
// the direct schedule's, bit for bit.
constexpr int RT_QDIV = 16;
constexpr int RT_QMAX = 1024;
// Smallest grab.  The sphere-only kernel's items are cheap (~6 segments of a brute-force loop), so
// 64-item grabs at the end of a launch put every wave on the one counter about every 7 us and
// the atomics serialise: 256 ran walled +1.6% (A/B, bit-identical).  Mesh items cost 30x more
// and need the fine end-of-launch balance: 128 ran biplane -10%.
constexpr int RT_QMIN = 64;
constexpr int RT_QMIN_SPH = 256;
// A grab must cover every lane of a wave that asks at once (up to 64 items: queue_kernel claims
// at most one grab per refill), and grabs stay multiples of 64.
static_assert(RT_QMIN >= 64 && RT_QMIN % 64 == 0, "RT_QMIN: a multiple of 64, at least 64");
static_assert(RT_QMIN_SPH >= 64 && RT_QMIN_SPH % 64 == 0, "RT_QMIN_SPH: a multiple of 64, at least 64");
static_assert(RT_QMAX >= RT_QMIN && RT_QMAX >= RT_QMIN_SPH && RT_QMAX % 64 == 0 && RT_QMAX <= 1024,
              "RT_QMAX: a multiple of 64 in [RT_QMIN, 1024] (the queue counter's overshoot bound)");
template <bool GEN>
__device__ __forceinline__ uint32_t grab_size(uint32_t remaining, uint32_t n_waves) {
    constexpr uint32_t qmin = GEN ? (uint32_t)RT_QMIN : (uint32_t)RT_QMIN_SPH;
    uint32_t g = remaining / (RT_QDIV * n_waves);
    g &= ~63u;
    return g < qmin ? qmin : (g > (uint32_t)RT_QMAX ? (uint32_t)RT_QMAX : g);
}

// The launch's items in a.n_shards sub-ranges (1..32), each with its own counter (a 128-B line
// of a.queue): every grab is one device-scope atomic, and on one counter they serialise — a
// cheap scene's 64-item grabs (triangles.yml at 10 spp: ~112 K atomics per 1.4 ms launch) waited
// on it for most of the launch.  A wave starts on shard blockIdx % n_shards (blocks are dealt to
// the 8 XCDs round-robin, so with 8 shards each XCD starts on its own) and moves to the next
// shard when its own is exhausted; it is done when it has found every shard exhausted (counters
// only grow).  Shard boundaries are multiples of 64, so a grab (a multiple of 64, at least 64)
// that starts inside a shard covers every lane that asks.  Which lane traces an item changes,
// never what the item computes: bit-identical images.  The runtime (runtime.hip queue_shards)
// gives 8 shards to tiny scenes (their grabs serialise on one counter: triangles.yml 4,937 ->
// 14,120 Msamples/s) and to scenes whose traversal data exceeds one XCD's 4 MiB L2 (each XCD then
// walks its own window of pixels: a380 +4..11% in synchronous launches); the mid-size meshes keep
// one counter, whose waves all work on one window of consecutive items (spaceship_r1 and biplane
// lose 3-8% with shards).
constexpr uint32_t QSHARD_STRIDE = 32;  // uint32 words between shard counters (128 B)
__device__ __forceinline__ uint32_t qshard_begin(const LaunchArgs& a, uint32_t k) {
    if (k == 0) return 0u;
    const uint64_t b = ((uint64_t)a.n_items * k / a.n_shards + 63u) & ~63ull;
    return b < a.n_items ? (uint32_t)b : a.n_items;
}
// One grab of `grab` items for the wave (wave-uniform; `lane_op` is the lane that issues the
// atomic): from shard qk, moving on while shards are exhausted.  Returns [*base, *end) (end the
// shard's end, so the pool is clipped to it); *exhausted when every shard is.
__device__ __forceinline__ void qgrab(const LaunchArgs& a, uint32_t grab, uint32_t lane_op, uint32_t& qk,
                                      uint32_t& q_seen, bool& exhausted, uint32_t* base, uint32_t* end) {
    const uint32_t lane = __lane_id();
    for (;;) {
        const uint32_t b = qshard_begin(a, qk), e = qshard_begin(a, qk + 1);
        uint32_t b0 = 0;
        if (lane == lane_op) b0 = atomicAdd(a.queue + qk * QSHARD_STRIDE, grab);
        const uint32_t off = __builtin_amdgcn_readfirstlane(__shfl(b0, lane_op));
        if (off < e - b) {
            *base = b + off;
            *end = e;
            return;
        }
        if (++q_seen >= a.n_shards) {  // every shard exhausted: no items
            exhausted = true;
            *base = *end = a.n_items;
            return;
        }
        qk = qk + 1 == a.n_shards ? 0u : qk + 1;
    }
}

// Path starts in batches (RT_START_BATCH, the sphere-only kernel, cameras without a lens).  A
// start is the item's pixel, the stream key, the SplitMix64 round and camera_ray's two jitter
// draws.  Made by the idle lanes alone, it ran at the width of the lanes that had just finished,
// so the wave waited for a dozen of them (RT_REGEN_MIN) while they idled through segments.
// Instead the wave makes the camera rays of its next 64 items together, one per lane, and keeps
// them in LDS (24 B: the unnormalized direction, the stream state after the draws, the radiance
// slot); idle lanes take the next ones in order, at every segment.  A start is a pure function of
// its item, so each item's path is the one start_path makes, bit for bit; only the lane that
// traces it changes.  (A lens adds the origin to an entry: measured −0.7% from the extra
// registers on walled, so lens scenes keep the per-lane starts.)
constexpr uint32_t START_NONE = 0xffffffffu;  // slot of an entry past the launch's items
constexpr int START_FIELDS = 6;
__shared__ uint32_t g_start[BLOCK / 64][START_FIELDS][64];

__device__ __forceinline__ void make_start(const LaunchArgs& a, const DevScene& sc, uint32_t item, uint32_t lane,
                                           uint32_t (*e)[64]) {
    uint32_t slot = START_NONE;
    V3 d = mk(0.f, 0.f, 0.f);
    rt_rng_state rng = 0;
    if (item < a.n_items) {
        uint32_t j, o;
        split_item(a, item, &j, &o);
        const uint4 q = a.pix_q[o];  // item j * n_pix + q: the q-th pixel in queue order
        const int x = (int)(q.x & 0xffffu), y = (int)(q.x >> 16);
        const uint64_t key = RT_PIX_KEY ? ((uint64_t)q.w << 32) | q.z
                                        : rt_rng_pixel_key(sc.seed, (uint32_t)y * sc.width + (uint32_t)x);
        rng = rt_rng_init_key(key, a.sample_begin + j);
        d = camera_ray(sc, camera_base_dir(sc, x, y), &rng).d;  // no lens: the origin is cam_o
        slot = j * a.n_pix + q.y;
    }
    e[0][lane] = __float_as_uint(d.x);
    e[1][lane] = __float_as_uint(d.y);
    e[2][lane] = __float_as_uint(d.z);
    e[3][lane] = (uint32_t)rng;
    e[4][lane] = (uint32_t)(rng >> 32);
    e[5][lane] = slot;
}

// STARTS (sphere-only kernel): paths start per lane (a lens camera, or no pixel table), not in the
// LDS batches.  A template parameter rather than a runtime flag: with both start paths in one
// loop, their merged Path state cost walled ~15 register copies per segment (+0.7% without).
template <bool GEN, bool DLS, bool RESTART, bool STARTS = false>
__global__ __launch_bounds__(BLOCK, GEN ? RT_MIN_WAVES_GEN : RT_MIN_WAVES) void queue_kernel(
    LaunchArgs a, const uint2* __restrict__ pk_nodes, const uint32_t* __restrict__ pk_refs,
    const float4* __restrict__ pk_prim4) {
    constexpr uint32_t TPB = (uint32_t)BLOCK;  // threads per workgroup
    extern __shared__ uint32_t dyn_lds[];
    const DevScene& sc = a.sc;
    TM_VAR(const unsigned long long tm_start = TM_NOW());
    if (!GEN) {  // only the sphere-only kernel reads the LDS sphere tables
        fill_lds_spheres(sc);
        __syncthreads();
    }
    uint32_t* st = GEN ? dyn_lds + threadIdx.x
                       : a.gstack + (size_t)blockIdx.x * BLOCK * sc.stack_depth + threadIdx.x;
    Ctr<false> c;
    const uint32_t lane = __lane_id();
    uint32_t pool = 0, pool_end = 0;  // wave-uniform: unclaimed items [pool, pool_end)
    const uint32_t n_waves = gridDim.x * (TPB / 64);
    constexpr bool batch_ok = !GEN && !STARTS;  // the host launches it so: no lens, a pixel table
    const uint32_t shard_waves = (n_waves + a.n_shards - 1) / a.n_shards;
    // (the batch starts use one counter over all the items: the first grab is sized for that)
    uint32_t grab = batch_ok ? grab_size<GEN>(a.n_items, n_waves) : grab_size<GEN>(a.n_items / a.n_shards, shard_waves);
    uint32_t qk = blockIdx.x % a.n_shards, q_seen = 0;  // wave-uniform: its shard, shards found exhausted
    bool q_out = false;                                 // wave-uniform: every shard exhausted
    bool have = false, done = false;
    uint32_t slot = 0;                // radiance index of the lane's item
    Path p;
    // RT_START_BATCH: the wave's current batch of starts, entries [st_pos, 64) not yet taken
    uint32_t st_pos = 64u, st_n = 0u;
    for (;;) {
        const uint64_t need = __ballot(!have && !done);
        // Starting paths is wave-wide work at the width of the idle lanes: ~10 of 64 lanes end a
        // path per segment, so without batched starts the wave waits for RT_REGEN_MIN of them.
        constexpr int regen_min = GEN ? RT_REGEN_MIN_GEN : (RT_START_BATCH ? RT_REGEN_MIN_BATCH : RT_REGEN_MIN);
        const bool regen = need && (regen_min <= 1 || __popcll(need) >= regen_min || __ballot(have) == 0);
        if (!GEN && RT_START_BATCH && regen && batch_ok) {
            RC(RC_REGEN);
            // the n idle lanes take entries st_pos .. st_pos + n - 1 of the batch, making the
            // next batch (the wave's next 64 items) when it runs out
            const uint32_t n = (uint32_t)__popcll(need);
            const bool idle = !have && !done;
            const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
            uint32_t (*e)[64] = g_start[threadIdx.x >> 6];
            uint32_t v[START_FIELDS] = {0u, 0u, 0u, 0u, 0u, START_NONE};
            auto take = [&](uint32_t ei) {
#pragma unroll
                for (int f = 0; f < START_FIELDS; ++f) v[f] = e[f][ei];
            };
            if (idle && r < st_n) take(st_pos + r);  // before the next batch overwrites them
            if (n > st_n) {
                RC(RC_BATCH);
                // One counter (a.queue[0] over all the items, whatever a.n_shards): the sphere-only
                // kernel's grabs are 256+ items (RT_QMIN_SPH), and the shard walk of qgrab cost
                // walled 1.7% here.
                if (pool == pool_end) {  // grabs are multiples of 64: a batch never spans two
                    uint32_t b0 = 0;
                    if (lane == 0) b0 = atomicAdd(a.queue, grab);
                    pool = __builtin_amdgcn_readfirstlane(b0);
                    pool_end = pool + grab;
                    grab = grab_size<GEN>(a.n_items > pool_end ? a.n_items - pool_end : 0u, n_waves);
                }
                __builtin_amdgcn_wave_barrier();
                make_start(a, sc, pool + lane, lane, e);
                pool += 64u;
                __builtin_amdgcn_wave_barrier();
                if (idle && r >= st_n) take(r - st_n);
                st_pos = n - st_n;
                st_n = 64u - st_pos;
            } else {
                st_pos += n;
                st_n -= n;
            }
            if (idle) {
                if (v[5] == START_NONE) {  // past the launch's items
                    done = true;
                } else {
                    p.ray.o = ld3(sc.cam_o);
                    p.ray.d = mk(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]));
                    p.rng = ((uint64_t)v[4] << 32) | v[3];
                    p.L = mk(0.f, 0.f, 0.f);
                    p.T = mk(1.f, 1.f, 1.f);
                    p.depth = 0;
                    p.dls_on = false;
                    slot = v[5];
                    have = true;
                }
            }
        } else if (regen) {
            const uint32_t n = (uint32_t)__popcll(need);
            const uint32_t left = pool_end - pool;
            // fresh items [base, e): the general kernel's sharded counters (none once q_out);
            // the sphere-only kernel keeps one counter (its lens cameras start here)
            uint32_t base = a.n_items, e = a.n_items;
            if (left < n && (!GEN || !q_out)) {
                const uint32_t first = (uint32_t)__ffsll((unsigned long long)need) - 1u;
                if constexpr (GEN) {
                    qgrab(a, grab, first, qk, q_seen, q_out, &base, &e);
                } else {
                    uint32_t b0 = 0;
                    if (lane == first) b0 = atomicAdd(a.queue, grab);
                    base = __builtin_amdgcn_readfirstlane(__shfl(b0, first));
                }
            }
            if (!have && !done) {
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const uint32_t item = r < left ? pool + r : base + (r - left);
                if (GEN ? item < (r < left ? pool_end : e) : item < a.n_items) {
                    uint32_t j, o;
                    split_item(a, item, &j, &o);
                    int x, y;
                    uint64_t key;
                    V3 dir;
                    if (GEN) { VC(6, 1); VC(14, 1); }
                    if (a.pix_q) {  // item j * n_pix + q: the q-th pixel in queue order
                        if (GEN) VL(6, a.pix_q + o, 16, true);
                        const uint4 e = a.pix_q[o];
                        x = (int)(e.x & 0xffffu);
                        y = (int)(e.x >> 16);
                        o = e.y;
                        key = RT_PIX_KEY ? ((uint64_t)e.w << 32) | e.z
                                         : rt_rng_pixel_key(sc.seed, (uint32_t)y * sc.width + (uint32_t)x);
                        dir = camera_base_dir(sc, x, y);
                    } else {
                        launch_pixel(a, o, &x, &y);
                        key = rt_rng_pixel_key(sc.seed, (uint32_t)y * sc.width + (uint32_t)x);
                        dir = camera_base_dir(sc, x, y);
                    }
                    start_path(sc, p, dir, key, a.sample_begin + j);
                    slot = j * a.n_pix + o;
                    have = true;
                } else {
                    done = !GEN || q_out;  // else the last shard ended short of this lane: next regen
                }
            }
            if (left < n) {
                if constexpr (GEN) {
                    // a successful grab starts inside its shard, whose end is a multiple of 64
                    // beyond it: it covers the n - left <= 64 lanes that asked
                    pool = base + (n - left) < e ? base + (n - left) : e;
                    pool_end = base + grab < e ? base + grab : e;
                    grab = grab_size<GEN>(e - pool_end, shard_waves);
                } else {
                    pool = base + (n - left);
                    pool_end = base + grab;
                    grab = grab_size<GEN>(a.n_items > pool_end ? a.n_items - pool_end : 0u, n_waves);
                }
            } else {
                pool += n;
            }
        }
        if (__ballot(have) == 0) {
            TM_ADD(2, TM_NOW() - tm_start);
            DIAG_WAVE_EXIT(GEN);
            break;
        }
        if (!GEN) {
            RC(RC_ITER);
            if (have) RC_LANES(RC_ITER_LANES);
        }
        // the cooperative traversal needs every lane of the wave: lanes without a path help
        const PkScene ps{pk_nodes, pk_refs, pk_prim4};
        const bool fin = GEN ? segment<false, GEN, DLS, GEN, RESTART>(sc, p, st, c, have, &ps) && have
                             : have && segment<false, GEN, DLS, false, RESTART>(sc, p, st, c);
        if (fin) {
            if (GEN) VC(13, 1);
            if (!GEN) RC(RC_STORE);
            float* r = a.radiance + 3 * (size_t)slot;
            r[0] = p.L.x;
            r[1] = p.L.y;
            r[2] = p.L.z;
            have = false;
        }
    }
}

// Running mean over the traced chunk, in sample order (draw_scene.rs:81-83): one lane per
// launch pixel; reads are coalesced across lanes ([sample][pixel] layout).
__global__ __launch_bounds__(256) void fold_kernel(LaunchArgs a) {
    const uint32_t o = blockIdx.x * 256 + threadIdx.x;
    if (o >= a.n_pix) return;
    int x, y;
    launch_pixel(a, o, &x, &y);
    const uint32_t pix = (uint32_t)y * a.sc.width + (uint32_t)x;
    V3 acc = mk(0.f, 0.f, 0.f);
    const uint64_t n0 = a.sample_begin - a.mean_base;  // the running mean's n of the first sample
    if (n0 > 0) acc = xyz(a.accum[pix]);
    // (r + acc n) / (n + 1) per channel, in sample order; div3 is the division bit for bit
    // (exact reciprocal + Markstein quotients under their range guard).  The samples' loads are
    // issued FOLD_U at a time ahead of the sequential fold: with few launch pixels (a rank's
    // share at N = 8: 90K threads) one load in flight per thread left the fold latency-bound.
constexpr int RT_FOLD_U = 8;
    constexpr uint32_t FOLD_U = RT_FOLD_U;
    uint32_t j = 0;
    for (; j + FOLD_U <= a.sample_count; j += FOLD_U) {
        float v[3 * FOLD_U];
#pragma unroll
        for (uint32_t u = 0; u < FOLD_U; ++u) {
            const float* r = a.radiance + 3 * ((size_t)(j + u) * a.n_pix + o);
            v[3 * u] = r[0];
            v[3 * u + 1] = r[1];
            v[3 * u + 2] = r[2];
        }
#pragma unroll
        for (uint32_t u = 0; u < FOLD_U; ++u) {
            const float n = (float)(n0 + j + u);
            acc = div3(mk(v[3 * u] + (acc.x * n), v[3 * u + 1] + (acc.y * n), v[3 * u + 2] + (acc.z * n)), n + 1.0f);
        }
    }
    for (; j < a.sample_count; ++j) {
        const float* r = a.radiance + 3 * ((size_t)j * a.n_pix + o);
        const float n = (float)(n0 + j);
        acc = div3(mk(r[0] + (acc.x * n), r[1] + (acc.y * n), r[2] + (acc.z * n)), n + 1.0f);
    }
    const float4 ov = make_float4(acc.x, acc.y, acc.z, 1.0f);
    a.accum[pix] = ov;
    if (a.out) a.out[o] = ov;
}


hipError_t launch_fold(const LaunchArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(fold_kernel, dim3((a.n_pix + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

static size_t stack_lds_bytes(const LaunchArgs& a) {
    return (size_t)a.sc.stack_depth * BLOCK * sizeof(uint32_t);
}

hipError_t launch_trace(const LaunchArgs& a, hipStream_t s) {
    if (a.sc.dls)
        hipLaunchKernelGGL((trace_kernel<false, true, true>), dim3(a.n_blocks), dim3(BLOCK), stack_lds_bytes(a), s, a);
    else if (a.sc.spheres_only)
        hipLaunchKernelGGL((trace_kernel<false, false>), dim3(a.n_blocks), dim3(BLOCK), stack_lds_bytes(a), s, a);
    else
        hipLaunchKernelGGL((trace_kernel<false, true>), dim3(a.n_blocks), dim3(BLOCK), stack_lds_bytes(a), s, a);
    return hipGetLastError();
}

// The queue kernel of a launch: sphere-only or general, with direct-light sampling, stackless or
// with a traversal stack (DevScene::restart).  The stack is in LDS for the general kernels and in
// global memory for the sphere-only one (queue_gstack_bytes); the stackless kernels need neither.
template <class F>
static hipError_t with_queue_kernel(const LaunchArgs& a, F f) {
    const bool rs = a.sc.restart != 0;
    if (a.sc.spheres_only) {
        if (a.sc.has_lens || a.pix_q == nullptr)  // per-lane path starts
            return rs ? f(queue_kernel<false, false, true, true>, false) : f(queue_kernel<false, false, false, true>, false);
        return rs ? f(queue_kernel<false, false, true>, false) : f(queue_kernel<false, false, false>, false);
    }
    if (a.sc.dls) return rs ? f(queue_kernel<true, true, true>, true) : f(queue_kernel<true, true, false>, true);
    return rs ? f(queue_kernel<true, false, true>, true) : f(queue_kernel<true, false, false>, true);
}
static size_t queue_lds_bytes(const LaunchArgs& a, bool gen) { return (gen && !a.sc.restart) ? stack_lds_bytes(a) : 0; }
uint32_t queue_block_threads(const LaunchArgs&) { return (uint32_t)BLOCK; }

// Resident workgroups per CU of the queue kernel this scene launches (its registers and LDS
// stack decide): the queue grid is exactly that many workgroups per CU.
hipError_t queue_blocks_per_cu(const LaunchArgs& a, int* blocks) {
    return with_queue_kernel(a, [&](auto k, bool gen) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, k, (int)queue_block_threads(a),
                                                            queue_lds_bytes(a, gen));
    });
}

size_t queue_gstack_bytes(const LaunchArgs& a, uint32_t n_blocks) {
    if (!a.sc.spheres_only || a.sc.dls || a.sc.restart) return 0;
    return (size_t)n_blocks * BLOCK * a.sc.stack_depth * sizeof(uint32_t);
}

hipError_t launch_trace_queue(const LaunchArgs& a, uint32_t n_blocks, hipStream_t s) {
    return with_queue_kernel(a, [&](auto k, bool gen) {
        hipLaunchKernelGGL(k, dim3(n_blocks), dim3(queue_block_threads(a)), queue_lds_bytes(a, gen), s, a, a.sc.nodes,
                           a.sc.refs, a.sc.prim4);
        return hipGetLastError();
    });
}
hipError_t launch_trace_count(const LaunchArgs& a, hipStream_t s) {
    if (a.sc.dls)
        hipLaunchKernelGGL((trace_kernel<true, true, true>), dim3(a.n_blocks), dim3(BLOCK), stack_lds_bytes(a), s, a);
    else if (a.sc.spheres_only)
        hipLaunchKernelGGL((trace_kernel<true, false>), dim3(a.n_blocks), dim3(BLOCK), stack_lds_bytes(a), s, a);
    else
        hipLaunchKernelGGL((trace_kernel<true, true>), dim3(a.n_blocks), dim3(BLOCK), stack_lds_bytes(a), s, a);
    return hipGetLastError();
}

}  // namespace rtd
