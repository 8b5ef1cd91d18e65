// oracle.cpp — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference CPU render path.
//
// Each function names the reference file:line it restates (joonhosung/GPU-Ray_Trace-Rust,
// snapshot 2024-12-18).  The structure deliberately mirrors the reference — trait-object
// elements, a pointer KD tree with an explicit std::vector stack, recursive radiance — so a
// reader can check it line by line; speed is secondary (it is also the "port" CPU baseline).
//
// Float conventions (parity unpinned beyond the reference's own tests):
// compiled with -ffp-contract=off; nalgebra dot = (a0b0 + a1b1) + a2b2, normalize divides
// each component by sqrt(dot), f32::min/max return the non-NaN operand (fminf/fmaxf),
// sin/cos/powf are the C library's (what Rust's f32 methods call on Linux), and
// `powf(x, 2.0)` is x*x (LLVM folds it so in the reference build).
#include "oracle.h"
#include "../include/rt_rng.h"

#include <atomic>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace orc {

static const float EPS = 1e-4f;  // src/lib.rs:20
static const float PI = 3.14159265358979323846f;

// ------------------------------------------------------------------ vector math (nalgebra)
struct V3 {
    float x, y, z;
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
static inline V3 mk(float x, float y, float z) { return V3{x, y, z}; }
static inline V3 mk(const float* p) { return V3{p[0], p[1], p[2]}; }
static inline V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 operator-(V3 a) { return mk(-a.x, -a.y, -a.z); }
static inline V3 operator*(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline V3 operator*(float s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
static inline V3 operator/(V3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline V3 cmul(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline float norm(V3 a) { return std::sqrt(dot(a, a)); }
static inline V3 normalize(V3 a) { return a / norm(a); }
static inline V3 cross(V3 a, V3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// Rust f32::min / f32::max: NaN-ignoring, like fminf/fmaxf.
static inline float rmin(float a, float b) { return std::fmin(a, b); }
static inline float rmax(float a, float b) { return std::fmax(a, b); }

struct M3 {  // row-major 3x3
    float m[3][3];
    V3 col(int j) const { return mk(m[0][j], m[1][j], m[2][j]); }
    void set_col(int j, V3 v) { m[0][j] = v.x; m[1][j] = v.y; m[2][j] = v.z; }
};
// nalgebra gemv: res_i = ((A_i0 x0) + A_i1 x1) + A_i2 x2.
static inline V3 mul(const M3& a, V3 v) {
    return mk((a.m[0][0] * v.x + a.m[0][1] * v.y) + a.m[0][2] * v.z,
              (a.m[1][0] * v.x + a.m[1][1] * v.y) + a.m[1][2] * v.z,
              (a.m[2][0] * v.x + a.m[2][1] * v.y) + a.m[2][2] * v.z);
}
static inline M3 mul(const M3& a, const M3& b) {
    M3 c;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            c.m[i][j] = (a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j]) + a.m[i][2] * b.m[2][j];
    return c;
}

// ------------------------------------------------------------------ RNG (src/lib.rs:22-27)
// The reference's thread_rng() is replaced by the rt_rng.h stream of the current
// (pixel, sample); every `crate::RNG.with_borrow_mut(|r| r.gen())` is one rng_f32().
static thread_local rt_rng_state g_rng;
// Shading-mix instrumentation (counted renders only, tools/min_insts.py): per continued ray by
// branch, the draws, and the Russian-roulette draws.
// MIX_NODE_D0 + d: branch nodes the traversal steps through at depth d (root = 0), the
// counted renders' descent profile (how much of a descent a top-of-tree node cache could hold)
enum { MIX_SPEC, MIX_DIFF, MIX_DIFFSPEC_DIFF, MIX_DIFFSPEC_SPEC, MIX_DIELECTRIC, MIX_RR, MIX_DRAWS, MIX_MESH,
       MIX_POSDISC, MIX_NODE_D0, MIX_N = MIX_NODE_D0 + ORACLE_MIX_DEPTHS };
static_assert(MIX_N == ORACLE_MIX_N, "oracle.h ORACLE_MIX_N");
static thread_local uint64_t* g_mix = nullptr;
#define MIX(i) do { if (g_mix) g_mix[i]++; } while (0)
static std::mutex g_mix_mu;
static uint64_t g_mix_total[MIX_N];
static inline float rng_f32() { MIX(MIX_DRAWS); return rt_rng_next_f32(&g_rng); }

// ------------------------------------------------------------------ instrumentation
static thread_local oracle_counts* g_cnt = nullptr;
#define COUNT(field, n) do { if (g_cnt) g_cnt->field += (n); } while (0)

// ------------------------------------------------------------------ ray (src/ray/mod.rs:11-15)
struct Ray { V3 d, o; };

// RayLen total order (src/ray/hit.rs:50-76): NaN == NaN, NaN greater than everything.
static inline int raylen_cmp(float a, float b) {
    bool an = std::isnan(a), bn = std::isnan(b);
    if (!an && !bn) return a < b ? -1 : (a > b ? 1 : 0);
    if (an && bn) return 0;
    return an ? 1 : -1;
}

// HitResult (hit.rs:7-10) with the element-specific `intermed` unboxed.
struct HitResult {
    float l;
    V3 pos;          // sphere: perfect hit position (sphere.rs:97)
    float bu, bv;    // triangle: barycentric (generic.rs:132)
};

// Seeding variants: SeedingRay (uniform_diff_spec.rs:21-24) and the mesh (bool, f32)
// (mesh/triangle.rs:187).
struct Seeding {
    bool diffspec = false;  // SeedingRay::DiffSpec(_) vs NoSeed
    bool diff = false;
    float rough = 0.f;
};

// HitInfo (hit.rs:12-18) with continue_info unboxed.
struct HitInfo {
    V3 emissive, pos, norm;
    bool dls;
    bool has_continue;
    Seeding seed;
    float bu, bv;
};

// ------------------------------------------------------------------ Aabb (src/accel/aabb.rs)
struct Aabb { float lo[3], hi[3]; };

static inline V3 centroid(const Aabb& b) {  // aabb.rs:19-21
    return mk(0.5f * (b.lo[0] + b.hi[0]), 0.5f * (b.lo[1] + b.hi[1]), 0.5f * (b.lo[2] + b.hi[2]));
}

// aabb.rs:22-62
static bool get_entry_exit(const Aabb& b, const Ray& ray, int* min_a, float* min_d, int* max_a,
                           float* max_d) {
    float lo_t[3], hi_t[3];
    for (int a = 0; a < 3; ++a) {
        float d = ray.d[a];
        if (std::fabs(d) < EPS) d = d < 0.0f ? -EPS : EPS;
        float f = 1.0f / d;
        lo_t[a] = (b.lo[a] - ray.o[a]) * f;
        hi_t[a] = (b.hi[a] - ray.o[a]) * f;
    }
    int ap = 0;
    float vp = rmin(lo_t[0], hi_t[0]);
    for (int a = 1; a < 3; ++a) {
        float v = rmin(lo_t[a], hi_t[a]);
        if (vp < v) { ap = a; vp = v; }
    }
    int bp = 0;
    float wp = rmax(lo_t[0], hi_t[0]);
    for (int a = 1; a < 3; ++a) {
        float w = rmax(lo_t[a], hi_t[a]);
        if (wp > w) { bp = a; wp = w; }
    }
    if (wp < 0.0f || vp > wp) return false;
    *min_a = ap; *min_d = vp; *max_a = bp; *max_d = wp;
    return true;
}

// ------------------------------------------------------------------ textures (uv_image.rs:9-23)
struct Image {
    const rt_texture* t = nullptr;
    V3 get_pixel(float u, float v) const {
        float width = (float)t->width, height = (float)t->height;
        float fx = rmin(rmax(u * width, 0.0f), width - 1.0f);
        float fy = rmin(rmax(v * height, 0.0f), height - 1.0f);
        // `(..).trunc() as u32`: saturating, NaN -> 0
        uint32_t x = std::isnan(fx) ? 0u : (uint32_t)std::trunc(fx);
        uint32_t y = std::isnan(fy) ? 0u : (uint32_t)std::trunc(fy);
        const float* p = t->rgb + 3 * ((size_t)y * t->width + x);
        return mk(p[0], p[1], p[2]);
    }
};

// ------------------------------------------------------------------ materials
// interaction.rs:6-9
static Ray spec(const Ray& ray, V3 n, V3 o) {
    V3 d = normalize(ray.d - (n * 2.0f) * dot(ray.d, n));
    return Ray{d, o};
}
// interaction.rs:11-27
static Ray diff(const Ray& ray, V3 n, V3 o) {
    V3 xd = normalize(ray.d - n * dot(ray.d, n));
    V3 yd = normalize(cross(n, xd));
    float u = rng_f32();
    float v = rng_f32();
    float r = std::sqrt(u);
    float thet = 2.0f * PI * v;
    float x = r * std::cos(thet);
    float y = r * std::sin(thet);
    V3 d = normalize((xd * x + yd * y) + n * std::sqrt(rmax(1.0f - u, 0.0f)));
    return Ray{d, o};
}
// interaction.rs:29-59; `draw` supplies the one uniform consumed after the TIR test.
template <class Draw>
static Ray refract(const Ray& ray, V3 n, V3 o, float n_out, float n_in, float* p, Draw draw) {
    float c_ = dot(n, ray.d);
    bool into = c_ < 0.0f;
    float n1, n2, c1;
    V3 norm_refr;
    if (into) { n1 = n_out; n2 = n_in; c1 = -c_; norm_refr = n; }
    else      { n1 = n_in; n2 = n_out; c1 = c_; norm_refr = -n; }
    float n_over = n1 / n2;
    float c22 = 1.0f - n_over * n_over * (1.0f - c1 * c1);
    bool total_internal = c22 < 0.0f;
    Ray refl = spec(ray, norm_refr, o);
    if (total_internal) { *p = 1.0f; return refl; }
    V3 trns = n_over * ray.d + norm_refr * (n_over * c1 - std::sqrt(c22));
    float q = (n1 - n2) / (n1 + n2);
    float r0 = q * q;  // .powf(2.0) — folded to a multiply by LLVM
    float c = 1.0f - (into ? c1 : dot(trns, n));
    float re = r0 + (1.0f + r0) * std::pow(c, 5.0f);  // (sic) 1 + r0, interaction.rs:50
    float u = draw();
    if (u < re) { *p = re; return refl; }
    *p = 1.0f - re;
    return Ray{normalize(trns), o};
}

// UniformDiffuseSpec (uniform_diff_spec.rs:26-68)
static Seeding generate_seed(const rt_material& m) {
    Seeding s;
    if (m.divert == RT_DIVERT_DIFFSPEC) {
        float u = rng_f32();
        s.diffspec = true;
        s.diff = u < m.diffp;
    }
    return s;
}
static bool should_dls(const rt_material& m, const Seeding& s) {
    return m.divert == RT_DIVERT_DIFF || (m.divert == RT_DIVERT_DIFFSPEC && s.diffspec && s.diff);
}
static Ray gen_new_ray(const rt_material& m, const Ray& ray, V3 n, V3 o, const Seeding& s,
                       float* p) {
    switch (m.divert) {
        case RT_DIVERT_SPEC: MIX(MIX_SPEC); *p = 1.0f; return spec(ray, n, o);
        case RT_DIVERT_DIFF: MIX(MIX_DIFF); *p = 1.0f; return diff(ray, n, o);
        case RT_DIVERT_DIFFSPEC:
            MIX(s.diff ? MIX_DIFFSPEC_DIFF : MIX_DIFFSPEC_SPEC);
            *p = 1.0f;
            return s.diff ? diff(ray, n, o) : spec(ray, n, o);
        default:
            MIX(MIX_DIELECTRIC);
            return refract(ray, n, o, m.n_out, m.n_in, p, [] { return rng_f32(); });
    }
}

// ------------------------------------------------------------------ elements
// Hitable + HasHitInfo + InteractsWithRay (hit.rs:20-32) as one abstract class.
struct Element {
    virtual ~Element() {}
    virtual bool intersect(const Ray& ray, HitResult* hr) const = 0;
    virtual bool give_aabb(Aabb* out) const = 0;
    virtual HitInfo hit_info(const HitResult& hr, const Ray& ray) const = 0;
    virtual bool continue_ray(const Ray& ray, const HitInfo& hi, V3* rgb, Ray* out) const = 0;
    virtual bool dls_emitter(V3 pos, V3* dir) const { (void)pos; (void)dir; return false; }
    virtual bool is_mesh() const { return false; }
};

// Sphere (src/elements/sphere.rs)
struct Sphere final : Element {
    const rt_sphere* s;
    explicit Sphere(const rt_sphere* s_) : s(s_) {}
    bool intersect(const Ray& ray, HitResult* hr) const override {  // :83-105
        COUNT(sphere_tests, 1);
        V3 c = mk(s->c);
        V3 oc = ray.o - c;
        float dir = dot(ray.d, oc);
        float consts = dot(oc, oc) - s->r * s->r;
        float thing2 = dir * dir - consts;
        if (!(thing2 > 0.0f)) return false;
        float offset = -dir;
        float thing = std::sqrt(thing2);
        float ls[2] = {offset + thing, offset - thing};
        bool have = false;
        float f = 0.f;
        for (float e : ls) {
            if (e > 0.0f) { f = have ? rmin(f, e) : e; have = true; }
        }
        if (!have) return false;
        hr->l = f;
        hr->pos = ray.o + ray.d * f;
        return true;
    }
    // tools/min_insts.py's event count: whether this ray's line meets the sphere (thing2 > 0,
    // the same f32 steps as intersect), i.e. whether a brute-force closest hit needs its roots
    bool disc_positive(const Ray& ray) const {
        V3 oc = ray.o - mk(s->c);
        float dir = dot(ray.d, oc);
        float consts = dot(oc, oc) - s->r * s->r;
        return dir * dir - consts > 0.0f;
    }
    bool give_aabb(Aabb* b) const override {  // :106-114
        for (int a = 0; a < 3; ++a) { b->lo[a] = s->c[a] - s->r; b->hi[a] = s->c[a] + s->r; }
        return true;
    }
    HitInfo hit_info(const HitResult& hr, const Ray&) const override {  // :64-80
        HitInfo hi{};
        V3 n = normalize(hr.pos - mk(s->c));
        hi.pos = hr.pos + n * EPS;
        hi.norm = n;
        hi.emissive = s->mat.has_emissive ? mk(s->mat.emissive) : mk(0.f, 0.f, 0.f);
        hi.seed = generate_seed(s->mat);
        hi.dls = should_dls(s->mat, hi.seed);
        hi.has_continue = true;
        return hi;
    }
    bool continue_ray(const Ray& ray, const HitInfo& hi, V3* rgb, Ray* out) const override {
        float p;  // :34-46
        *out = gen_new_ray(s->mat, ray, hi.norm, hi.pos, hi.seed, &p);
        *rgb = mk(s->rgb) * p;
        return true;
    }
    bool dls_emitter(V3 pos, V3* dir) const override {  // :47-62
        if (!s->mat.has_emissive) return false;
        *dir = normalize(mk(s->c) - pos);
        return true;
    }
};

// Generic Möller–Trumbore (src/elements/triangle/generic.rs:102-156).
static bool mt_intersect(V3 v0, V3 v1, V3 v2, const Ray& ray, HitResult* hr) {
    COUNT(tri_tests, 1);
    V3 e1 = v1 - v0;
    V3 e2 = v2 - v0;
    V3 ray_x_e2 = cross(ray.d, e2);
    float det = dot(e1, ray_x_e2);
    if (std::fabs(det) < EPS) return false;
    float inv_det = 1.0f / det;
    V3 rhs = ray.o - v0;
    float u = inv_det * dot(rhs, ray_x_e2);
    if (u < 0.0f || u > 1.0f) return false;
    V3 rhs_x_e1 = cross(rhs, e1);
    float v = inv_det * dot(ray.d, rhs_x_e1);
    if (v < 0.0f || (u + v) > 1.0f) return false;
    float l = inv_det * dot(e2, rhs_x_e1);
    if (l < EPS) return false;
    hr->l = l;
    hr->bu = u;
    hr->bv = v;
    return true;
}
static void tri_aabb(V3 v0, V3 v1, V3 v2, Aabb* b) {  // generic.rs:138-156
    for (int a = 0; a < 3; ++a) {
        b->lo[a] = rmin(rmin(v0[a], v1[a]), v2[a]);
        b->hi[a] = rmax(rmax(v0[a], v1[a]), v2[a]);
    }
}

// FreeTriangle (triangle/free.rs + generic.rs:59-92)
struct FreeTri final : Element {
    const rt_free_triangle* t;
    explicit FreeTri(const rt_free_triangle* t_) : t(t_) {}
    V3 vert(int i) const { return mk(t->verts[i]); }
    bool intersect(const Ray& ray, HitResult* hr) const override {
        return mt_intersect(vert(0), vert(1), vert(2), ray, hr);
    }
    bool give_aabb(Aabb* b) const override { tri_aabb(vert(0), vert(1), vert(2), b); return true; }
    HitInfo hit_info(const HitResult& hr, const Ray& ray) const override {  // generic.rs:78-92
        HitInfo hi{};
        V3 n = mk(t->norm);  // UniformNorm::get_norm
        hi.seed = generate_seed(t->mat);  // divert_ray_seed (free.rs:22-24)
        hi.bu = hr.bu; hi.bv = hr.bv;
        hi.pos = (ray.d * hr.l + ray.o) + n * EPS;
        hi.norm = n;
        hi.emissive = mk(0.f, 0.f, 0.f);  // triangles never emit (generic.rs:86)
        hi.dls = false;
        hi.has_continue = true;
        return hi;
    }
    bool continue_ray(const Ray& ray, const HitInfo& hi, V3* rgb, Ray* out) const override {
        float p;  // generic.rs:59-67
        *out = gen_new_ray(t->mat, ray, hi.norm, hi.pos, hi.seed, &p);
        *rgb = mk(t->rgb) * p;
        return true;
    }
};

// DistantCubeMap (src/elements/distant_cube_map.rs)
struct CubeMap final : Element {
    const rt_cube_map* m;
    Image face[6];
    CubeMap(const rt_cube_map* m_, const rt_scene_desc* sc) : m(m_) {
        for (int f = 0; f < 6; ++f) face[f].t = &sc->textures[m->face[f].texture];
    }
    bool intersect(const Ray&, HitResult* hr) const override {  // :72-74
        hr->l = INFINITY;
        return true;
    }
    bool give_aabb(Aabb*) const override { return false; }
    V3 sample_face(float u, float v, float fact, int f) const {  // :62-69
        float us = m->face[f].us, vs = m->face[f].vs;
        float u1 = u * us / fact, v1 = v * vs / fact;
        return face[f].get_pixel(0.5f * u1 + 0.5f, 0.5f * v1 + 0.5f);
    }
    HitInfo hit_info(const HitResult&, const Ray& ray) const override {  // :27-59
        int max_idx = 0;
        float max_c = ray.d.x;
        for (int i = 1; i < 3; ++i) {
            float c = ray.d[i];
            if (std::fabs(c) > std::fabs(max_c)) { max_idx = i; max_c = c; }
        }
        V3 d = normalize(ray.d);
        HitInfo hi{};
        hi.pos = ray.d * INFINITY;
        hi.norm = -ray.d;
        hi.dls = false;
        hi.has_continue = false;
        if (!(max_c < 0.0f) && !(max_c > 0.0f)) {  // partial_cmp Equal/None: reference panics
            hi.emissive = mk(0.f, 0.f, 0.f);
            return hi;
        }
        bool neg = max_c < 0.0f;
        switch (max_idx) {
            case 0: hi.emissive = sample_face(d.z, d.y, d.x, neg ? RT_FACE_NEG_X : RT_FACE_POS_X); break;
            case 1: hi.emissive = sample_face(d.x, d.z, d.y, neg ? RT_FACE_NEG_Y : RT_FACE_POS_Y); break;
            default: hi.emissive = sample_face(d.x, d.y, d.z, neg ? RT_FACE_NEG_Z : RT_FACE_POS_Z); break;
        }
        return hi;
    }
    bool continue_ray(const Ray&, const HitInfo&, V3*, Ray*) const override { return false; }
};

// ------------------------------------------------------------------ meshes
// 4x4 inverse as nalgebra's do_inverse4 (cofactor expansion, MESA gluInvertMatrix form) on
// the column-major slice m; false when the determinant is zero.
static bool inverse4(const float* m, float* inv) {
    inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] +
             m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] -
             m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] +
             m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] -
              m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] -
             m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] +
             m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] -
             m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] +
              m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] +
             m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] -
             m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] +
              m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] -
              m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] -
             m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] +
             m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] -
              m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] +
              m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    float det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    if (det == 0.0f) return false;
    float inv_det = 1.0f / det;
    for (int i = 0; i < 16; ++i) inv[i] = inv[i] * inv_det;
    return true;
}

struct MeshTri final : Element {
    const rt_scene_desc* sc;
    const rt_mesh_prim* pr;
    uint32_t tri;
    M3 normal_transform;
    Image tex, nmap, mrmap;

    MeshTri(const rt_scene_desc* sc_, const rt_mesh* mesh, const rt_mesh_prim* pr_, uint32_t tri_)
        : sc(sc_), pr(pr_), tri(tri_) {
        if (pr->base_color_tex >= 0) tex.t = &sc->textures[pr->base_color_tex];
        if (pr->normal_tex >= 0) nmap.t = &sc->textures[pr->normal_tex];
        if (pr->metal_rough_tex >= 0) mrmap.t = &sc->textures[pr->metal_rough_tex];
        normal_transform = generate_norm_type(mesh);
    }
    uint32_t idx(int k) const { return pr->indices[3 * (size_t)tri + k]; }
    V3 pos(uint32_t i) const { return mk(pr->poses + 3 * (size_t)i); }
    V3 vert(int k) const { return pos(idx(k)); }  // VertexFromMesh::index (mesh/triangle.rs:16-23)

    // NormFromMesh::get_face_norm (mesh/triangle.rs:125-132)
    V3 face_norm() const { return normalize(cross(vert(1) - vert(0), vert(2) - vert(0))); }

    // NormFromMesh::generate_norm_type (mesh/triangle.rs:45-83)
    M3 generate_norm_type(const rt_mesh* mesh) const {
        float inv[16];
        if (!inverse4(mesh->trans_mat, inv)) std::abort();  // "non invertible world?"
        M3 t3;  // transpose(inverse) resized to 3x3; inv is column-major
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) t3.m[i][j] = inv[i * 4 + j];
        V3 fn = face_norm();
        if (pr->normal_tex < 0) return t3;
        if (pr->tangents) {
            V3 tan = mk(0.f, 0.f, 0.f);  // Sum<Vector3>: fold from zero
            for (int k = 0; k < 3; ++k) tan = tan + mk(pr->tangents + 3 * (size_t)idx(k));
            tan = normalize(tan);
            V3 bitan = cross(tan, fn);
            M3 cols{};
            cols.set_col(0, normalize(tan));
            cols.set_col(1, normalize(bitan));
            cols.set_col(2, mk(0.f, 0.f, 0.f));
            M3 r = mul(t3, cols);
            r.set_col(2, fn);
            for (int i = 0; i < 3; ++i) r.set_col(i, normalize(r.col(i)));
            return r;
        }
        return norm_type_from_tex_coords(fn, t3);
    }
    // mesh/triangle.rs:85-122 (uses the base-colour UVs)
    M3 norm_type_from_tex_coords(V3 fn, const M3& t3) const {
        if (!pr->base_color_uv) return t3;
        const float* uv = pr->base_color_uv;
        float t1x = uv[2 * idx(1)] - uv[2 * idx(0)], t1y = uv[2 * idx(1) + 1] - uv[2 * idx(0) + 1];
        float t2x = uv[2 * idx(2)] - uv[2 * idx(0)], t2y = uv[2 * idx(2) + 1] - uv[2 * idx(0) + 1];
        // Matrix2::from_columns([t1, t2]) = [[t1x, t2x], [t1y, t2y]]; nalgebra 2x2 inverse.
        float m11 = t1x, m12 = t2x, m21 = t1y, m22 = t2y;
        float det = m11 * m22 - m21 * m12;
        if (det == 0.0f) return t3;
        float i11 = m22 / det, i12 = -m12 / det, i21 = -m21 / det, i22 = m11 / det;
        V3 e1 = vert(1) - vert(0), e2 = vert(2) - vert(0);
        // incomplete = [e1 e2] * inv  (3x2 * 2x2)
        M3 r{};
        r.set_col(0, mk(e1.x * i11 + e2.x * i21, e1.y * i11 + e2.y * i21, e1.z * i11 + e2.z * i21));
        r.set_col(1, mk(e1.x * i12 + e2.x * i22, e1.y * i12 + e2.y * i22, e1.z * i12 + e2.z * i22));
        r.set_col(2, mk(0.f, 0.f, 0.f));
        for (int i = 0; i < 2; ++i) r.set_col(i, normalize(r.col(i)));
        r = mul(t3, r);
        r.set_col(2, fn);
        for (int i = 0; i < 3; ++i) r.set_col(i, normalize(r.col(i)));
        return r;
    }
    // tex_coord_from_bary (mesh/triangle.rs:228-237)
    void tex_coord(const float* coords, float b1, float b2, float* u, float* v) const {
        float b0 = 1.0f - b2 - b1;
        float bc[3] = {b0, b1, b2};
        float su = 0.0f, sv = 0.0f;
        for (int k = 0; k < 3; ++k) {
            su = su + coords[2 * idx(k)] * bc[k];
            sv = sv + coords[2 * idx(k) + 1] * bc[k];
        }
        *u = su; *v = sv;
    }
    // NormFromMesh::get_norm (mesh/triangle.rs:136-157)
    V3 get_norm(float b1, float b2) const {
        if (pr->normal_tex >= 0) {
            float u, v;
            tex_coord(pr->normal_uv, b1, b2, &u, &v);
            M3 sm;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) sm.m[i][j] = pr->normal_scale * normal_transform.m[i][j];
            return normalize(mul(sm, nmap.get_pixel(u, v)));
        }
        V3 cum = mk(0.f, 0.f, 0.f);
        for (int k = 0; k < 3; ++k) cum = cum + mk(pr->norms + 3 * (size_t)idx(k));
        cum = mul(normal_transform, cum);
        return normalize(cum);
    }
    // RgbFromMesh::get_rgb (mesh/triangle.rs:166-178)
    V3 get_rgb(float b1, float b2) const {
        V3 f = mk(pr->base_color_factor);
        if (!pr->base_color_uv || pr->base_color_tex < 0) return f;
        float u, v;
        tex_coord(pr->base_color_uv, b1, b2, &u, &v);
        return cmul(f, tex.get_pixel(u, v));
    }
    // DivertsRayFromMesh::divert_ray_seed (mesh/triangle.rs:190-207)
    Seeding divert_ray_seed(const Ray& ray, V3 n, float b1, float b2) const {
        float metal, rough;
        if (pr->metal_rough_uv && pr->metal_rough_tex >= 0) {
            float u, v;
            tex_coord(pr->metal_rough_uv, b1, b2, &u, &v);
            V3 mr = mrmap.get_pixel(u, v);
            metal = mr.z * pr->metal;
            rough = mr.y * pr->rough;
        } else {
            metal = pr->metal;
            rough = pr->rough;
        }
        const float CUSTOM_ATTEN = 1.0f;
        float r0 = 0.04f + (1.0f - 0.04f) * metal;
        float reflectance = r0 + (1.0f - r0) * CUSTOM_ATTEN * (1.0f - std::pow(std::fabs(dot(ray.d, n)), 5.0f));
        Seeding s;
        float u = rng_f32();  // DynDiffSpec::should_diff (dyn_diff_spec.rs:9-13)
        s.diff = u < 1.0f - reflectance;
        s.rough = rough;
        return s;
    }

    bool is_mesh() const override { return true; }
    bool intersect(const Ray& ray, HitResult* hr) const override {
        return mt_intersect(vert(0), vert(1), vert(2), ray, hr);
    }
    bool give_aabb(Aabb* b) const override { tri_aabb(vert(0), vert(1), vert(2), b); return true; }
    HitInfo hit_info(const HitResult& hr, const Ray& ray) const override {  // generic.rs:78-92
        HitInfo hi{};
        V3 n = get_norm(hr.bu, hr.bv);
        hi.seed = divert_ray_seed(ray, n, hr.bu, hr.bv);
        hi.bu = hr.bu; hi.bv = hr.bv;
        hi.pos = (ray.d * hr.l + ray.o) + n * EPS;
        hi.norm = n;
        hi.emissive = mk(0.f, 0.f, 0.f);
        hi.dls = false;
        hi.has_continue = true;
        return hi;
    }
    bool continue_ray(const Ray& ray, const HitInfo& hi, V3* rgb, Ray* out) const override {
        // divert_new_ray (mesh/triangle.rs:209-225) then get_rgb (generic.rs:64)
        MIX(MIX_MESH);
        Ray r = hi.seed.diff ? diff(ray, hi.norm, hi.pos) : spec(ray, hi.norm, hi.pos);
        float u = rng_f32();
        float v = rng_f32();
        float w = rng_f32();
        V3 scatter = hi.seed.rough * normalize(mk(u, v, w));
        r.d = normalize(r.d + scatter);
        *out = r;
        *rgb = get_rgb(hi.bu, hi.bv) * 1.0f;
        return true;
    }
};

// ------------------------------------------------------------------ closest hit
// (src/ray/closest_hit.rs:6-30)
struct Indexed { uint32_t idx; const Element* e; };
struct Closest {
    bool found = false;
    uint32_t elem_idx = 0;
    HitResult hr{};
};
static Closest closest_ray_hit(const Ray& ray, const Indexed* elems, size_t n) {
    Closest best;
    const float lim = EPS * 20.0f;
    for (size_t k = 0; k < n; ++k) {
        HitResult hr;
        if (!elems[k].e->intersect(ray, &hr)) continue;
        if (raylen_cmp(hr.l, lim) < 0) continue;               // :16
        if (!best.found || raylen_cmp(hr.l, best.hr.l) < 0) {   // min_by_key: first minimum
            best.found = true;
            best.elem_idx = elems[k].idx;
            best.hr = hr;
        }
    }
    return best;
}

// ------------------------------------------------------------------ KD tree (kdtree.rs)
struct Node {
    bool leaf = false;
    int axis = 0;
    float split = 0.f;
    std::unique_ptr<Node> low, high;
    std::vector<Indexed> elems;
};
struct EA { uint32_t idx; const Element* e; Aabb b; };

// node_from_elems (kdtree.rs:107-137)
static std::unique_ptr<Node> node_from_elems(const std::vector<const EA*>& ea, size_t depth,
                                             size_t max_depth) {
    auto node = std::make_unique<Node>();
    int axis = (int)(depth % 3);
    if (depth > max_depth || ea.size() <= 1) {
        node->leaf = true;
        node->elems.reserve(ea.size());
        for (const EA* p : ea) node->elems.push_back(Indexed{p->idx, p->e});
        return node;
    }
    V3 sum = mk(0.f, 0.f, 0.f);  // Sum<Vector3>: fold from zero, sequential
    for (const EA* p : ea) sum = sum + centroid(p->b);
    V3 split = sum / (float)ea.size();
    std::vector<const EA*> low, high;
    for (const EA* p : ea) {
        if (p->b.hi[axis] >= split[axis]) high.push_back(p);
        if (p->b.lo[axis] <= split[axis]) low.push_back(p);
    }
    node->axis = axis;
    node->split = split[axis];
    node->low = node_from_elems(low, depth + 1, max_depth);
    node->high = node_from_elems(high, depth + 1, max_depth);
    return node;
}

struct KdTree {
    Aabb aabb;
    std::unique_ptr<Node> node;
    std::vector<Indexed> unconditional;

    // KdTree::build (kdtree.rs:26-56)
    void build(const std::vector<EA>& ea, size_t max_depth) {
        for (int a = 0; a < 3; ++a) {
            float lo = ea[0].b.lo[a], hi = ea[0].b.hi[a];
            for (size_t k = 1; k < ea.size(); ++k) { lo = rmin(lo, ea[k].b.lo[a]); hi = rmax(hi, ea[k].b.hi[a]); }
            aabb.lo[a] = lo; aabb.hi[a] = hi;
        }
        std::vector<const EA*> ptrs;
        ptrs.reserve(ea.size());
        for (const EA& e : ea) ptrs.push_back(&e);
        node = node_from_elems(ptrs, 0, max_depth);
    }

    // closest_ray_hit (kdtree.rs:58-64)
    Closest closest(const Ray& ray) const {
        int a0, a1;
        float entry, exit_t;
        if (!node || !get_entry_exit(aabb, ray, &a0, &entry, &a1, &exit_t))
            return closest_ray_hit(ray, unconditional.data(), unconditional.size());
        return stack_search(ray, entry, exit_t);
    }

    // stack_search (kdtree.rs:66-104)
    Closest stack_search(const Ray& ray, float entry_t0, float exit_t0) const {
        struct Item { const Node* n; float entry, exit; int depth; };  // depth: instrumentation only
        std::vector<Item> stack;
        stack.push_back(Item{node.get(), entry_t0, exit_t0, 0});
        while (!stack.empty()) {
            Item it = stack.back();
            stack.pop_back();
            const Node* cur = it.n;
            float entry_t = it.entry, exit_t = it.exit;
            int depth = it.depth;
            while (!cur->leaf) {
                COUNT(nodes, 1);
                if (g_mix) g_mix[MIX_NODE_D0 + (depth < 39 ? depth : 39)]++;
                int a = cur->axis;
                float d = ray.d[a];
                if (std::fabs(d) < EPS) d = d < 0.0f ? -EPS : EPS;
                float t = (cur->split - ray.o[a]) / d;
                const Node* near = d > 0.0f ? cur->low.get() : cur->high.get();
                const Node* far = d > 0.0f ? cur->high.get() : cur->low.get();
                if (t >= exit_t) {
                    cur = near;
                } else if (t <= entry_t) {
                    cur = far;
                } else {
                    stack.push_back(Item{far, t, exit_t, depth + 1});
                    cur = near;
                    exit_t = t;
                }
                ++depth;
            }
            COUNT(nodes, 1);
            COUNT(leaf_refs, cur->elems.size());
            Closest c = closest_ray_hit(ray, cur->elems.data(), cur->elems.size());
            if (c.found && c.hr.l <= exit_t + EPS) return c;
        }
        return closest_ray_hit(ray, unconditional.data(), unconditional.size());
    }
};

// ------------------------------------------------------------------ scene assembly
struct Scene {
    std::vector<std::unique_ptr<Element>> owned;
    std::vector<const Element*> renderables;
    KdTree kd;

    // decompose_groups + renderable split (draw_scene.rs:57-69, 112-130)
    bool build(const rt_scene_desc* sc, size_t kd_depth) {
        for (uint32_t i = 0; i < sc->n_elems; ++i) {
            const rt_elem& el = sc->elems[i];
            switch (el.kind) {
                case RT_ELEM_SPHERE: owned.emplace_back(new Sphere(&sc->spheres[el.index])); break;
                case RT_ELEM_FREE_TRI: owned.emplace_back(new FreeTri(&sc->free_tris[el.index])); break;
                case RT_ELEM_CUBE_MAP: owned.emplace_back(new CubeMap(&sc->cube_maps[el.index], sc)); break;
                default: return false;
            }
        }
        for (uint32_t m = 0; m < sc->n_meshes; ++m) {
            const rt_mesh& mesh = sc->meshes[m];
            for (uint32_t p = 0; p < mesh.n_prims; ++p)
                for (uint32_t t = 0; t < mesh.prims[p].n_tris; ++t)
                    owned.emplace_back(new MeshTri(sc, &mesh, &mesh.prims[p], t));
        }
        std::vector<EA> ea;
        for (size_t i = 0; i < owned.size(); ++i) {
            renderables.push_back(owned[i].get());
            Aabb b;
            if (owned[i]->give_aabb(&b)) ea.push_back(EA{(uint32_t)i, owned[i].get(), b});
            else kd.unconditional.push_back(Indexed{(uint32_t)i, owned[i].get()});
        }
        if (!ea.empty()) kd.build(ea, kd_depth);
        // The reference's KdTree::build unwraps the AABB reduce and panics on an empty list;
        // with no AABB'd renderables the oracle tests the unconditional list only.
        ea_keep = std::move(ea);
        return true;
    }
    std::vector<EA> ea_keep;  // node_from_elems holds pointers into this
};

// ------------------------------------------------------------------ radiance (radiance.rs)
struct RadInfo { bool debug_single_ray, dir_light_samp; int assured_depth; int accum; };

// russian_roulette_filter (radiance.rs:74-86); max_thres is ignored by the reference.
static bool russian_roulette(int depth, int assured, float* atten) {
    if (depth > assured) {
        MIX(MIX_RR);
        float rr = rng_f32();
        static const float THRES = 0.4f;
        if (rr < THRES) { *atten = THRES; return true; }
        return false;
    }
    *atten = 0.f;
    return true;
}

// establish_dls_contrib (radiance.rs:89-120): brute force over every renderable.
static V3 dls_contrib(const Scene& s, uint32_t omit0, int omit1, const HitInfo& hi, const Ray& ray) {
    const float NORMZE = 1.0f / (30.0f * PI);
    V3 acc = mk(0.f, 0.f, 0.f);
    std::vector<Indexed> all;
    all.reserve(s.renderables.size());
    for (size_t i = 0; i < s.renderables.size(); ++i) all.push_back(Indexed{(uint32_t)i, s.renderables[i]});
    for (size_t i = 0; i < s.renderables.size(); ++i) {
        V3 d;
        if (!s.renderables[i]->dls_emitter(hi.pos, &d)) continue;
        if (i == omit0 || (omit1 >= 0 && i == (size_t)omit1)) continue;
        float light_dot = dot(d, hi.norm);
        if (!(light_dot > 0.0f)) continue;
        Ray dr{d, hi.pos};
        Closest c = closest_ray_hit(dr, all.data(), all.size());
        if (c.found && c.elem_idx == i) {
            // The light's hit_info (radiance.rs:108) seeds a DiffSpec emitter with one draw
            // (sphere.rs:76, uniform_diff_spec.rs:33-36).  The reference makes that call only
            // after the whole recursive subtree below the vertex (radiance.rs:44-56), when no
            // path draw is left, and the emission does not depend on the seed: the draw is
            // invisible.  Restoring the stream keeps it so in the forward order too, where a
            // vertex's term is evaluated mid-path.
            const rt_rng_state saved = g_rng;
            HitInfo lh = s.renderables[i]->hit_info(c.hr, ray);
            g_rng = saved;
            acc = acc + (light_dot * lh.emissive) * NORMZE;
        }
    }
    return acc;
}

struct RadOut { V3 rgb; bool has_idx; uint32_t idx; };

// radiance (radiance.rs:20-72), recursive, no depth cap.
static RadOut radiance(const Ray& ray, const Scene& s, int depth, const RadInfo& ri) {
    COUNT(segments, 1);
    Closest c = s.kd.closest(ray);
    if (!c.found) return RadOut{mk(0.f, 0.f, 0.f), false, 0};
    COUNT(hits, 1);
    const Element* elem = s.renderables[c.elem_idx];
    if (elem->is_mesh()) COUNT(mesh_hits, 1);
    HitInfo hi = elem->hit_info(c.hr, ray);
    if (ri.debug_single_ray) return RadOut{hi.emissive, true, c.elem_idx};
    float atten;
    if (!russian_roulette(depth, ri.assured_depth, &atten)) return RadOut{hi.emissive, true, c.elem_idx};
    if (!hi.has_continue) return RadOut{hi.emissive, true, c.elem_idx};
    V3 rgb;
    Ray nr;
    elem->continue_ray(ray, hi, &rgb, &nr);
    if (atten != 0.f) rgb = rgb / atten;
    RadOut in = radiance(nr, s, depth + 1, ri);
    V3 mul = in.rgb;
    if (ri.dir_light_samp && hi.dls)
        mul = in.rgb + dls_contrib(s, c.elem_idx, in.has_idx ? (int)in.idx : -1, hi, ray);
    return RadOut{hi.emissive + cmul(rgb, mul), true, c.elem_idx};
}

// The same estimator accumulated front to back (the device path's order).
// Direct-light sampling (radiance.rs:46-56) needs the element the continued ray hits (the second
// omitted index), so a vertex's DLS term is deferred: once the next segment's closest hit is
// known, L += T_after_vertex (x) dls_contrib(vertex), before that segment's own emission.
static V3 radiance_forward(Ray ray, const Scene& s, const RadInfo& ri) {
    V3 L = mk(0.f, 0.f, 0.f), T = mk(1.f, 1.f, 1.f);
    bool pending = false;   // a DLS-eligible vertex waits for the next hit
    HitInfo p_hi{};
    Ray p_ray{};
    uint32_t p_idx = 0;
    V3 p_T = mk(0.f, 0.f, 0.f);
    for (int depth = 0;; ++depth) {
        COUNT(segments, 1);
        if (g_mix)  // spheres whose roots a brute-force closest hit computes (min_insts.py)
            for (const Element* e : s.renderables)
                if (const Sphere* sp = dynamic_cast<const Sphere*>(e)) { if (sp->disc_positive(ray)) MIX(MIX_POSDISC); }
        Closest c = s.kd.closest(ray);
        if (pending) {
            L = L + cmul(p_T, dls_contrib(s, p_idx, c.found ? (int)c.elem_idx : -1, p_hi, p_ray));
            pending = false;
        }
        if (!c.found) break;
        COUNT(hits, 1);
        const Element* elem = s.renderables[c.elem_idx];
        if (elem->is_mesh()) COUNT(mesh_hits, 1);
        HitInfo hi = elem->hit_info(c.hr, ray);
        L = L + cmul(T, hi.emissive);
        if (ri.debug_single_ray) break;
        float atten;
        if (!russian_roulette(depth, ri.assured_depth, &atten)) break;
        if (!hi.has_continue) break;
        V3 rgb;
        Ray nr;
        elem->continue_ray(ray, hi, &rgb, &nr);
        if (atten != 0.f) rgb = rgb / atten;
        T = cmul(T, rgb);
        if (ri.dir_light_samp && hi.dls) {
            pending = true;
            p_hi = hi;
            p_ray = ray;
            p_idx = c.elem_idx;
            p_T = T;
        }
        ray = nr;
    }
    return L;
}

// ------------------------------------------------------------------ ray generation (generate.rs)
struct RayCompute {
    float x_cf, y_cf, x_off, y_off;
    V3 right;
    RayCompute(int w, int h, const rt_camera& cam) {  // :13-23
        x_cf = cam.screen_width / (float)w;
        y_cf = cam.screen_height / (float)h;
        right = normalize(cross(normalize(mk(cam.d)), mk(cam.up)));
        x_off = (float)w / 2.0f;
        y_off = (float)h / 2.0f;
    }
    Ray raw(int x, int y, const rt_camera& cam) const {  // :39-66
        V3 up = mk(cam.up);
        float s_x = x_cf * ((float)x - x_off);
        float s_y = y_cf * ((float)y - y_off);
        V3 d = (mk(cam.d) + s_x * right) + s_y * up;
        if (cam.has_lens) {
            float a = cam.lens_r;
            float u = rng_f32();
            float v = rng_f32();
            float r = std::sqrt(u);
            float thet = 2.0f * PI * v;
            float lx = (r - 0.5f) * 2.0f * a * std::cos(thet);
            float ly = (r - 0.5f) * 2.0f * a * std::sin(thet);
            V3 off = right * lx + up * ly;
            return Ray{d - off, off + mk(cam.o)};
        }
        return Ray{d, mk(cam.o)};
    }
    Ray rand_ray(int x, int y, const rt_camera& cam) const {  // :24-37
        Ray ray = raw(x, y, cam);
        V3 up = mk(cam.up);
        float u = rng_f32() - 0.5f;
        float v = rng_f32() - 0.5f;
        ray.d = (ray.d + (right * u) * x_cf) + (up * v) * y_cf;
        ray.d = normalize(ray.d);
        return ray;
    }
};

}  // namespace orc

using namespace orc;

// ================================================================== C entry points
extern "C" int oracle_render(const rt_scene_desc* scene, const rt_camera* cam,
                             const rt_render_info* info, const rt_tile* tiles, uint32_t n_tiles,
                             uint64_t sample_begin, uint32_t sample_count, int threads,
                             int accum_mode, float* out_rgba, oracle_counts* counts) {
    return oracle_render_ex(scene, cam, info, tiles, n_tiles, sample_begin, sample_count, threads, accum_mode,
                            0, out_rgba, counts);
}

// mean_base: the running mean's n for sample s is s - mean_base.  0 is render_to_target_cpu's
// frame mean (draw_scene.rs:81-83); the first sample of a batch gives one batch's own mean, the
// WGSL kernel's per-dispatch fold from zero (trace.wgsl:277-318) that block_and_get_single_result
// returns (gpu_utils.rs:681-724).
extern "C" int oracle_render_ex(const rt_scene_desc* scene, const rt_camera* cam,
                                const rt_render_info* info, const rt_tile* tiles, uint32_t n_tiles,
                                uint64_t sample_begin, uint32_t sample_count, int threads,
                                int accum_mode, uint64_t mean_base, float* out_rgba, oracle_counts* counts) {
    if (mean_base > sample_begin) return RT_ERR_INVALID_ARG;
    if (!scene || !cam || !info || !tiles || !out_rgba) return RT_ERR_INVALID_ARG;
    Scene s;
    if (!s.build(scene, info->kd_tree_depth)) return RT_ERR_INVALID_ARG;
    RayCompute rc((int)info->width, (int)info->height, *cam);
    RadInfo ri{info->debug_single_ray != 0, info->dir_light_samp != 0, info->assured_depth, accum_mode};

    // pixel list: tiles concatenated (out_rgba order)
    std::vector<uint64_t> offs(n_tiles + 1, 0);
    for (uint32_t t = 0; t < n_tiles; ++t) offs[t + 1] = offs[t] + (uint64_t)tiles[t].w * tiles[t].h;
    const uint64_t n_pix = offs[n_tiles];
    if (threads <= 0) threads = (int)std::thread::hardware_concurrency();
    if (threads <= 0) threads = 1;

    std::atomic<uint64_t> next{0};
    std::vector<oracle_counts> per(threads);
    std::memset(per.data(), 0, sizeof(oracle_counts) * per.size());
    auto worker = [&](int tid) {
        g_cnt = counts ? &per[tid] : nullptr;
        uint64_t mix[MIX_N] = {0};
        g_mix = counts ? mix : nullptr;
        struct Flush {
            uint64_t* m;
            ~Flush() {
                if (!g_mix) return;
                std::lock_guard<std::mutex> lk(g_mix_mu);
                for (int i = 0; i < MIX_N; ++i) g_mix_total[i] += m[i];
                g_mix = nullptr;
            }
        } flush{mix};
        const uint64_t CH = 16;  // rayon-like dynamic chunks of pixels
        for (;;) {
            uint64_t b = next.fetch_add(CH);
            if (b >= n_pix) break;
            uint64_t e = b + CH < n_pix ? b + CH : n_pix;
            for (uint64_t p = b; p < e; ++p) {
                uint32_t t = 0;
                while (offs[t + 1] <= p) ++t;
                uint64_t local = p - offs[t];
                int32_t x = (int32_t)(tiles[t].x0 + local % tiles[t].w);
                int32_t y = (int32_t)(tiles[t].y0 + local / tiles[t].w);
                uint32_t pix = (uint32_t)y * info->width + (uint32_t)x;
                float* acc = out_rgba + 4 * p;
                float pr = 0.f, pg = 0.f, pb = 0.f;
                if (sample_begin > mean_base) { pr = acc[0]; pg = acc[1]; pb = acc[2]; }
                for (uint64_t sidx = sample_begin; sidx < sample_begin + sample_count; ++sidx) {
                    g_rng = rt_rng_init(info->seed, pix, sidx);
                    if (g_cnt) g_cnt->samples += 1;
                    Ray ray = rc.rand_ray(x, y, *cam);
                    V3 rgb = accum_mode == ORACLE_ACCUM_FORWARD ? radiance_forward(ray, s, ri)
                                                                : radiance(ray, s, 0, ri).rgb;
                    float sc = (float)(sidx - mean_base);  // draw_scene.rs:81-83
                    pr = (rgb.x + (pr * sc)) / (sc + 1.0f);
                    pg = (rgb.y + (pg * sc)) / (sc + 1.0f);
                    pb = (rgb.z + (pb * sc)) / (sc + 1.0f);
                }
                acc[0] = pr; acc[1] = pg; acc[2] = pb; acc[3] = 1.0f;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(worker, t);
    worker(0);
    for (auto& th : pool) th.join();
    g_cnt = nullptr;
    if (counts) {
        std::memset(counts, 0, sizeof(*counts));
        for (auto& c : per) {
            counts->samples += c.samples; counts->segments += c.segments;
            counts->nodes += c.nodes; counts->leaf_refs += c.leaf_refs;
            counts->sphere_tests += c.sphere_tests; counts->tri_tests += c.tri_tests;
            counts->hits += c.hits; counts->mesh_hits += c.mesh_hits;
        }
    }
    return RT_OK;
}

static void dump_dfs(const Node* n, std::vector<uint32_t>& rows, std::vector<uint32_t>& refs) {
    uint32_t split_bits;
    std::memcpy(&split_bits, &n->split, 4);
    rows.push_back(n->leaf ? 1u : 0u);
    rows.push_back((uint32_t)n->axis);
    rows.push_back(n->leaf ? (uint32_t)n->elems.size() : split_bits);
    rows.push_back((uint32_t)refs.size());
    if (n->leaf) {
        for (const Indexed& e : n->elems) refs.push_back(e.idx);
        return;
    }
    dump_dfs(n->low.get(), rows, refs);
    dump_dfs(n->high.get(), rows, refs);
}

extern "C" int oracle_kd_dump(const rt_scene_desc* scene, uint32_t max_depth, uint32_t* node_rows,
                              uint32_t node_cap, uint32_t* refs, uint32_t ref_cap,
                              uint32_t* n_refs, float bounds[6]) {
    Scene s;
    if (!s.build(scene, max_depth)) return RT_ERR_INVALID_ARG;
    if (!s.kd.node) return 0;
    std::vector<uint32_t> rows, rr;
    dump_dfs(s.kd.node.get(), rows, rr);
    uint32_t nn = (uint32_t)(rows.size() / 4);
    if (n_refs) *n_refs = (uint32_t)rr.size();
    if (bounds)
        for (int a = 0; a < 3; ++a) { bounds[2 * a] = s.kd.aabb.lo[a]; bounds[2 * a + 1] = s.kd.aabb.hi[a]; }
    if (node_rows && node_cap >= nn) std::memcpy(node_rows, rows.data(), rows.size() * 4);
    if (refs && ref_cap >= rr.size()) std::memcpy(refs, rr.data(), rr.size() * 4);
    return (int)nn;
}

extern "C" int oracle_mesh_normal_transforms(const rt_scene_desc* scene, float* out9, uint64_t cap) {
    uint64_t k = 0;
    for (uint32_t m = 0; m < scene->n_meshes; ++m) {
        const rt_mesh& mesh = scene->meshes[m];
        for (uint32_t p = 0; p < mesh.n_prims; ++p)
            for (uint32_t t = 0; t < mesh.prims[p].n_tris; ++t, ++k) {
                if (k >= cap) return RT_ERR_INVALID_ARG;
                MeshTri mt(scene, &mesh, &mesh.prims[p], t);
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j) out9[9 * k + 3 * i + j] = mt.normal_transform.m[i][j];
            }
    }
    return (int)k;
}

extern "C" int oracle_aabb_entry_exit(const float bounds[6], const float d[3], const float o[3],
                                      int* min_axis, float* entry, int* max_axis, float* exit_t) {
    Aabb b;
    for (int a = 0; a < 3; ++a) { b.lo[a] = bounds[2 * a]; b.hi[a] = bounds[2 * a + 1]; }
    return get_entry_exit(b, Ray{mk(d), mk(o)}, min_axis, entry, max_axis, exit_t) ? 1 : 0;
}

extern "C" int oracle_raylen_cmp(float a, float b) { return raylen_cmp(a, b); }

extern "C" void oracle_chunk_to_pix(int32_t idx, int32_t width, int32_t* x, int32_t* y) {
    int32_t xx = idx % width;  // target.rs:9-14
    *x = xx;
    *y = (idx - xx) / width;
}

extern "C" int oracle_sphere_intersect(const float c[3], float r, const float d[3], const float o[3],
                                       float* l) {
    rt_sphere s{};
    for (int a = 0; a < 3; ++a) s.c[a] = c[a];
    s.r = r;
    Sphere sp(&s);
    HitResult hr;
    if (!sp.intersect(Ray{mk(d), mk(o)}, &hr)) return 0;
    *l = hr.l;
    return 1;
}

extern "C" int oracle_triangle_intersect(const float v[9], const float d[3], const float o[3],
                                         float* l, float* u, float* v_out) {
    HitResult hr;
    if (!mt_intersect(mk(v), mk(v + 3), mk(v + 6), Ray{mk(d), mk(o)}, &hr)) return 0;
    *l = hr.l; *u = hr.bu; *v_out = hr.bv;
    return 1;
}

extern "C" void oracle_rng_stream(uint64_t seed, uint32_t pixel, uint64_t sample, uint32_t n, float* out) {
    rt_rng_state st = rt_rng_init(seed, pixel, sample);
    for (uint32_t i = 0; i < n; ++i) out[i] = rt_rng_next_f32(&st);
}

extern "C" void oracle_camera_ray(const rt_camera* cam, uint32_t w, uint32_t h, int32_t x, int32_t y,
                                  uint64_t seed, uint64_t sample, float d_out[3], float o_out[3]) {
    RayCompute rc((int)w, (int)h, *cam);
    g_rng = rt_rng_init(seed, (uint32_t)y * w + (uint32_t)x, sample);
    Ray r = rc.rand_ray(x, y, *cam);
    d_out[0] = r.d.x; d_out[1] = r.d.y; d_out[2] = r.d.z;
    o_out[0] = r.o.x; o_out[1] = r.o.y; o_out[2] = r.o.z;
}

extern "C" void oracle_refract(const float d[3], const float n[3], float n_out, float n_in, float u,
                               float d_out[3], float* p) {
    Ray r = refract(Ray{mk(d), mk(0.f, 0.f, 0.f)}, mk(n), mk(0.f, 0.f, 0.f), n_out, n_in, p,
                    [u] { return u; });
    d_out[0] = r.d.x; d_out[1] = r.d.y; d_out[2] = r.d.z;
}

// Shading mix of the counted renders since the last reset (continued rays by material branch:
// spec, diff, diffspec->diff, diffspec->spec, dielectric; Russian-roulette draws; all draws;
// mesh continues; forward-order segments' spheres with a positive discriminant), for
// tools/min_insts.py; then the traversal's branch-node visits by depth (tools/descent_depths.py).
extern "C" void oracle_mix_counts(uint64_t out[MIX_N], int reset) {
    std::lock_guard<std::mutex> lk(g_mix_mu);
    for (int i = 0; i < MIX_N; ++i) {
        out[i] = g_mix_total[i];
        if (reset) g_mix_total[i] = 0;
    }
}
