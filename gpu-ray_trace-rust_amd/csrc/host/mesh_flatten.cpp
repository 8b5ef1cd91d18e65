// mesh_flatten.cpp — host precompute for mesh triangles (compiled with -ffp-contract=off).
//
// Flattens every rt_mesh primitive into device-ready arrays: pre-gathered vertex positions
// per triangle (for Möller–Trumbore), the per-triangle normal transform of
// NormFromMesh::generate_norm_type (src/elements/mesh/triangle.rs:45-122) — already scaled by
// the normal-map scale when the primitive has a normal map (get_norm multiplies scale * M,
// mesh/triangle.rs:145) — and per-vertex pools (normals, the three UV sets) indexed by a
// global vertex index.  Matrix products keep nalgebra's accumulation order.
#include "mesh_flatten.h"

#include <cmath>

namespace rth {

namespace {

struct V3 { float x, y, z; };
inline V3 ld(const float* p) { return V3{p[0], p[1], p[2]}; }
inline V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 add(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
inline float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline V3 normalize(V3 a) {
    float n = std::sqrt(dot(a, a));
    return V3{a.x / n, a.y / n, a.z / n};
}
inline V3 cross(V3 a, V3 b) {
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

struct M3 {
    float m[3][3];
    V3 col(int j) const { return V3{m[0][j], m[1][j], m[2][j]}; }
    void set_col(int j, V3 v) { m[0][j] = v.x; m[1][j] = v.y; m[2][j] = v.z; }
};
M3 mul(const M3& a, const M3& b) {
    M3 c;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            c.m[i][j] = (a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j]) + a.m[i][2] * b.m[2][j];
    return c;
}

// nalgebra's 4x4 try_inverse (cofactor expansion over the column-major slice, then one
// reciprocal of the determinant applied to every entry).
bool inverse4(const float* m, float* inv) {
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
    float r = 1.0f / det;
    for (int i = 0; i < 16; ++i) inv[i] = inv[i] * r;
    return true;
}

// generate_norm_type (mesh/triangle.rs:45-83) + norm_type_from_tex_coords (:85-122)
M3 normal_transform(const rt_mesh_prim& pr, const M3& t3, uint32_t i0, uint32_t i1, uint32_t i2) {
    V3 p0 = ld(pr.poses + 3 * (size_t)i0), p1 = ld(pr.poses + 3 * (size_t)i1), p2 = ld(pr.poses + 3 * (size_t)i2);
    V3 fn = normalize(cross(sub(p1, p0), sub(p2, p0)));
    if (pr.normal_tex < 0) return t3;
    if (pr.tangents) {
        V3 tan{0.f, 0.f, 0.f};
        tan = add(tan, ld(pr.tangents + 3 * (size_t)i0));
        tan = add(tan, ld(pr.tangents + 3 * (size_t)i1));
        tan = add(tan, ld(pr.tangents + 3 * (size_t)i2));
        tan = normalize(tan);
        V3 bitan = cross(tan, fn);
        M3 cols{};
        cols.set_col(0, normalize(tan));
        cols.set_col(1, normalize(bitan));
        cols.set_col(2, V3{0.f, 0.f, 0.f});
        M3 r = mul(t3, cols);
        r.set_col(2, fn);
        for (int c = 0; c < 3; ++c) r.set_col(c, normalize(r.col(c)));
        return r;
    }
    if (!pr.base_color_uv) return t3;
    const float* uv = pr.base_color_uv;
    float m11 = uv[2 * i1] - uv[2 * i0], m21 = uv[2 * i1 + 1] - uv[2 * i0 + 1];
    float m12 = uv[2 * i2] - uv[2 * i0], m22 = uv[2 * i2 + 1] - uv[2 * i0 + 1];
    float det = m11 * m22 - m21 * m12;
    if (det == 0.0f) return t3;
    float a11 = m22 / det, a12 = -m12 / det, a21 = -m21 / det, a22 = m11 / det;
    V3 e1 = sub(p1, p0), e2 = sub(p2, p0);
    M3 r{};
    r.set_col(0, V3{e1.x * a11 + e2.x * a21, e1.y * a11 + e2.y * a21, e1.z * a11 + e2.z * a21});
    r.set_col(1, V3{e1.x * a12 + e2.x * a22, e1.y * a12 + e2.y * a22, e1.z * a12 + e2.z * a22});
    r.set_col(2, V3{0.f, 0.f, 0.f});
    for (int c = 0; c < 2; ++c) r.set_col(c, normalize(r.col(c)));
    r = mul(t3, r);
    r.set_col(2, fn);
    for (int c = 0; c < 3; ++c) r.set_col(c, normalize(r.col(c)));
    return r;
}

}  // namespace

int flatten_meshes(const rt_scene_desc* sc, MeshFlat* out) {
    *out = MeshFlat{};
    uint32_t vbase = 0;
    for (uint32_t m = 0; m < sc->n_meshes; ++m) {
        const rt_mesh& mesh = sc->meshes[m];
        float inv[16];
        if (!inverse4(mesh.trans_mat, inv)) return RT_ERR_INVALID_ARG;  // "non invertible world?"
        M3 t3;  // (M^-1)^T, top-left 3x3; inv is column-major
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) t3.m[i][j] = inv[i * 4 + j];
        for (uint32_t p = 0; p < mesh.n_prims; ++p) {
            const rt_mesh_prim& pr = mesh.prims[p];
            if (!pr.poses || !pr.norms || !pr.indices) return RT_ERR_INVALID_ARG;
            for (int t : {pr.base_color_tex, pr.normal_tex, pr.metal_rough_tex})
                if (t >= (int32_t)sc->n_textures) return RT_ERR_INVALID_ARG;
            if ((pr.normal_tex >= 0 && !pr.normal_uv) || (pr.base_color_tex >= 0 && !pr.base_color_uv))
                return RT_ERR_INVALID_ARG;
            const uint32_t prim_id = (uint32_t)out->prims.size();
            FlatPrim fp{};
            for (int i = 0; i < 3; ++i) fp.base_factor[i] = pr.base_color_factor[i];
            fp.base_tex = (pr.base_color_uv && pr.base_color_tex >= 0) ? pr.base_color_tex : -1;
            fp.normal_tex = pr.normal_tex;
            fp.mr_tex = (pr.metal_rough_uv && pr.metal_rough_tex >= 0) ? pr.metal_rough_tex : -1;
            fp.metal = pr.metal;
            fp.rough = pr.rough;
            out->prims.push_back(fp);
            for (uint32_t v = 0; v < pr.n_verts; ++v) {
                out->norms.push_back(pr.norms[3 * (size_t)v]);
                out->norms.push_back(pr.norms[3 * (size_t)v + 1]);
                out->norms.push_back(pr.norms[3 * (size_t)v + 2]);
                out->norms.push_back(0.f);
                for (int k = 0; k < 2; ++k) {
                    out->base_uv.push_back(pr.base_color_uv ? pr.base_color_uv[2 * (size_t)v + k] : 0.f);
                    out->normal_uv.push_back(pr.normal_uv ? pr.normal_uv[2 * (size_t)v + k] : 0.f);
                    out->mr_uv.push_back(pr.metal_rough_uv ? pr.metal_rough_uv[2 * (size_t)v + k] : 0.f);
                }
            }
            for (uint32_t t = 0; t < pr.n_tris; ++t) {
                uint32_t i0 = pr.indices[3 * (size_t)t], i1 = pr.indices[3 * (size_t)t + 1],
                         i2 = pr.indices[3 * (size_t)t + 2];
                if (i0 >= pr.n_verts || i1 >= pr.n_verts || i2 >= pr.n_verts) return RT_ERR_INVALID_ARG;
                FlatTri ft{};
                ft.prim = prim_id;
                ft.v[0] = vbase + i0;
                ft.v[1] = vbase + i1;
                ft.v[2] = vbase + i2;
                M3 nt = normal_transform(pr, t3, i0, i1, i2);
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j)
                        ft.m[3 * i + j] = pr.normal_tex >= 0 ? pr.normal_scale * nt.m[i][j] : nt.m[i][j];
                out->tris.push_back(ft);
                for (uint32_t idx : {i0, i1, i2})
                    for (int k = 0; k < 4; ++k) out->verts.push_back(k < 3 ? pr.poses[3 * (size_t)idx + k] : 0.f);
            }
            vbase += pr.n_verts;
        }
    }
    return RT_OK;
}

}  // namespace rth

// Test hook (not in rt_abi.h): the per-triangle normal transforms exactly as uploaded,
// row-major, for comparison with the oracle's restatement.  Returns the triangle count.
extern "C" int rtx_mesh_normal_transforms(const rt_scene_desc* sc, float* out9, uint64_t cap) {
    rth::MeshFlat f;
    int st = rth::flatten_meshes(sc, &f);
    if (st) return st;
    if (f.tris.size() > cap) return RT_ERR_INVALID_ARG;
    for (size_t t = 0; t < f.tris.size(); ++t)
        for (int i = 0; i < 9; ++i) out9[9 * t + i] = f.tris[t].m[i];
    return (int)f.tris.size();
}
