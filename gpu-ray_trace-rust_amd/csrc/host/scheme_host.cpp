// scheme_host.cpp — the caller of the boundary in C++: scheme YAML (or its JSON form) +
// glTF models + asset packs -> rt_scene_desc / rt_camera / rt_render_info, and the PNG output
// writer.  Restates, in the reference's f32 operation order:
//   Scheme::from_yml + apply_corrections     src/builder/mod.rs:63-72
//   Vec<Member> -> renderables               src/builder/inner.rs:21-64 (member order)
//   Model::to_meshes                         src/builder/pr/model.rs:19-207
//   DistantCubeMap textures                  src/builder/pr/distant_cube_map.rs:19-23
//   process_output_routine (flipped PNG)     src/ui_util.rs:37-54
// It produces bit-identical descriptions to the Python host (rt_amd/scheme.py, rt_amd/gltf.py;
// tests/test_host_cpp.py checks every array).  Assets come from the pack store (pack.h).
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/rt_abi.h"
#include "doc.h"
#include "pack.h"

using rth::Node;
using rth::NodeP;

namespace {

thread_local std::string g_err;

float f32(const Node* n) {
    if (!n) throw std::runtime_error("missing number");
    return (float)n->num();  // serde: f64 parse, rounded to f32
}
const Node* need(const Node* m, const char* key) {
    const Node* v = m ? m->get(key) : nullptr;
    if (!v) throw std::runtime_error(std::string("scheme: missing '") + key + "'");
    return v;
}
void v3(const Node* n, float out[3]) {
    if (!n || n->kind != Node::Seq || n->seq.size() != 3) throw std::runtime_error("expected a 3-vector");
    for (int i = 0; i < 3; ++i) out[i] = f32(n->seq[i].get());
}
// (tag, value) of an externally tagged enum; a unit variant is a plain string
std::string tag_of(const Node* n, const Node** val) {
    if (n && n->kind == Node::Tag) {
        *val = n->tagged();
        return n->text;
    }
    if (n && (n->kind == Node::Scalar || n->kind == Node::String)) {
        *val = nullptr;
        return n->text;
    }
    throw std::runtime_error("scheme: expected an enum value");
}

rt_material material(const Node* m) {  // UniformDiffuseSpec (material/uniform_diff_spec.rs:7-19)
    rt_material out{};
    const Node* em = m->get("emissive");
    if (em && em->kind != Node::Null) {
        out.has_emissive = 1;
        v3(em, out.emissive);
    }
    const Node* val = nullptr;
    const std::string k = tag_of(need(m, "divert_ray"), &val);
    if (k == "Spec") out.divert = RT_DIVERT_SPEC;
    else if (k == "Diff") out.divert = RT_DIVERT_DIFF;
    else if (k == "DiffSpec") {
        out.divert = RT_DIVERT_DIFFSPEC;
        out.diffp = f32(need(val, "diffp"));
    } else if (k == "Dielectric") {
        out.divert = RT_DIVERT_DIELECTRIC;
        out.n_out = f32(need(val, "n_out"));
        out.n_in = f32(need(val, "n_in"));
    } else {
        throw std::runtime_error("unknown divert_ray " + k);
    }
    return out;
}

// ------------------------------------------------------------------ f32 matrix helpers (row-major)
struct M4 {
    float m[4][4];
};
M4 eye4() {
    M4 r{};
    for (int i = 0; i < 4; ++i) r.m[i][i] = 1.0f;
    return r;
}
M4 mul4(const M4& a, const M4& b) {  // nalgebra accumulation order
    M4 c{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float s = a.m[i][0] * b.m[0][j];
            for (int k = 1; k < 4; ++k) s = s + a.m[i][k] * b.m[k][j];
            c.m[i][j] = s;
        }
    return c;
}
M4 euler4(float r, float p, float y) {  // Rotation3::from_euler_angles, homogeneous
    const float sr = sinf(r), cr = cosf(r), sp = sinf(p), cp = cosf(p), sy = sinf(y), cy = cosf(y);
    M4 m = eye4();
    m.m[0][0] = cy * cp;
    m.m[0][1] = (cy * sp) * sr - sy * cr;
    m.m[0][2] = (cy * sp) * cr + sy * sr;
    m.m[1][0] = sy * cp;
    m.m[1][1] = (sy * sp) * sr + cy * cr;
    m.m[1][2] = (sy * sp) * cr - cy * sr;
    m.m[2][0] = -sp;
    m.m[2][1] = cp * sr;
    m.m[2][2] = cp * cr;
    return m;
}
M4 node_matrix(const Node* node) {  // gltf::scene::Transform::matrix()
    M4 r = eye4();
    if (const Node* mm = node->get("matrix")) {
        if (mm->kind != Node::Seq || mm->seq.size() != 16) throw std::runtime_error("glTF: bad node matrix");
        for (int c = 0; c < 4; ++c)
            for (int rr = 0; rr < 4; ++rr) r.m[rr][c] = f32(mm->seq[(size_t)(c * 4 + rr)].get());  // column-major
        return r;
    }
    float t[3] = {0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 1.f}, s[3] = {1.f, 1.f, 1.f};
    if (const Node* n = node->get("translation")) v3(n, t);
    if (const Node* n = node->get("rotation"))
        for (int i = 0; i < 4; ++i) q[i] = f32(n->seq.at((size_t)i).get());
    if (const Node* n = node->get("scale")) v3(n, s);
    const float qx = q[0], qy = q[1], qz = q[2], qw = q[3];
    const float x2 = qx + qx, y2 = qy + qy, z2 = qz + qz;
    const float xx2 = x2 * qx, xy2 = x2 * qy, xz2 = x2 * qz;
    const float yy2 = y2 * qy, yz2 = y2 * qz, zz2 = z2 * qz;
    const float sy2 = y2 * qw, sz2 = z2 * qw, sx2 = x2 * qw;
    M4 R = eye4();
    R.m[0][0] = 1.0f - yy2 - zz2;
    R.m[0][1] = xy2 - sz2;
    R.m[0][2] = xz2 + sy2;
    R.m[1][0] = xy2 + sz2;
    R.m[1][1] = 1.0f - xx2 - zz2;
    R.m[1][2] = yz2 - sx2;
    R.m[2][0] = xz2 - sy2;
    R.m[2][1] = yz2 + sx2;
    R.m[2][2] = 1.0f - xx2 - yy2;
    M4 T = eye4();
    T.m[0][3] = t[0];
    T.m[1][3] = t[1];
    T.m[2][3] = t[2];
    M4 S = eye4();
    S.m[0][0] = s[0];
    S.m[1][1] = s[1];
    S.m[2][2] = s[2];
    return mul4(mul4(T, R), S);
}

}  // namespace

// ---------------------------------------------------------------------------- the scheme object
struct rt_scheme {
    struct Prim {
        std::vector<float> poses, norms, tangents, base_uv, normal_uv, mr_uv;
        std::vector<uint32_t> indices;
        bool has_tangents = false;
        rt_mesh_prim abi{};
    };
    struct Mesh {
        std::vector<Prim> prims;
        std::vector<rt_mesh_prim> abi_prims;
        rt_mesh abi{};
    };
    std::vector<rt_elem> elems;
    std::vector<rt_sphere> spheres;
    std::vector<rt_free_triangle> free_tris;
    std::vector<rt_cube_map> cube_maps;
    std::vector<std::vector<float>> texels;      // RGB f32 per texture
    std::vector<std::pair<uint32_t, uint32_t>> tex_dims;  // (width, height)
    std::vector<rt_texture> textures;
    std::vector<std::unique_ptr<Mesh>> meshes;
    std::vector<rt_mesh> abi_meshes;
    rt_scene_desc desc{};
    rt_camera cam{};
    rt_render_info info{};
    uint32_t spp = 0, batch = 0, use_gpu = 0, animation = 0;
    // kept to build animation frames (rt_scheme_frame)
    NodeP root;
    std::string assets_root;
    bool has_assets = false;
    uint64_t seed = 0;
};

// Per-member replacement values of one animation frame (extract_anim, inner.rs:113-210).
struct MemberOverride {
    bool c = false, trans = false, euler = false;
    float cv[3], tv[3], ev[3];
};

namespace {

int add_texture(rt_scheme* s, const rth::NpyArray& img) {  // image::to_rgb32f: c / 255
    if (img.descr != "|u1" || img.shape.size() != 3) throw std::runtime_error("texture is not H x W x C u8");
    const uint64_t h = img.shape[0], w = img.shape[1], c = img.shape[2];
    if (c != 1 && c != 3 && c != 4) throw std::runtime_error("texture channel count");
    std::vector<float> t(3 * h * w);
    for (uint64_t p = 0; p < h * w; ++p)
        for (int k = 0; k < 3; ++k) t[3 * p + (uint64_t)k] = (float)img.data[p * c + (c == 1 ? 0 : (uint64_t)k)] / 255.0f;
    s->texels.push_back(std::move(t));
    s->tex_dims.emplace_back((uint32_t)w, (uint32_t)h);
    return (int)s->texels.size() - 1;
}

struct Accessor {
    std::vector<uint8_t> raw;  // count * n * itemsize, tightly packed
    uint32_t comp = 0, n = 0, count = 0, itemsize = 0;
};

Accessor read_accessor(const Node* doc, const std::vector<rth::NpyArray>& bufs, size_t idx) {
    const Node* acc = need(doc, "accessors")->seq.at(idx).get();
    if (acc->get("sparse")) throw std::runtime_error("glTF: sparse accessors");
    Accessor a;
    a.comp = (uint32_t)need(acc, "componentType")->num();
    const std::string ty = need(acc, "type")->str();
    a.n = ty == "SCALAR" ? 1 : ty == "VEC2" ? 2 : ty == "VEC3" ? 3 : ty == "VEC4" ? 4 : ty == "MAT2" ? 4 : ty == "MAT3" ? 9 : 16;
    a.itemsize = (a.comp == 5120 || a.comp == 5121) ? 1 : (a.comp == 5122 || a.comp == 5123) ? 2 : 4;
    a.count = (uint32_t)need(acc, "count")->num();
    const size_t row = (size_t)a.n * a.itemsize;
    a.raw.assign((size_t)a.count * row, 0);
    const Node* bvi = acc->get("bufferView");
    if (!bvi) return a;
    const Node* bv = need(doc, "bufferViews")->seq.at((size_t)bvi->num()).get();
    const rth::NpyArray& buf = bufs.at((size_t)need(bv, "buffer")->num());
    const size_t off = (size_t)(bv->get("byteOffset") ? bv->get("byteOffset")->num() : 0) +
                       (size_t)(acc->get("byteOffset") ? acc->get("byteOffset")->num() : 0);
    size_t stride = bv->get("byteStride") ? (size_t)bv->get("byteStride")->num() : 0;
    if (!stride) stride = row;
    if (a.count && off + (size_t)(a.count - 1) * stride + row > buf.data.size()) throw std::runtime_error("glTF: accessor out of range");
    for (uint32_t i = 0; i < a.count; ++i) std::memcpy(&a.raw[i * row], &buf.data[off + i * stride], row);
    return a;
}
// component k of element i as f32: float accessors verbatim; integers as value (astype) or,
// when `norm`, value / max of the type (gltf Normalize, u8/255, u16/65535)
float comp_f32(const Accessor& a, uint32_t i, uint32_t k, bool norm) {
    const uint8_t* p = &a.raw[((size_t)i * a.n + k) * a.itemsize];
    switch (a.comp) {
        case 5126: { float v; std::memcpy(&v, p, 4); return v; }
        case 5121: return norm ? (float)p[0] / 255.0f : (float)p[0];
        case 5120: return norm ? (float)(int8_t)p[0] / 127.0f : (float)(int8_t)p[0];
        case 5123: { uint16_t v; std::memcpy(&v, p, 2); return norm ? (float)v / 65535.0f : (float)v; }
        case 5122: { int16_t v; std::memcpy(&v, p, 2); return norm ? (float)v / 32767.0f : (float)v; }
        case 5125: { uint32_t v; std::memcpy(&v, p, 4); return norm ? (float)v / 4294967295.0f : (float)v; }
    }
    throw std::runtime_error("glTF: component type");
}
uint32_t comp_u32(const Accessor& a, uint32_t i) {
    const uint8_t* p = &a.raw[(size_t)i * a.n * a.itemsize];
    switch (a.comp) {
        case 5121: return p[0];
        case 5123: { uint16_t v; std::memcpy(&v, p, 2); return v; }
        case 5125: { uint32_t v; std::memcpy(&v, p, 4); return v; }
    }
    throw std::runtime_error("glTF: index component type");
}

void load_model(rt_scheme* s, const Node* model, rth::PackStore& store, const MemberOverride* o) {  // Model::to_meshes
    std::string dir, rel;
    rth::PackStore::split(need(model, "path")->str(), &dir, &rel);
    const rth::NpzFile* pk = store.pack(dir);
    if (!pk || !pk->has("gltf:" + rel)) throw std::runtime_error("glTF not in the asset pack: " + rel);
    const rth::NpyArray js = pk->read("gltf:" + rel);
    const NodeP doc = rth::parse_json(std::string(js.data.begin(), js.data.end()));
    std::vector<rth::NpyArray> bufs;
    if (const Node* b = doc->get("buffers"))
        for (size_t i = 0; i < b->seq.size(); ++i) bufs.push_back(pk->read("buf:" + rel + ":" + std::to_string(i)));
    const std::string base = rel.find('/') == std::string::npos ? "" : rel.substr(0, rel.rfind('/'));
    std::map<size_t, int> tex_ids;
    auto texture = [&](const Node* tinfo) -> int {  // images[texture index] (model.rs:157)
        const size_t ti = (size_t)need(tinfo, "index")->num();
        auto it = tex_ids.find(ti);
        if (it != tex_ids.end()) return it->second;
        int id = -1;
        const Node* images = doc->get("images");
        const Node* uri = images && ti < images->seq.size() ? images->seq[ti]->get("uri") : nullptr;
        if (uri) {
            const std::string key = "img:" + (base.empty() ? uri->str() : base + "/" + uri->str());
            if (pk->has(key)) id = add_texture(s, pk->read(key));  // absent image: declared fallback
        }
        tex_ids[ti] = id;
        return id;
    };

    // T(translation) * S(uniform_scale) * R(euler) (model.rs:23-29)
    float t[3], e[3];
    v3(need(model, "translation"), t);
    v3(need(model, "euler_angles"), e);
    if (o && o->trans) std::memcpy(t, o->tv, sizeof(t));
    if (o && o->euler) std::memcpy(e, o->ev, sizeof(e));
    const float sc = f32(need(model, "uniform_scale"));
    M4 T = eye4(), S = eye4();
    T.m[0][3] = t[0];
    T.m[1][3] = t[1];
    T.m[2][3] = t[2];
    S.m[0][0] = S.m[1][1] = S.m[2][2] = sc;
    const M4 transform = mul4(mul4(T, S), euler4(e[0], e[1], e[2]));

    std::function<void(size_t, const M4&)> explore = [&](size_t ni, const M4& parent) {  // model.rs:43-53
        const Node* node = need(doc.get(), "nodes")->seq.at(ni).get();
        const M4 trans = mul4(parent, node_matrix(node));
        if (const Node* mi = node->get("mesh")) {
            auto mesh = std::make_unique<rt_scheme::Mesh>();
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < 4; ++r) mesh->abi.trans_mat[c * 4 + r] = trans.m[r][c];  // column-major
            const Node* m = need(doc.get(), "meshes")->seq.at((size_t)mi->num()).get();
            for (const NodeP& prim : need(m, "primitives")->seq) {  // model.rs:56-134
                if (prim->get("mode") && prim->get("mode")->num() != 4) throw std::runtime_error("glTF: only triangle lists");
                const Node* attrs = need(prim.get(), "attributes");
                rt_scheme::Prim P;
                const Accessor ia = read_accessor(doc.get(), bufs, (size_t)need(prim.get(), "indices")->num());
                P.indices.resize(ia.count * ia.n);
                for (uint32_t i = 0; i < ia.count * ia.n; ++i) P.indices[i] = comp_u32(ia, i);
                const Accessor pa = read_accessor(doc.get(), bufs, (size_t)need(attrs, "POSITION")->num());
                P.poses.resize(3 * (size_t)pa.count);
                for (uint32_t v = 0; v < pa.count; ++v) {
                    const float x = comp_f32(pa, v, 0, false), y = comp_f32(pa, v, 1, false), z = comp_f32(pa, v, 2, false);
                    for (int r = 0; r < 3; ++r)
                        P.poses[3 * (size_t)v + r] = ((trans.m[r][0] * x + trans.m[r][1] * y) + trans.m[r][2] * z) + trans.m[r][3] * 1.0f;
                }
                const Accessor na = read_accessor(doc.get(), bufs, (size_t)need(attrs, "NORMAL")->num());
                P.norms.resize(3 * (size_t)na.count);
                for (uint32_t v = 0; v < na.count; ++v)
                    for (uint32_t k = 0; k < 3; ++k) P.norms[3 * (size_t)v + k] = comp_f32(na, v, k, false);
                if (const Node* ta = attrs->get("TANGENT")) {
                    const Accessor tg = read_accessor(doc.get(), bufs, (size_t)ta->num());
                    P.tangents.resize(3 * (size_t)tg.count);
                    for (uint32_t v = 0; v < tg.count; ++v)
                        for (uint32_t k = 0; k < 3; ++k) P.tangents[3 * (size_t)v + k] = comp_f32(tg, v, k, false);
                    P.has_tangents = true;
                }
                const Node* mats = doc->get("materials");
                const Node* mat = prim->get("material") ? mats->seq.at((size_t)prim->get("material")->num()).get() : nullptr;
                const Node* pbr = mat ? mat->get("pbrMetallicRoughness") : nullptr;
                rt_mesh_prim& A = P.abi;
                A.base_color_factor[0] = A.base_color_factor[1] = A.base_color_factor[2] = 1.0f;
                if (const Node* f = pbr ? pbr->get("baseColorFactor") : nullptr)
                    for (int k = 0; k < 3; ++k) A.base_color_factor[k] = f32(f->seq.at((size_t)k).get());
                auto coords = [&](const Node* tinfo, std::vector<float>* uv) {
                    const Node* tc = tinfo->get("texCoord");
                    const std::string key = "TEXCOORD_" + std::to_string(tc ? (int)tc->num() : 0);
                    const Accessor ua = read_accessor(doc.get(), bufs, (size_t)need(attrs, key.c_str())->num());
                    uv->resize(2 * (size_t)ua.count);
                    for (uint32_t v = 0; v < ua.count; ++v)
                        for (uint32_t k = 0; k < 2; ++k) (*uv)[2 * (size_t)v + k] = comp_f32(ua, v, k, true);
                };
                A.base_color_tex = A.normal_tex = A.metal_rough_tex = -1;
                A.normal_scale = 1.0f;
                if (const Node* bt = pbr ? pbr->get("baseColorTexture") : nullptr) {
                    const int id = texture(bt);
                    if (id >= 0) {
                        A.base_color_tex = id;
                        coords(bt, &P.base_uv);
                    }
                }
                if (const Node* nt = mat ? mat->get("normalTexture") : nullptr) {
                    const int id = texture(nt);
                    if (id >= 0) {
                        A.normal_tex = id;
                        coords(nt, &P.normal_uv);
                        A.normal_scale = nt->get("scale") ? f32(nt->get("scale")) : 1.0f;
                    }
                }
                if (const Node* mt = pbr ? pbr->get("metallicRoughnessTexture") : nullptr) {
                    const int id = texture(mt);
                    if (id >= 0) {
                        A.metal_rough_tex = id;
                        coords(mt, &P.mr_uv);
                    }
                }
                A.metal = pbr && pbr->get("metallicFactor") ? f32(pbr->get("metallicFactor")) : 1.0f;
                A.rough = pbr && pbr->get("roughnessFactor") ? f32(pbr->get("roughnessFactor")) : 1.0f;
                mesh->prims.push_back(std::move(P));
            }
            s->meshes.push_back(std::move(mesh));
        }
        if (const Node* ch = node->get("children"))
            for (const NodeP& c : ch->seq) explore((size_t)c->num(), trans);
    };
    if (const Node* scenes = doc->get("scenes"))
        for (const NodeP& scn : scenes->seq)
            if (const Node* nodes = scn->get("nodes"))
                for (const NodeP& n : nodes->seq) explore((size_t)n->num(), transform);
}

void build(rt_scheme* s, const Node* root, const char* assets_root, uint64_t seed,
           const std::vector<MemberOverride>* ov = nullptr) {
    const Node* ri = need(root, "render_info");
    s->info.width = (uint32_t)need(ri, "width")->num();
    s->info.height = (uint32_t)need(ri, "height")->num();
    s->info.kd_tree_depth = (uint32_t)need(ri, "kd_tree_depth")->num();
    const Node* rad = need(ri, "rad_info");
    const Node* rr = need(rad, "russ_roull_info");
    s->info.assured_depth = (int32_t)need(rr, "assured_depth")->num();
    s->info.max_thres = f32(need(rr, "max_thres"));
    s->info.debug_single_ray = need(rad, "debug_single_ray")->is_true() ? 1u : 0u;
    s->info.dir_light_samp = need(rad, "dir_light_samp")->is_true() ? 1u : 0u;
    s->info.seed = seed;
    s->spp = (uint32_t)need(ri, "samps_per_pix")->num();
    const Node* b = ri->get("gpu_render_batch");
    s->batch = b && b->kind != Node::Null ? (uint32_t)b->num() : 0u;
    s->use_gpu = ri->get("use_gpu") && ri->get("use_gpu")->is_true() ? 1u : 0u;
    s->animation = ri->get("animation") && ri->get("animation")->is_true() ? 1u : 0u;

    const Node* cam = need(root, "cam");  // From<pr::Cam> (builder/pr/cam.rs:19-81)
    float d[3], o[3], up[3], eul[3];
    v3(need(cam, "d"), d);
    v3(need(cam, "o"), o);
    v3(need(cam, "up"), up);
    v3(need(cam, "view_eulers"), eul);
    const Node* lens = cam->get("lens_r");
    const bool has_lens = lens && lens->kind != Node::Null;
    const int st = rt_camera_from_scheme(d, o, up, f32(need(cam, "screen_width")), f32(need(cam, "screen_height")),
                                         has_lens ? 1u : 0u, has_lens ? f32(lens) : 0.0f, eul, &s->cam);
    if (st) throw std::runtime_error("camera conversion failed");

    rth::PackStore store(assets_root ? assets_root : "");
    std::map<std::string, int> tex_cache;
    const Node* members = need(root, "scene_members");
    for (size_t mi = 0; mi < members->seq.size(); ++mi) {  // inner.rs:21-64, member order
        const Node* v = nullptr;
        const std::string kind = tag_of(members->seq[mi].get(), &v);
        const MemberOverride* o = ov && mi < ov->size() ? &(*ov)[mi] : nullptr;
        if (kind == "Sphere") {
            rt_sphere sp{};
            v3(need(v, "c"), sp.c);
            if (o && o->c) std::memcpy(sp.c, o->cv, sizeof(sp.c));
            sp.r = f32(need(v, "r"));
            const Node* cv = nullptr;
            if (tag_of(need(v, "coloring"), &cv) != "Solid") throw std::runtime_error("unknown coloring");
            v3(cv, sp.rgb);
            sp.mat = material(need(v, "mat"));
            s->elems.push_back(rt_elem{RT_ELEM_SPHERE, (uint32_t)s->spheres.size()});
            s->spheres.push_back(sp);
        } else if (kind == "FreeTriangle") {
            rt_free_triangle t{};
            const Node* vs = need(v, "verts");
            for (size_t i = 0; i < 3; ++i) v3(vs->seq.at(i).get(), t.verts[i]);
            float n[3];
            v3(need(v, "norm"), n);
            const float len = sqrtf((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]);  // inner.rs:48
            for (int i = 0; i < 3; ++i) t.norm[i] = n[i] / len;
            v3(need(v, "rgb"), t.rgb);
            t.mat = material(need(v, "mat"));
            s->elems.push_back(rt_elem{RT_ELEM_FREE_TRI, (uint32_t)s->free_tris.size()});
            s->free_tris.push_back(t);
        } else if (kind == "DistantCubeMap") {
            if (!assets_root) throw std::runtime_error("DistantCubeMap needs an assets root");
            rt_cube_map cm{};
            static const char* faces[6] = {"neg_x", "pos_x", "neg_y", "pos_y", "neg_z", "pos_z"};
            for (int fi = 0; fi < 6; ++fi) {
                const Node* f = need(v, faces[fi]);
                const std::string path = f->seq.at(0)->str();
                if (!tex_cache.count(path)) {
                    rth::NpyArray img;
                    if (!store.image(path, &img)) throw std::runtime_error("cube map image not in the asset pack: " + path);
                    tex_cache[path] = add_texture(s, img);
                }
                cm.face[fi].texture = tex_cache[path];
                cm.face[fi].us = f32(f->seq.at(1).get());
                cm.face[fi].vs = f32(f->seq.at(2).get());
            }
            s->elems.push_back(rt_elem{RT_ELEM_CUBE_MAP, (uint32_t)s->cube_maps.size()});
            s->cube_maps.push_back(cm);
        } else if (kind == "Model") {
            if (!assets_root) throw std::runtime_error("Model needs an assets root");
            load_model(s, v, store, o);
        } else {
            throw std::runtime_error("unknown scene member " + kind);
        }
    }

    // the C views (every owning vector is final now)
    s->textures.clear();
    for (size_t i = 0; i < s->texels.size(); ++i)
        s->textures.push_back(rt_texture{s->tex_dims[i].first, s->tex_dims[i].second, s->texels[i].data()});
    s->desc.n_textures = (uint32_t)s->textures.size();
    s->desc.textures = s->textures.data();
    s->desc.n_elems = (uint32_t)s->elems.size();
    s->desc.elems = s->elems.data();
    s->desc.n_spheres = (uint32_t)s->spheres.size();
    s->desc.spheres = s->spheres.data();
    s->desc.n_free_tris = (uint32_t)s->free_tris.size();
    s->desc.free_tris = s->free_tris.data();
    s->desc.n_cube_maps = (uint32_t)s->cube_maps.size();
    s->desc.cube_maps = s->cube_maps.data();
    for (auto& mp : s->meshes) {
        rt_scheme::Mesh& M = *mp;
        M.abi_prims.clear();
        for (auto& P : M.prims) {
            rt_mesh_prim A = P.abi;
            A.n_verts = (uint32_t)(P.poses.size() / 3);
            A.n_tris = (uint32_t)(P.indices.size() / 3);
            A.poses = P.poses.data();
            A.norms = P.norms.data();
            A.indices = P.indices.data();
            A.tangents = P.has_tangents ? P.tangents.data() : nullptr;
            A.base_color_uv = P.base_uv.empty() ? nullptr : P.base_uv.data();
            A.normal_uv = P.normal_uv.empty() ? nullptr : P.normal_uv.data();
            A.metal_rough_uv = P.mr_uv.empty() ? nullptr : P.mr_uv.data();
            M.abi_prims.push_back(A);
        }
        M.abi.n_prims = (uint32_t)M.abi_prims.size();
        M.abi.prims = M.abi_prims.data();
        s->abi_meshes.push_back(M.abi);
    }
    s->desc.n_meshes = (uint32_t)s->abi_meshes.size();
    s->desc.meshes = s->abi_meshes.data();
}

}  // namespace

extern "C" int rt_scheme_load(const char* text, uint64_t len, uint32_t format, const char* assets_root,
                              uint64_t seed, rt_scheme** out) {
    if (!text || !out || format > RT_SCHEME_JSON) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    try {
        const std::string src(text, (size_t)len);
        const NodeP root = format == RT_SCHEME_YAML ? rth::parse_yaml(src) : rth::parse_json(src);
        std::unique_ptr<rt_scheme> s(new rt_scheme());
        build(s.get(), root.get(), assets_root, seed);
        s->root = root;
        s->has_assets = assets_root != nullptr;
        s->assets_root = assets_root ? assets_root : "";
        s->seed = seed;
        *out = s.release();
        return RT_OK;
    } catch (const std::bad_alloc&) {
        g_err = "out of host memory";
        return RT_ERR_OOM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return RT_ERR_INVALID_ARG;
    }
}

// ------------------------------------------------------------------------------ animation
// extract_anim (builder/inner.rs:113-210) over keyframe 1.1.1's AnimationSequence.  The crate
// is not vendored: its sequence and easing arithmetic are restated from its published behaviour
// (parity unpinned): keyframes sorted by time; the value at time t tweens from the last
// keyframe at or before t to the next one with the *earlier* keyframe's easing function of the
// clamped progress (t - t0) / (t1 - t0); the tween is per component in f64, from + (to - from) y,
// rounded to f32; at or past the last keyframe its value holds.  advance_by adds the frame
// period to an f64 clock clamped to [0, last keyframe time].
namespace {

double ease_y(const std::string& f, double x) {
    auto bezier = [](double x1, double y1, double x2, double y2, double x) {  // CSS cubic-bezier
        auto bx = [&](double t) { return 3 * (1 - t) * (1 - t) * t * x1 + 3 * (1 - t) * t * t * x2 + t * t * t; };
        auto by = [&](double t) { return 3 * (1 - t) * (1 - t) * t * y1 + 3 * (1 - t) * t * t * y2 + t * t * t; };
        double lo = 0.0, hi = 1.0, t = x;
        for (int i = 0; i < 64; ++i) {  // bisection to full double precision
            t = 0.5 * (lo + hi);
            if (bx(t) < x) lo = t;
            else hi = t;
        }
        return by(t);
    };
    if (f == "Linear") return x;
    if (f == "Step") return x < 0.5 ? 0.0 : 1.0;
    if (f == "Hold") return x < 1.0 ? 0.0 : 1.0;
    if (f == "EaseIn") return bezier(0.42, 0.0, 1.0, 1.0, x);
    if (f == "EaseOut") return bezier(0.0, 0.0, 0.58, 1.0, x);
    if (f == "EaseInOut") return bezier(0.42, 0.0, 0.58, 1.0, x);
    if (f == "EaseInQuad") return x * x;
    if (f == "EaseOutQuad") return -x * (x - 2.0);
    if (f == "EaseInOutQuad") return x < 0.5 ? 2.0 * x * x : -2.0 * x * x + 4.0 * x - 1.0;
    if (f == "EaseInCubic") return x * x * x;
    if (f == "EaseOutCubic") { const double y = x - 1.0; return y * y * y + 1.0; }
    if (f == "EaseInOutCubic") {
        if (x < 0.5) return 4.0 * x * x * x;
        const double y = 2.0 * x - 2.0;
        return 0.5 * y * y * y + 1.0;
    }
    if (f == "EaseInQuart") return x * x * x * x;
    if (f == "EaseOutQuart") { const double y = x - 1.0; return -(y * y * y * y - 1.0); }
    if (f == "EaseInOutQuart") {
        if (x < 0.5) return 8.0 * x * x * x * x;
        const double y = x - 1.0;
        return -8.0 * y * y * y * y + 1.0;
    }
    if (f == "EaseInQuint") return x * x * x * x * x;
    if (f == "EaseOutQuint") { const double y = x - 1.0; return y * y * y * y * y + 1.0; }
    if (f == "EaseInOutQuint") {
        if (x < 0.5) return 16.0 * x * x * x * x * x;
        const double y = x - 1.0;
        return 16.0 * y * y * y * y * y + 1.0;
    }
    throw std::runtime_error("Unsupported easing function: " + f);  // builder/mod.rs:58
}

struct Key {
    double time;
    float v[6];       // translation, euler angles
    std::string ease; // Keyframe::get_ease_type, default EaseInOut (builder/mod.rs:38)
};

struct Sequence {
    std::vector<Key> keys;
    double clock = 0.0;
    double duration() const { return keys.empty() ? 0.0 : keys.back().time; }
    void advance_by(double dt) {
        double t = clock + dt;
        clock = t < 0.0 ? 0.0 : (t > duration() ? duration() : t);
    }
    void now(int n, float* out) const {
        size_t k = 0;
        bool found = false;
        for (size_t i = 0; i < keys.size(); ++i)
            if (keys[i].time <= clock) {
                k = i;
                found = true;
            }
        if (!found) {
            for (int c = 0; c < n; ++c) out[c] = keys.front().v[c];
            return;
        }
        if (k + 1 >= keys.size()) {
            for (int c = 0; c < n; ++c) out[c] = keys[k].v[c];
            return;
        }
        const Key &a = keys[k], &b = keys[k + 1];
        double x = (clock - a.time) / (b.time - a.time);
        x = x < 0.0 ? 0.0 : (x > 1.0 ? 1.0 : x);
        const double y = ease_y(a.ease, x);
        for (int c = 0; c < n; ++c) out[c] = (float)((double)a.v[c] + ((double)b.v[c] - (double)a.v[c]) * y);
    }
};

// the member's keyframe sequence, or false when it has no animation
bool member_sequence(const Node* v, bool model, Sequence* seq) {
    const Node* anim = v->get("animation");
    if (!anim || anim->kind == Node::Null) return false;
    for (const NodeP& kf : need(anim, "keyframes")->seq) {
        Key k{};
        k.time = (double)f32(need(kf.get(), "time"));
        v3(need(kf.get(), "translation"), k.v);
        if (model) {
            const Node* e = kf->get("euler_angles");
            if (!e || e->kind == Node::Null) throw std::runtime_error("model keyframe without euler_angles");
            v3(e, k.v + 3);
        }
        const Node* et = kf->get("ease_type");
        k.ease = et && et->kind != Node::Null ? et->str() : "EaseInOut";
        (void)ease_y(k.ease, 0.0);  // unknown names fail at load, as get_ease_type panics
        for (const Key& o : seq->keys)
            if (o.time == k.time) throw std::runtime_error("two keyframes at the same time");
        seq->keys.push_back(k);
    }
    std::stable_sort(seq->keys.begin(), seq->keys.end(), [](const Key& a, const Key& b) { return a.time < b.time; });
    return true;
}

// number_of_frames and the per-member sequences (extract_anim, inner.rs:113-124)
uint32_t frame_plan(const rt_scheme* s, std::vector<std::pair<int, Sequence>>* seqs, double* tpf) {
    const Node* root = s->root.get();
    const Node* ri = need(root, "render_info");
    const Node* members = need(root, "scene_members");
    float last = 0.0f;
    bool any = false;
    for (size_t mi = 0; mi < members->seq.size(); ++mi) {
        const Node* v = nullptr;
        const std::string kind = tag_of(members->seq[mi].get(), &v);
        if (kind != "Sphere" && kind != "Model") continue;
        Sequence q;
        if (!member_sequence(v, kind == "Model", &q)) {
            any = true;
            continue;
        }
        // get_last_timestamp: the member's last keyframe in file order, reduced with f32::max
        const Node* kfs = need(v->get("animation"), "keyframes");
        const float t = f32(need(kfs->seq.back().get(), "time"));
        last = any ? std::fmax(last, t) : t;
        any = true;
        seqs->emplace_back((int)mi, std::move(q));
    }
    const Node* fr = ri->get("framerate");
    if (!fr || fr->kind == Node::Null) throw std::runtime_error("Ensure the framerate is added for use_gpu!");
    *tpf = 1.0 / (double)f32(fr);
    return (uint32_t)((double)last / *tpf);
}

}  // namespace

extern "C" int rt_scheme_frames(rt_scheme* s, uint32_t* n_frames) {
    if (!s || !n_frames) return RT_ERR_INVALID_ARG;
    *n_frames = 0;
    if (!s->animation) return RT_OK;
    try {
        std::vector<std::pair<int, Sequence>> seqs;
        double tpf;
        *n_frames = frame_plan(s, &seqs, &tpf);
        return RT_OK;
    } catch (const std::exception& e) {
        g_err = e.what();
        return RT_ERR_INVALID_ARG;
    }
}

extern "C" int rt_scheme_frame(rt_scheme* s, uint32_t frame, rt_scheme** out) {
    if (!s || !out || !s->animation) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    try {
        std::vector<std::pair<int, Sequence>> seqs;
        double tpf;
        const uint32_t n = frame_plan(s, &seqs, &tpf);
        if (frame >= n) return RT_ERR_INVALID_ARG;
        const Node* members = need(s->root.get(), "scene_members");
        std::vector<MemberOverride> ov(members->seq.size());
        for (auto& ms : seqs) {
            Sequence& q = ms.second;
            for (uint32_t i = 0; i < frame; ++i) q.advance_by(tpf);  // one advance per frame
            const Node* v = nullptr;
            const bool model = tag_of(members->seq[(size_t)ms.first].get(), &v) == "Model";
            float val[6];
            q.now(model ? 6 : 3, val);
            MemberOverride& o = ov[(size_t)ms.first];
            if (model) {
                o.trans = o.euler = true;
                std::memcpy(o.tv, val, sizeof(o.tv));
                std::memcpy(o.ev, val + 3, sizeof(o.ev));
            } else {
                o.c = true;
                std::memcpy(o.cv, val, sizeof(o.cv));
            }
        }
        std::unique_ptr<rt_scheme> f(new rt_scheme());
        build(f.get(), s->root.get(), s->has_assets ? s->assets_root.c_str() : nullptr, s->seed, &ov);
        f->info = s->info;  // the caller's overrides (size, flags) carry over
        f->root = s->root;
        f->has_assets = s->has_assets;
        f->assets_root = s->assets_root;
        f->seed = s->seed;
        f->animation = 0;   // a frame is a still scene
        *out = f.release();
        return RT_OK;
    } catch (const std::bad_alloc&) {
        g_err = "out of host memory";
        return RT_ERR_OOM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return RT_ERR_INVALID_ARG;
    }
}

extern "C" int rt_scheme_view_get(rt_scheme* s, rt_scheme_view* out) {
    if (!s || !out) return RT_ERR_INVALID_ARG;
    out->scene = &s->desc;
    out->cam = &s->cam;
    out->info = &s->info;
    out->samps_per_pix = s->spp;
    out->gpu_render_batch = s->batch;
    out->use_gpu = s->use_gpu;
    out->animation = s->animation;
    return RT_OK;
}

extern "C" const char* rt_scheme_last_error(void) { return g_err.c_str(); }

extern "C" int rt_scheme_free(rt_scheme* s) {
    if (!s) return RT_ERR_INVALID_ARG;
    delete s;
    return RT_OK;
}

// --------------------------------------------------------------------------------- PNG output
namespace {
void put32(std::vector<uint8_t>& b, uint32_t v) {
    for (int k = 3; k >= 0; --k) b.push_back((uint8_t)(v >> (8 * k)));
}
void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
    put32(out, (uint32_t)data.size());
    const size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    put32(out, (uint32_t)crc32(0L, &out[start], (uInt)(out.size() - start)));
}
}  // namespace

// process_output_routine (ui_util.rs:37-54): RGBA8 buffer -> flip_vertical -> PNG.  The image
// crate's encoder settings (filters, compression level) are not reproduced: the decoded pixels
// are the same, the file bytes are not.
extern "C" int rt_write_png(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height,
                            uint32_t flip_vertical) {
    if (!path || !rgba8 || !width || !height) return RT_ERR_INVALID_ARG;
    const size_t row = (size_t)width * 4;
    std::vector<uint8_t> raw((row + 1) * height);
    for (uint32_t y = 0; y < height; ++y) {
        const uint32_t sy = flip_vertical ? height - 1 - y : y;
        raw[y * (row + 1)] = 0;  // filter: none
        std::memcpy(&raw[y * (row + 1) + 1], rgba8 + (size_t)sy * row, row);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return RT_ERR_OOM;
    z.resize(zlen);
    std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    put32(ihdr, width);
    put32(ihdr, height);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit RGBA, deflate, no filter method, no interlace
    chunk(png, "IHDR", ihdr);
    chunk(png, "IDAT", z);
    chunk(png, "IEND", {});
    FILE* f = std::fopen(path, "wb");
    if (!f) return RT_ERR_INVALID_ARG;
    const size_t w = std::fwrite(png.data(), 1, png.size(), f);
    std::fclose(f);
    return w == png.size() ? RT_OK : RT_ERR_INVALID_ARG;
}
