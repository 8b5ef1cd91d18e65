// kd_build.cpp — host side of the boundary: KD-tree build + flattening, camera conversion,
// RGBA8 conversion.  Compiled with -ffp-contract=off so every f32 rounding step equals the
// reference's (Rust never contracts a*b+c).
//
// rt_kd_build restates KdTree::build / node_from_elems (src/accel/kdtree.rs:26-56,107-137)
// iteratively (breadth first) into the 8-byte node layout of rt_abi.h, then re-lays the nodes
// in 128-byte blocks (relayout_blocked) for cache-line locality on the device.  The split of a node is the f32 sequential mean of its elements' AABB centroids on
// the node's axis (Sum<Vector3<f32>> folds from zero in element order, kdtree.rs:113); an
// element goes high when aabb.high >= split and low when aabb.low <= split (both allowed,
// kdtree.rs:119-127); a node is a leaf when depth > max_depth or it holds <= 1 element.
#include "host_internal.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <new>
#include <thread>
#include <vector>

namespace rth {

static inline float rmin(float a, float b) { return std::fmin(a, b); }  // Rust f32::min
static inline float rmax(float a, float b) { return std::fmax(a, b); }  // Rust f32::max

int gather_renderables(const rt_scene_desc* sc, std::vector<Renderable>* out) {
    if (!sc) return RT_ERR_INVALID_ARG;
    out->clear();
    for (uint32_t i = 0; i < sc->n_elems; ++i) {
        const rt_elem& e = sc->elems[i];
        Renderable r{};
        r.kind = e.kind;
        r.index = e.index;
        switch (e.kind) {
            case RT_ELEM_SPHERE: {  // Sphere::give_aabb (sphere.rs:106-114)
                if (e.index >= sc->n_spheres) return RT_ERR_INVALID_ARG;
                const rt_sphere& s = sc->spheres[e.index];
                r.has_aabb = true;
                for (int a = 0; a < 3; ++a) { r.lo[a] = s.c[a] - s.r; r.hi[a] = s.c[a] + s.r; }
                break;
            }
            case RT_ELEM_FREE_TRI: {  // Triangle::give_aabb (generic.rs:138-156)
                if (e.index >= sc->n_free_tris) return RT_ERR_INVALID_ARG;
                const rt_free_triangle& t = sc->free_tris[e.index];
                r.has_aabb = true;
                for (int a = 0; a < 3; ++a) {
                    r.lo[a] = rmin(rmin(t.verts[0][a], t.verts[1][a]), t.verts[2][a]);
                    r.hi[a] = rmax(rmax(t.verts[0][a], t.verts[1][a]), t.verts[2][a]);
                }
                break;
            }
            case RT_ELEM_CUBE_MAP:  // DistantCubeMap::give_aabb -> None
                if (e.index >= sc->n_cube_maps) return RT_ERR_INVALID_ARG;
                r.has_aabb = false;
                break;
            default:
                return RT_ERR_INVALID_ARG;
        }
        out->push_back(r);
    }
    uint32_t mesh_tri = 0;
    for (uint32_t m = 0; m < sc->n_meshes; ++m) {
        const rt_mesh& mesh = sc->meshes[m];
        for (uint32_t p = 0; p < mesh.n_prims; ++p) {
            const rt_mesh_prim& pr = mesh.prims[p];
            for (uint32_t t = 0; t < pr.n_tris; ++t) {
                Renderable r{};
                r.kind = RT_KIND_MESH_TRI;
                r.index = mesh_tri++;
                r.has_aabb = true;
                for (int a = 0; a < 3; ++a) {
                    float v0 = pr.poses[3 * (size_t)pr.indices[3 * (size_t)t + 0] + a];
                    float v1 = pr.poses[3 * (size_t)pr.indices[3 * (size_t)t + 1] + a];
                    float v2 = pr.poses[3 * (size_t)pr.indices[3 * (size_t)t + 2] + a];
                    r.lo[a] = rmin(rmin(v0, v1), v2);
                    r.hi[a] = rmax(rmax(v0, v1), v2);
                }
                out->push_back(r);
            }
        }
    }
    return RT_OK;
}

}  // namespace rth

using namespace rth;

// Re-lays a BFS-built tree into 128-byte blocks of 16 nodes: block 0 holds the root and the
// next three levels (1 + 2 + 4 + 8 nodes); every other block holds one sibling pair and the
// two levels below it (2 + 4 + 8).  Children stay adjacent (low, low + 1), so the node format
// is unchanged; a descent touches one cache line per 3 levels instead of one per level.
static std::vector<rt_kd_node> relayout_blocked(const std::vector<rt_kd_node>& in) {
    std::vector<rt_kd_node> out;
    if (in.empty()) return out;
    std::vector<uint32_t> new_of(in.size(), UINT32_MAX);
    struct Pending { uint32_t old_first; uint32_t count; uint32_t parent_new; };  // count 1 (root) or 2
    std::deque<Pending> q;
    q.push_back(Pending{0, 1, UINT32_MAX});
    auto is_leaf = [&](uint32_t i) { return (in[i].b & 3u) == RT_KD_LEAF; };
    while (!q.empty()) {
        Pending pb = q.front();
        q.pop_front();
        const uint32_t base = (uint32_t)out.size();
        out.resize(base + 16, rt_kd_node{0, RT_KD_LEAF});  // padding slots: empty leaves, never referenced
        const int levels = pb.count == 1 ? 4 : 3;
        std::vector<uint32_t> level;
        for (uint32_t k = 0; k < pb.count; ++k) level.push_back(pb.old_first + k);
        uint32_t slot = base;
        std::vector<uint32_t> block_nodes;
        for (int l = 0; l < levels && !level.empty(); ++l) {
            std::vector<uint32_t> next;
            for (uint32_t o : level) {
                new_of[o] = slot++;
                block_nodes.push_back(o);
            }
            if (l + 1 < levels)
                for (uint32_t o : level)
                    if (!is_leaf(o)) { next.push_back(in[o].b >> 2); next.push_back((in[o].b >> 2) + 1); }
            level.swap(next);
        }
        if (pb.parent_new != UINT32_MAX)
            out[pb.parent_new].b = (base << 2) | (out[pb.parent_new].b & 3u);
        for (uint32_t o : block_nodes) {
            const uint32_t nw = new_of[o];
            out[nw] = in[o];
            if (is_leaf(o)) continue;
            const uint32_t low = in[o].b >> 2;
            if (new_of[low] != UINT32_MAX) {  // children inside this block
                out[nw].b = (new_of[low] << 2) | (in[o].b & 3u);
            } else {  // children start a new block; the pointer is patched when it is emitted
                q.push_back(Pending{low, 2, nw});
            }
        }
    }
    return out;
}

struct KdTreeOwned {
    rt_kd_tree pub;
    std::vector<rt_kd_node> nodes;
    std::vector<uint32_t> refs;
    std::vector<uint32_t> uncond;
};

// One node of a subtree built on its own (local indices): a branch {split, axis, low child}, or
// a leaf {its refs in the subtree's ref list}; `ext` >= 0 marks a frontier node of the top part
// whose subtree was built separately.
struct SubNode {
    uint32_t a = 0;          // split bits (branch) or ref count (leaf)
    uint32_t axis = 0;       // RT_KD_LEAF for a leaf
    uint32_t low = 0;        // low child (local), branch only
    uint32_t ref_off = 0;    // leaf only
    int32_t ext = -1;        // frontier: index of the separately built subtree
};
struct SubTree {
    std::vector<SubNode> nodes;
    std::vector<uint32_t> refs;
    uint32_t max_leaf_depth = 0;
};
struct Frontier {
    uint32_t depth;
    std::vector<uint32_t> elems;
};

// node_from_elems (kdtree.rs:107-137), breadth first, from (elems, depth0).  Items reaching
// depth `stop` (when frontier != nullptr) are not expanded: they become frontier nodes, built
// later as subtrees of their own.  The node order within the subtree is the breadth-first order
// of the whole build restricted to it, so merging (merge_bfs) reproduces the sequential numbering.
// Limits of the flat layout: node and ref indices fit 30 bits (rt_kd_node.b holds index << 2), and
// a level's concatenated element lists are indexed by uint32.  `budget` counts the nodes and refs
// of the whole build (all threads): past 2^30 of either the build stops with RT_ERR_OOM instead of
// growing to the end (a tree whose elements straddle every split copies them at every level).
// RT_DEBUG_KD_BUDGET lowers the limit (tests/test_kd.py reaches it on a small scene).
struct BuildBudget {
    std::atomic<uint64_t> nodes{0}, refs{0};
    std::atomic<bool> over{false};
    uint64_t limit = 1ull << 30;
    BuildBudget() {
        if (const char* e = std::getenv("RT_DEBUG_KD_BUDGET")) {
            const unsigned long long v = std::strtoull(e, nullptr, 10);
            if (v > 0 && v < limit) limit = v;
        }
    }
    bool charge(uint64_t n, uint64_t r) {
        if (over.load(std::memory_order_relaxed)) return false;
        if (nodes.fetch_add(n) + n >= limit || refs.fetch_add(r) + r >= limit) over = true;
        return !over.load(std::memory_order_relaxed);
    }
};
static int build_subtree(const std::vector<Renderable>& rs, const std::vector<float>& cen, std::vector<uint32_t> elems,
                         uint32_t depth0, uint32_t max_depth, uint32_t stop, SubTree* out,
                         std::vector<Frontier>* frontier, BuildBudget* budget) {
    // Level by level: a level's element lists concatenated in one array (no per-node vectors),
    // its items in breadth-first order; the children of level L are level L + 1, in order.
    struct Item { uint32_t node; uint32_t begin, end; };
    std::vector<uint32_t> cur = std::move(elems), nxt;
    std::vector<Item> items{Item{0, 0, (uint32_t)cur.size()}}, nitems;
    out->nodes.emplace_back();
    for (uint32_t depth = depth0; !items.empty(); ++depth) {
        nxt.clear();
        nitems.clear();
        // the level's nodes and refs are charged to the shared budget once, at its end
        uint64_t lvl_nodes = 0, lvl_refs = 0;
        const uint32_t axis = depth % 3;
        for (const Item& it : items) {
            SubNode& nd = out->nodes[it.node];
            const uint32_t n = it.end - it.begin;
            if (frontier && depth == stop) {
                nd.ext = (int32_t)frontier->size();
                frontier->push_back(Frontier{depth, std::vector<uint32_t>(cur.begin() + it.begin, cur.begin() + it.end)});
                continue;
            }
            if (depth > max_depth || n <= 1) {
                nd.a = n;
                nd.axis = RT_KD_LEAF;
                nd.ref_off = (uint32_t)out->refs.size();
                lvl_refs += n;
                out->refs.insert(out->refs.end(), cur.begin() + it.begin, cur.begin() + it.end);
                if (depth > out->max_leaf_depth) out->max_leaf_depth = depth;
                continue;
            }
            float sum = 0.0f;  // centroid component on `axis`, folded in element order (kdtree.rs:113)
            for (uint32_t k = it.begin; k < it.end; ++k) sum = sum + cen[3 * (size_t)cur[k] + axis];
            const float split = sum / (float)n;
            const uint32_t child = (uint32_t)out->nodes.size();
            std::memcpy(&nd.a, &split, 4);
            nd.axis = axis;
            nd.low = child;
            const uint32_t lb = (uint32_t)nxt.size();
            for (uint32_t k = it.begin; k < it.end; ++k)
                if (rs[cur[k]].lo[axis] <= split) nxt.push_back(cur[k]);
            const uint32_t hb = (uint32_t)nxt.size();
            for (uint32_t k = it.begin; k < it.end; ++k)
                if (rs[cur[k]].hi[axis] >= split) nxt.push_back(cur[k]);
            if (nxt.size() >= (1ull << 32)) return RT_ERR_OOM;
            lvl_nodes += 2;
            nitems.push_back(Item{child, lb, hb});
            nitems.push_back(Item{child + 1, hb, (uint32_t)nxt.size()});
            out->nodes.emplace_back();
            out->nodes.emplace_back();
        }
        if (!budget->charge(lvl_nodes, lvl_refs)) return RT_ERR_OOM;
        cur.swap(nxt);
        items.swap(nitems);
    }
    return RT_OK;
}

// The whole tree in the sequential build's breadth-first numbering: a node's index is its
// position in the breadth-first order, children appended as their parent is processed, and leaf
// refs appended as each leaf is processed.
static int merge_bfs(const SubTree& top, const std::vector<SubTree>& subs, KdTreeOwned* kt) {
    struct Ref { uint32_t tree; uint32_t node; };  // tree UINT32_MAX: the top part
    auto resolve = [&](Ref r) {
        if (r.tree == UINT32_MAX && top.nodes[r.node].ext >= 0) return Ref{(uint32_t)top.nodes[r.node].ext, 0u};
        return r;
    };
    auto node_of = [&](Ref r) -> const SubNode& { return r.tree == UINT32_MAX ? top.nodes[r.node] : subs[r.tree].nodes[r.node]; };
    auto refs_of = [&](Ref r) -> const std::vector<uint32_t>& { return r.tree == UINT32_MAX ? top.refs : subs[r.tree].refs; };
    size_t total = top.nodes.size();
    for (const SubTree& t : subs) total += t.nodes.size() - 1;
    if (total >= (1u << 30)) return RT_ERR_OOM;
    kt->nodes.assign(total, rt_kd_node{0, 0});
    std::vector<Ref> order;  // breadth-first: order[i] is global node i
    order.reserve(total);
    order.push_back(resolve(Ref{UINT32_MAX, 0}));
    for (size_t i = 0; i < order.size(); ++i) {
        const SubNode& nd = node_of(order[i]);
        if (nd.axis == RT_KD_LEAF) {
            const std::vector<uint32_t>& rf = refs_of(order[i]);
            if (kt->refs.size() + nd.a >= (1u << 30)) return RT_ERR_OOM;
            kt->nodes[i].a = nd.a;
            kt->nodes[i].b = ((uint32_t)kt->refs.size() << 2) | RT_KD_LEAF;
            kt->refs.insert(kt->refs.end(), rf.begin() + nd.ref_off, rf.begin() + nd.ref_off + nd.a);
            continue;
        }
        const uint32_t child = (uint32_t)order.size();
        kt->nodes[i].a = nd.a;
        kt->nodes[i].b = (child << 2) | nd.axis;
        order.push_back(resolve(Ref{order[i].tree, nd.low}));
        order.push_back(resolve(Ref{order[i].tree, nd.low + 1}));
    }
    return order.size() == total ? RT_OK : RT_ERR_INVALID_ARG;
}

extern "C" int rt_kd_build(const rt_scene_desc* scene, uint32_t max_depth, rt_kd_tree** out) {
    if (!scene || !out) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    std::vector<Renderable> rs;
    int st = gather_renderables(scene, &rs);
    if (st) return st;
    KdTreeOwned* kt = new (std::nothrow) KdTreeOwned();
    if (!kt) return RT_ERR_OOM;
    std::memset(&kt->pub, 0, sizeof(kt->pub));

    // elems_and_aabbs / unconditional split (draw_scene.rs:60-68)
    std::vector<uint32_t> root;
    for (uint32_t i = 0; i < rs.size(); ++i) {
        if (rs[i].has_aabb) root.push_back(i);
        else kt->uncond.push_back(i);
    }
    uint32_t max_leaf_depth = 0;
    if (!root.empty()) {
        // root Aabb: per-axis reduce with f32::min / f32::max (kdtree.rs:29-49)
        for (int a = 0; a < 3; ++a) {
            float lo = rs[root[0]].lo[a], hi = rs[root[0]].hi[a];
            for (size_t k = 1; k < root.size(); ++k) {
                lo = rmin(lo, rs[root[k]].lo[a]);
                hi = rmax(hi, rs[root[k]].hi[a]);
            }
            kt->pub.bounds[2 * a] = lo;
            kt->pub.bounds[2 * a + 1] = hi;
        }
        // each element's Aabb centroid 0.5 * (lo + hi) per axis (Aabb::centroid, the value
        // kdtree.rs:113 sums), computed once with the same f32 operations
        std::vector<float> cen(3 * rs.size());
        for (size_t e = 0; e < rs.size(); ++e)
            for (int a = 0; a < 3; ++a) cen[3 * e + a] = 0.5f * (rs[e].lo[a] + rs[e].hi[a]);
        // The top STOP levels are built here; the subtrees below them, independent of each other,
        // on a few threads (RT_DEBUG_KD_THREADS, default up to 8; 1: all on this thread).  The merge
        // renumbers everything breadth first, so the tree is byte-identical either way.
        unsigned n_thr = std::min(8u, std::max(1u, std::thread::hardware_concurrency()));
        if (const char* e = std::getenv("RT_DEBUG_KD_THREADS")) n_thr = (unsigned)std::max(1, std::atoi(e));
        if (root.size() < 4096) n_thr = 1;
        const uint32_t STOP = n_thr > 1 ? 4u : UINT32_MAX;
        // Nothing throws across the ABI: an allocation failure inside a worker (std::bad_alloc,
        // std::length_error) or a thread that cannot start becomes RT_ERR_OOM / fewer threads.
        BuildBudget budget;
        std::atomic<int> status{RT_OK};
        try {
            SubTree top;
            std::vector<Frontier> frontier;
            st = build_subtree(rs, cen, std::move(root), 0, max_depth, STOP, &top, n_thr > 1 ? &frontier : nullptr,
                               &budget);
            if (st) { delete kt; return st; }
            std::vector<SubTree> subs(frontier.size());
            std::atomic<uint32_t> next{0};
            auto work = [&]() {
                try {
                    for (uint32_t k; status.load() == RT_OK && (k = next.fetch_add(1)) < frontier.size();) {
                        const int r = build_subtree(rs, cen, std::move(frontier[k].elems), frontier[k].depth, max_depth,
                                                    0, &subs[k], nullptr, &budget);
                        if (r) status = r;
                    }
                } catch (...) {
                    status = RT_ERR_OOM;
                }
            };
            std::vector<std::thread> pool;
            for (unsigned t = 1; t < n_thr && t < frontier.size(); ++t) {
                try {
                    pool.emplace_back(work);
                } catch (...) {
                    break;  // run with the threads that started (the caller's thread always works)
                }
            }
            work();
            for (auto& th : pool) th.join();
            if ((st = status.load())) { delete kt; return st; }
            max_leaf_depth = top.max_leaf_depth;
            for (const SubTree& t : subs) max_leaf_depth = std::max(max_leaf_depth, t.max_leaf_depth);
            st = merge_bfs(top, subs, kt);
        } catch (...) {
            st = RT_ERR_OOM;
        }
        if (st) { delete kt; return st; }
    }
    try {
        kt->nodes = relayout_blocked(kt->nodes);
    } catch (...) {
        delete kt;
        return RT_ERR_OOM;
    }
    if (kt->nodes.size() >= (1u << 30)) { delete kt; return RT_ERR_OOM; }
    kt->pub.n_nodes = (uint32_t)kt->nodes.size();
    kt->pub.n_refs = (uint32_t)kt->refs.size();
    kt->pub.max_leaf_depth = max_leaf_depth;
    kt->pub.n_unconditional = (uint32_t)kt->uncond.size();
    kt->pub.nodes = kt->nodes.data();
    kt->pub.refs = kt->refs.data();
    kt->pub.unconditional = kt->uncond.data();
    *out = &kt->pub;
    return RT_OK;
}

extern "C" void rt_kd_free(rt_kd_tree* tree) {
    if (!tree) return;
    // pub is the first member of KdTreeOwned
    delete reinterpret_cast<KdTreeOwned*>(tree);
}

// From<pr::Cam> for scene::Cam (src/builder/pr/cam.rs:19-81) after apply_corrections
// (src/builder/mod.rs:69-72).  Rotation3::from_euler_angles(roll, pitch, yaw) = Rz(yaw)
// Ry(pitch) Rx(roll) in nalgebra's row-major constructor order; R*v via gemv column order.
extern "C" int rt_camera_from_scheme(const float d[3], const float o[3], const float up[3],
                                     float screen_width, float screen_height, uint32_t has_lens,
                                     float lens_r, const float view_eulers[3], rt_camera* out) {
    if (!d || !o || !up || !view_eulers || !out) return RT_ERR_INVALID_ARG;
    float n = std::sqrt((up[0] * up[0] + up[1] * up[1]) + up[2] * up[2]);
    float u[3] = {up[0] / n, up[1] / n, up[2] / n};
    float sr = std::sin(view_eulers[0]), cr = std::cos(view_eulers[0]);
    float sp = std::sin(view_eulers[1]), cp = std::cos(view_eulers[1]);
    float sy = std::sin(view_eulers[2]), cy = std::cos(view_eulers[2]);
    float R[3][3] = {
        {cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr},
        {sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr},
        {-sp, cp * sr, cp * cr},
    };
    for (int i = 0; i < 3; ++i) {
        out->d[i] = (R[i][0] * d[0] + R[i][1] * d[1]) + R[i][2] * d[2];
        out->up[i] = (R[i][0] * u[0] + R[i][1] * u[1]) + R[i][2] * u[2];
        out->o[i] = o[i];
    }
    out->screen_width = screen_width;
    out->screen_height = screen_height;
    out->has_lens = has_lens ? 1u : 0u;
    out->lens_r = lens_r;
    return RT_OK;
}

// rgb_f_to_u8 (draw_scene.rs:104-108): (f.clamp(0,1) * 255 + 0.5).trunc() as u8; `as u8`
// saturates and maps NaN to 0; alpha 255 (draw_scene.rs:93).
extern "C" int rt_rgba_to_u8(const float* rgba, uint64_t n_pixels, uint8_t* out) {
    if ((!rgba || !out) && n_pixels) return RT_ERR_INVALID_ARG;
    for (uint64_t p = 0; p < n_pixels; ++p) {
        for (int c = 0; c < 3; ++c) {
            float f = rgba[4 * p + c];
            if (f < 0.0f) f = 0.0f;
            if (f > 1.0f) f = 1.0f;
            float g = std::trunc(f * 255.0f + 0.5f);
            out[4 * p + c] = std::isnan(g) ? 0 : (g >= 255.0f ? 255 : (uint8_t)g);
        }
        out[4 * p + 3] = 255;
    }
    return RT_OK;
}

extern "C" int rt_abi_version(void) { return RT_ABI_VERSION; }

extern "C" const char* rt_status_string(int s) {
    switch (s) {
        case RT_OK: return "ok";
        case RT_ERR_INVALID_ARG: return "invalid argument";
        case RT_ERR_OOM: return "out of memory";
        case RT_ERR_HIP: return "HIP runtime error";
        case RT_ERR_UNSUPPORTED: return "unsupported on the device path";
        case RT_ERR_NO_DEVICE: return "no such gfx950 device";
        case RT_ERR_BATCH: return "samps_per_pix is not divisible by gpu_render_batch";
        default: return "unknown status";
    }
}
