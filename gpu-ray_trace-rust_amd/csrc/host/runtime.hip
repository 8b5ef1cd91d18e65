// runtime.hip — host runtime behind the C ABI: device pick, scene flattening and upload,
// launches, events, errors.  Replaces GPUState / ComputePipeline
// (src/render/gpu_utils.rs:257-724) and the batch loop of render_to_target_gpu
// (src/render/draw_scene.rs:17-47).  Host float work here (RayCompute) is compiled with
// -ffp-contract=off, like the oracle.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../../include/rt_abi.h"
#include "../../../include/rt_rng.h"
#include "../kernel/device_scene.h"
#include "host_internal.h"
#include "mesh_flatten.h"

using namespace rtd;
using namespace rth;

// Radiance buffer cap per queue launch (floats): 16 GiB of 288 GB HBM, so a 1000-spp step of a
// 1200x600 frame (8.6 GB) is one launch.  Every launch ends in a drain tail (lanes idle while the
// last paths finish): walled's bench step ran 3.4% faster as one launch than as three of 334 spp
// (4 GiB cap).  RT_DEBUG_LAUNCH radiance_gib overrides it; only what a launch needs is allocated.
static constexpr uint64_t QUEUE_RADIANCE_FLOATS = 1ull << 32;

// Overlapped queue launches rotate over pipeline slots, each with its own stream, radiance
// buffer, item counter and traversal-stack scratch: launch i + 1 starts while launch i drains
// (its last paths finish on a few lanes), and only the folds, which update the shared
// accumulators and the output, are chained in order by events.  A mesh launch's drain tail is
// ~8-10 ms; a 1-spp a380 launch holds ~2 ms of work, so small launches (up to 2^21 samples) need
// many of them in flight to cover one tail, larger ones fewer (mid_slots_for; round 2, biplane at
// 10 spp: 590 / 587 / 569 with 2 / 3 / 4).  The slots' streams overlap only on separate hardware queues: HIP maps
// streams onto GPU_MAX_HW_QUEUES queues (4 by default) as they are created, and streams sharing
// a queue run in order (a380 at 1 spp: 4 queues 187 Msamples/s whatever the slots; 8 queues with
// 2 / 4 / 6 slots 137 / 229 / 272; 12 queues, 8 slots 288-356).  So a context creates a slot's
// stream on first use, and small launches use slots_for_queues(GPU_MAX_HW_QUEUES) slots: four
// queues are left to the caller's streams (torch's, RCCL's), at most 12 slots (16 queues:
// 12 slots; with 32 queues and 24 slots a380 fell to 183, the queues oversubscribed).
// While the pipeline is busy, a small launch also takes only 1/grid_div of the resident grid
// (small_grid_div): its waves then trace several items per lane, so the drain of each wave's
// last paths, which holds its slot on the CU, is spread over more work, and more launches run
// side by side.  a380 at 1 spp, 16 queues (round 3, tools/gpu_a380_calib.py): 8 slots, full grid
// 356; 8 slots, 1/4 grid 370 (1/6: 350, 1/8: 318); 12 slots, 1/6 389, 1/8 400, 1/10 380;
// biplane / spaceship launches (2 slots) lose with a smaller grid (1/2: -14% / -2%), so they keep
// the full one.  The first launch of an idle pipeline (and every synchronous call) keeps the full
// grid too.  RT_DEBUG_LAUNCH slots (2-32) and grid_div (1-64) override.
constexpr int N_SLOTS = 32;          // slots a context holds (RT_DEBUG_LAUNCH slots up to this)
// A launch's item counters: one 128-B line per shard of its items (trace.hip RT_QSHARDS, <= 32)
constexpr size_t QUEUE_BYTES = 32 * 128;
static uint32_t slots_for_queues(int hw_queues) {
    const int s = hw_queues - 4;
    return s < 2 ? 2u : (s > 12 ? 12u : (uint32_t)s);
}
static uint32_t small_grid_div(uint32_t slots) { return slots >= 12 ? 8u : (slots >= 8 ? 4u : 1u); }
// Mid-size overlapped launches (2^21 .. 2^23 samples): half the small-launch slots, at most 6 (round
// 4: a380's 10-batch launches of 7.2 M samples, 16 queues: 2 / 4 / 6 / 8 slots 400 / 421 / 426 /
// 426 Msamples/s; at 4 queues 2 slots stay, where 4 ran -8.5%).  Larger ones keep 2 (biplane's
// 14.4 M-sample launches: 6 slots -1.1%).
static uint32_t mid_slots_for(uint32_t small_slots) { return std::max(2u, std::min(6u, small_slots / 2)); }
constexpr uint64_t MID_LAUNCH_ITEMS = 1ull << 23;
constexpr uint64_t SMALL_LAUNCH_ITEMS = 1ull << 21;  // default of rt_ctx::small_items
struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t fold_done = nullptr;   // this slot's last fold (its radiance buffer is free again)
    float* radiance = nullptr;
    uint64_t radiance_cap = 0;        // floats
    uint32_t* queue = nullptr;        // queue schedule item counter
    uint32_t* gstack = nullptr;       // sphere-only queue kernel's traversal stacks (queue_gstack_bytes)
    size_t gstack_cap = 0;
};

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;     // = slot[0].stream: uploads, synchronous paths
    Slot slot[N_SLOTS];
    uint32_t cur_slot = 0;            // the slot of the last enqueued launch
    hipEvent_t last_fold = nullptr;   // the most recent fold enqueued (nullptr: none pending)
    hipEvent_t caller_ev = nullptr;   // the caller's stream, recorded at an async call
    // Timing window: every trace launch since the window opened, as start / stop event pairs,
    // and the whole window from its first launch to its last fold (closed by rt_synchronize
    // or at the end of a synchronous call).
    // Per-launch events are kept for the first MAX_TIMED_LAUNCHES launches of a window only, so
    // a caller that never calls rt_synchronize (it syncs through its own stream) does not grow
    // the pool without bound; later launches are counted but not timed.
    std::vector<hipEvent_t> lev;
    uint32_t n_launch = 0;            // trace launches in the window
    uint32_t n_timed = 0;             // ... of which timed (lev[2i], lev[2i + 1])
    hipEvent_t win_end = nullptr;     // the window's last event (win_end_ev or a launch stop)
    hipEvent_t win_end_ev = nullptr;
    bool pending = false;             // enqueued work not yet synchronised
    float trace_ms = 0.f;
    DevScene sc{};
    std::vector<void*> allocs;
    float4* accum = nullptr;
    float4* accum_range = nullptr;    // rt_render_range's per-call mean (allocated on first use)
    DevTile* d_tiles = nullptr;
    uint32_t d_tiles_cap = 0;
    uint32_t* d_pixmap = nullptr;     // launch pixel -> (y << 16 | x), multi-tile launches
    uint4* d_pixq = nullptr;          // queue order of the launch pixels (LaunchArgs::pix_q)
    uint32_t pix_block = 1;           // RT_DEBUG_PIX_BLOCK: the queue order's blocks are pix_block x pix_block
    uint64_t d_pixmap_cap = 0;
    std::vector<DevTile> pixmap_tiles;  // the tiles d_pixmap was built for
    float4* d_out = nullptr;
    uint64_t d_out_cap = 0;
    DevCounts* d_counts = nullptr;
    uint64_t lane_capacity = 0;   // lanes resident at the kernel's occupancy
    uint32_t n_cu = 0;
    uint32_t forced_k = 0;        // RT_DEBUG_SCHED=direct:K (tests / tuning)
    int sched = 0;                // RT_DEBUG_SCHED: 0 auto, 1 direct, 2 queue
    uint64_t queue_floats = 0;    // radiance buffer cap per queue launch (RT_DEBUG_LAUNCH radiance_gib / radiance_floats)
    bool overlap = true;          // launch i + 1 may start during launch i's drain (RT_DEBUG_LAUNCH overlap)
    uint64_t overlap_max_items = 1ull << 27;  // ... when it has at most this many samples
    uint32_t n_slots = 0;         // RT_DEBUG_LAUNCH slots: slots the overlapped launches rotate over (0: by size)
    uint32_t small_slots = 8;     // slots of small overlapped launches (slots_for_queues)
    uint32_t mid_slots = 2;       // slots of larger overlapped launches (mid_slots_for)
    uint32_t small_div = 0;       // grid share of a small launch behind a busy pipeline (0: small_grid_div)
    uint64_t small_items = SMALL_LAUNCH_ITEMS;  // RT_DEBUG_LAUNCH small_items: launches this size or less are small
    uint32_t grid_div = 0;        // RT_DEBUG_LAUNCH grid_div; 0: small_grid_div(the launch's slots)
    uint32_t queue_shards = 1;    // item counters per queue launch (queue_shards; RT_DEBUG_LAUNCH shards)
    uint64_t group_items = 0;     // rt_render_to_target: samples per batch group (RT_DEBUG_LAUNCH group_items; 0: GROUP_ITEMS)
    float last_ms = 0.f;
    std::string err;
};

#define HIPCHK(ctx, call)                                                          \
    do {                                                                           \
        hipError_t e_ = (call);                                                    \
        if (e_ != hipSuccess) {                                                    \
            if (ctx) (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_); \
            return RT_ERR_HIP;                                                     \
        }                                                                          \
    } while (0)

static int set_err(rt_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

// Nothing throws across the C ABI: a host allocation failure (std::bad_alloc from a vector of the
// scene's size) or a thread that cannot start becomes a status code.
template <class F>
static int guarded(rt_ctx* c, F f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return set_err(c, RT_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return set_err(c, RT_ERR_OOM, std::string("host runtime: ") + e.what());
    }
}

constexpr uint32_t RT_PIX_BLOCK = 8;  // queue order of a launch's pixels: B x B blocks of each tile (1: row order)

// A/B and test knobs of the runtime, all named RT_DEBUG_<name> (INTEGRATION.md lists them), read
// here; the host KD build reads its own two, RT_DEBUG_KD_THREADS and RT_DEBUG_KD_BUDGET
// (kd_build.cpp).  A caller needs none of them: each selects an alternative schedule or layout that
// the GPU tests check bit-invariant against the oracle.  The one other variable the library reads
// is HIP's own GPU_MAX_HW_QUEUES (the hardware queues the launch pipeline can use).
static const char* debug_env(const char* name) {
    char key[64];
    std::snprintf(key, sizeof key, "RT_DEBUG_%s", name);
    return std::getenv(key);
}

template <class T>
static int upload(rt_ctx* c, const std::vector<T>& v, const T** out) {
    *out = nullptr;
    if (v.empty()) return RT_OK;
    void* p = nullptr;
    // 64 zero bytes past the end: the packet traversal's scalar loads read refs eight at a time
    constexpr size_t PAD = 64;
    if (hipMalloc(&p, v.size() * sizeof(T) + PAD) != hipSuccess) return set_err(c, RT_ERR_OOM, "hipMalloc failed");
    c->allocs.push_back(p);
    HIPCHK(c, hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemset(static_cast<char*>(p) + v.size() * sizeof(T), 0, PAD));
    *out = static_cast<const T*>(p);
    return RT_OK;
}

static bool is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

extern "C" int rt_device_count(int* n) {
    if (!n) return RT_ERR_INVALID_ARG;
    *n = 0;
    int total = 0;
    if (hipGetDeviceCount(&total) != hipSuccess) return RT_OK;
    for (int d = 0; d < total; ++d) *n += is_gfx950(d) ? 1 : 0;
    return RT_OK;
}

static DevMat make_mat(const rt_material& m, const float rgb[3]) {
    DevMat d{};
    for (int i = 0; i < 3; ++i) {
        d.rgb[i] = rgb[i];
        d.em[i] = m.has_emissive ? m.emissive[i] : 0.0f;
    }
    d.divert = m.divert;
    d.diffp = m.diffp;
    d.n_out = m.n_out;
    d.n_in = m.n_in;
    d.over_in = m.n_out / m.n_in;
    d.over_out = m.n_in / m.n_out;
    const float q = (m.n_out - m.n_in) / (m.n_out + m.n_in);
    d.r0 = q * q;
    for (int i = 0; i < 3; ++i) d.rgb_atten[i] = d.rgb[i] / 0.4f;  // RR_THRES
    return d;
}

// Every texel channel of every texture as an 8-bit k with (float)k / 255.0f == the channel, bit
// for bit (the value image::to_rgb32f makes of an 8-bit image), packed as RGBA8 words in pool
// order; false at the first channel that is not (NaN, -0, values off the k / 255 grid).  Split
// over a few threads: a380's 44 M texels take ~20 ms.
static bool pack_texels_u8(const rt_scene_desc* scene, const std::vector<DevTex>& texs, uint64_t texel_count,
                           std::vector<uint32_t>* out) {
    uint32_t lut[256];
    for (uint32_t k = 0; k < 256; ++k) {
        const float f = (float)k / 255.0f;
        std::memcpy(&lut[k], &f, 4);
    }
    out->assign(texel_count, 0u);
    std::atomic<bool> ok{true};
    auto work = [&](uint32_t t0, uint32_t t1, uint64_t p0, uint64_t p1) {
        for (uint32_t i = t0; i < t1 && ok.load(std::memory_order_relaxed); ++i) {
            const rt_texture& tx = scene->textures[i];
            const uint64_t n = (uint64_t)tx.width * tx.height;
            const uint64_t b = i == t0 ? p0 : 0, e = i + 1 == t1 && p1 ? p1 : n;
            uint32_t* dst = out->data() + texs[i].off;
            for (uint64_t q = b; q < e; ++q) {
                uint32_t w = 0;
                for (int ch = 0; ch < 3; ++ch) {
                    const float v = tx.rgb[3 * q + (uint64_t)ch];
                    const float s = v * 255.0f + 0.5f;  // k for v = k / 255 (NaN / negative fail below)
                    if (!(s >= 0.0f && s < 256.0f)) { ok = false; return; }
                    const uint32_t k = (uint32_t)s;
                    uint32_t bits;
                    std::memcpy(&bits, &v, 4);
                    if (bits != lut[k]) { ok = false; return; }
                    w |= k << (8 * ch);
                }
                dst[q] = w;
            }
        }
    };
    // split the pool into ~equal texel ranges: (texture, first texel) .. (texture, end texel)
    const unsigned n_thr = std::max(1u, std::min(8u, (unsigned)(texel_count >> 20)));
    std::vector<std::thread> pool;
    uint64_t per = (texel_count + n_thr - 1) / n_thr;
    uint32_t ti = 0;
    uint64_t at = 0;  // texels before texture ti
    for (unsigned k = 0; k < n_thr; ++k) {
        const uint64_t g0 = k * per, g1 = std::min<uint64_t>(texel_count, g0 + per);
        if (g0 >= g1) break;
        while (ti < scene->n_textures && at + (uint64_t)scene->textures[ti].width * scene->textures[ti].height <= g0) {
            at += (uint64_t)scene->textures[ti].width * scene->textures[ti].height;
            ++ti;
        }
        // [g0, g1) in pool order: from texture ti at g0 - at to the texture holding g1 - 1
        uint32_t tj = ti;
        uint64_t at2 = at;
        while (at2 + (uint64_t)scene->textures[tj].width * scene->textures[tj].height < g1) {
            at2 += (uint64_t)scene->textures[tj].width * scene->textures[tj].height;
            ++tj;
        }
        pool.emplace_back(work, ti, tj + 1, g0 - at, g1 - at2);
    }
    for (auto& th : pool) th.join();
    return ok.load();
}

// Item counters of a queue launch (trace.hip qgrab).  Each grab is one device-scope atomic; on a
// single counter they serialise once items are cheap: triangles.yml (6 primitives, kd depth 0,
// ~24 us per item and lane) at 10 spp made 112 K of them per 1.4 ms launch, and 8 counters (one
// shard of the items per XCD) ran it 4,937 -> 14,120 Msamples/s.  So a tiny scene (tiny_scene:
// at most 64 primitives, with triangles) gets 8 shards.  So does a scene whose traversal data
// (nodes, refs and leaf-test primitives) exceeds one XCD's 4 MiB L2: each XCD then walks its own
// shard of the launch's items (a wave starts on shard blockIdx % 8, and workgroups are dealt to
// the XCDs round-robin), so at any moment its waves are on a window of pixels of their own and its
// L2 holds a smaller window's geometry.  Measured points: a380 (~10 MiB) +4..11% in
// synchronous launches, L2 hit rate 0.935 -> 0.944; spaceship_r1 and biplane (well under 4 MiB)
// lose 3% with shards and keep one counter.  Scenes between those sizes are unmeasured.
constexpr uint64_t XCD_L2_BYTES = 4ull << 20;
static bool tiny_scene(uint32_t n_spheres, uint32_t n_free_tris, size_t n_mesh_tris) {
    return (n_free_tris + n_mesh_tris) > 0 && (uint64_t)n_spheres + n_free_tris + n_mesh_tris <= 64;
}
static uint32_t queue_shards(bool tiny, uint64_t traversal_bytes) {
    return (tiny || traversal_bytes > XCD_L2_BYTES) ? 8u : 1u;
}

// A pipeline slot's stream, fold event and item counter, created on the slot's first use: HIP
// maps streams onto its GPU_MAX_HW_QUEUES hardware queues as they are created, so a context
// makes only the streams its launches rotate over (one for large launches, n_slots for small
// overlapped ones) and leaves the other queues to the caller's streams.
static int ensure_slot(rt_ctx* c, uint32_t k) {
    Slot& sl = c->slot[k];
    if (sl.stream) return RT_OK;
    HIPCHK(c, hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
    HIPCHK(c, hipEventCreateWithFlags(&sl.fold_done, hipEventDisableTiming));
    if (hipMalloc(&sl.queue, QUEUE_BYTES) != hipSuccess) return set_err(c, RT_ERR_OOM, "queue alloc failed");
    return RT_OK;
}

static void destroy_ctx(rt_ctx* c) {
    if (!c) return;
    if (c->stream) (void)hipSetDevice(c->device);
    for (Slot& sl : c->slot) if (sl.stream) (void)hipStreamSynchronize(sl.stream);
    for (void* p : c->allocs) (void)hipFree(p);
    if (c->accum) (void)hipFree(c->accum);
    if (c->accum_range) (void)hipFree(c->accum_range);
    if (c->d_tiles) (void)hipFree(c->d_tiles);
    if (c->d_pixmap) (void)hipFree(c->d_pixmap);
    if (c->d_pixq) (void)hipFree(c->d_pixq);
    if (c->d_out) (void)hipFree(c->d_out);
    if (c->d_counts) (void)hipFree(c->d_counts);
    for (Slot& sl : c->slot) {
        if (sl.queue) (void)hipFree(sl.queue);
        if (sl.gstack) (void)hipFree(sl.gstack);
        if (sl.radiance) (void)hipFree(sl.radiance);
        if (sl.fold_done) (void)hipEventDestroy(sl.fold_done);
        if (sl.stream) (void)hipStreamDestroy(sl.stream);
    }
    for (hipEvent_t e : c->lev) (void)hipEventDestroy(e);
    if (c->caller_ev) (void)hipEventDestroy(c->caller_ev);
    if (c->win_end_ev) (void)hipEventDestroy(c->win_end_ev);
    delete c;
}

// RT_DEBUG_CREATE_TIMING=1: rt_create prints the wall time of its phases to stderr (tools/host_rates.py).
struct PhaseClock {
    bool on = debug_env("CREATE_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "rt_create %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
};

static int create_impl(rt_ctx* c, const rt_scene_desc* scene, const rt_camera* cam,
                       const rt_render_info* info, const rt_kd_tree* tree_in) {
    PhaseClock pc;
    if (info->width == 0 || info->height == 0) return set_err(c, RT_ERR_INVALID_ARG, "empty frame");
    if ((uint64_t)info->width * info->height >= (1ull << 31))
        return set_err(c, RT_ERR_INVALID_ARG, "frame too large");

    std::vector<Renderable> rs;
    int st = gather_renderables(scene, &rs);
    if (st) return set_err(c, st, "invalid scene description");

    // The 8-bit texel pool is checked and packed (pack_texels_u8) on a thread of its own while
    // the KD tree is built and the scene flattened: a380's 44 M texels take ~40 ms.
    std::vector<DevTex> texs(scene->n_textures);
    uint64_t texel_count = 0;
    for (uint32_t i = 0; i < scene->n_textures; ++i) {
        const rt_texture& tx = scene->textures[i];
        if (!tx.rgb || !tx.width || !tx.height) return set_err(c, RT_ERR_INVALID_ARG, "empty texture");
        if (texel_count + (uint64_t)tx.width * tx.height >= (1ull << 32)) return set_err(c, RT_ERR_INVALID_ARG, "texture pool too large");
        texs[i] = DevTex{(uint32_t)texel_count, tx.width, tx.height, 0};
        texel_count += (uint64_t)tx.width * tx.height;
    }
    std::vector<uint32_t> t8;
    bool t8_ok = false;
    std::thread packer;
    if (texel_count && !debug_env("TEXELS_F32"))
        packer = std::thread([&] { t8_ok = pack_texels_u8(scene, texs, texel_count, &t8); });
    struct Join { std::thread& t; ~Join() { if (t.joinable()) t.join(); } } join{packer};

    rt_kd_tree* built = nullptr;
    const rt_kd_tree* tree = tree_in;
    if (!tree) {
        st = rt_kd_build(scene, info->kd_tree_depth, &built);
        if (st) return set_err(c, st, "KD build failed");
        tree = built;
    }
    struct Guard { rt_kd_tree* t; ~Guard() { rt_kd_free(t); } } guard{built};
    pc.mark("kd_build");

    if (tree->max_leaf_depth > (uint32_t)MAX_STACK)
        return set_err(c, RT_ERR_UNSUPPORTED, "KD tree deeper than the device traversal stack");
    for (uint32_t i = 0; i < tree->n_nodes; ++i) {  // validate topology before any launch
        const rt_kd_node& n = tree->nodes[i];
        uint32_t k = n.b >> 2;
        if ((n.b & 3u) == RT_KD_LEAF) {
            if ((uint64_t)k + n.a > tree->n_refs) return set_err(c, RT_ERR_INVALID_ARG, "leaf refs out of range");
        } else if (k + 1 >= tree->n_nodes || k <= i) {
            return set_err(c, RT_ERR_INVALID_ARG, "KD child index out of range");
        }
    }

    std::vector<uint2> nodes(tree->n_nodes);
    for (uint32_t i = 0; i < tree->n_nodes; ++i) nodes[i] = make_uint2(tree->nodes[i].a, tree->nodes[i].b);
    // Leaves with identical ref lists share one copy.  A primitive that straddles many splits
    // is copied into every leaf it overlaps (kdtree.rs:119-127), so neighbouring leaves often
    // hold the same list: biplane's 5.48 M refs are 0.66 M distinct-list refs, spaceship's 3.81 M
    // are 0.14 M, which then fit in L2.  Lists keep their order, so ties resolve as before.  An
    // open-addressing table keyed on a hash of the list (the lists compared on a hash match).
    std::vector<uint32_t> refs;  // the packed lists, then converted to device refs below
    {
        const uint32_t* tr = tree->refs;
        size_t n_leaf = 0;
        for (const uint2& n : nodes) n_leaf += (n.y & 3u) == RT_KD_LEAF;
        size_t cap = 16;
        while (cap < 2 * n_leaf) cap <<= 1;
        struct Entry { uint64_t h; uint32_t at, len; };
        std::vector<Entry> table(cap, Entry{0, UINT32_MAX, 0});
        refs.reserve(tree->n_refs / 4 + 16);
        for (uint2& n : nodes) {
            if ((n.y & 3u) != RT_KD_LEAF) continue;
            if (n.x == 0) {  // an empty leaf points at the start of the packed list: its old
                n.y = RT_KD_LEAF;  // offset may lie past the end of it (no read needs it anyway)
                continue;
            }
            const uint32_t off = n.y >> 2, len = n.x;
            uint64_t h = 0x9e3779b97f4a7c15ull ^ len;
            for (uint32_t k = 0; k < len; ++k) h = (h ^ tr[off + k]) * 0xff51afd7ed558ccdull, h ^= h >> 29;
            size_t i = h & (cap - 1);
            uint32_t at = UINT32_MAX;
            for (;; i = (i + 1) & (cap - 1)) {
                const Entry& e = table[i];
                if (e.at == UINT32_MAX) break;
                if (e.h == h && e.len == len && std::memcmp(refs.data() + e.at, tr + off, 4 * (size_t)len) == 0) {
                    at = e.at;
                    break;
                }
            }
            if (at == UINT32_MAX) {
                at = (uint32_t)refs.size();
                refs.insert(refs.end(), tr + off, tr + off + len);
                table[i] = Entry{h, at, len};
            }
            n.y = (at << 2) | RT_KD_LEAF;
        }
    }
    // device refs: renderable index -> (kind, index of kind)
    for (uint32_t& ref : refs) {
        const uint32_t ri = ref;
        if (ri >= rs.size() || !rs[ri].has_aabb) return set_err(c, RT_ERR_INVALID_ARG, "bad leaf ref");
        uint32_t kind = rs[ri].kind == RT_KIND_SPHERE ? K_SPHERE : (rs[ri].kind == RT_KIND_FREE_TRI ? K_FREE_TRI : K_MESH_TRI);
        const uint32_t base = kind == K_SPHERE ? 0u : (kind == K_FREE_TRI ? scene->n_spheres
                                                                          : scene->n_spheres + scene->n_free_tris);
        ref = (kind << REF_KIND_SHIFT) | (base + rs[ri].index);  // pool index (DevScene::prim4)
    }
    // Leading sphere refs of every leaf (device_scene.h LEAF_LEAD_SHIFT): the general kernel
    // tests them per lane and leaves only triangles to the wave's cooperative passes.
    for (uint2& n : nodes) {
        if ((n.y & 3u) != RT_KD_LEAF) continue;
        if (n.x > LEAF_COUNT_MASK) return set_err(c, RT_ERR_UNSUPPORTED, "KD leaf with over 2^24 refs");
        const uint32_t off = n.y >> 2;
        uint32_t lead = 0;
        while (lead < n.x && lead < 255u && (refs[off + lead] >> REF_KIND_SHIFT) == K_SPHERE) ++lead;
        n.x |= lead << LEAF_LEAD_SHIFT;
    }

    // Direct-light sampling (radiance.rs:89-120): every AABB'd renderable as a device ref in
    // renderable order (the shadow ray's brute-force closest_ray_hit), and the emissive spheres
    // with their position in that list.  Cube maps hit at +inf and can never be a shadow ray's
    // first minimum ahead of a light, so they are left out.
    std::vector<uint32_t> elem_refs;
    std::vector<uint2> emit;
    if (info->dir_light_samp) {
        for (size_t ri = 0; ri < rs.size(); ++ri) {
            if (!rs[ri].has_aabb) continue;
            const uint32_t kind = rs[ri].kind == RT_KIND_SPHERE ? K_SPHERE : (rs[ri].kind == RT_KIND_FREE_TRI ? K_FREE_TRI : K_MESH_TRI);
            const uint32_t base = kind == K_SPHERE ? 0u : (kind == K_FREE_TRI ? scene->n_spheres
                                                                              : scene->n_spheres + scene->n_free_tris);
            if (kind == K_SPHERE && scene->spheres[rs[ri].index].mat.has_emissive)
                emit.push_back(make_uint2(rs[ri].index, (uint32_t)elem_refs.size()));
            elem_refs.push_back((kind << REF_KIND_SHIFT) | (base + rs[ri].index));
        }
    }

    bool tiny = false;  // tiny_scene (set with the leaf-test pool below)
    std::vector<float4> sph(scene->n_spheres);
    std::vector<DevMat> sph_mat(scene->n_spheres);
    for (uint32_t i = 0; i < scene->n_spheres; ++i) {
        const rt_sphere& s = scene->spheres[i];
        sph[i] = make_float4(s.c[0], s.c[1], s.c[2], s.r);
        sph_mat[i] = make_mat(s.mat, s.rgb);
    }
    std::vector<float4> ftri(3 * (size_t)scene->n_free_tris), ftri_n(scene->n_free_tris);
    std::vector<DevMat> ftri_mat(scene->n_free_tris);
    for (uint32_t i = 0; i < scene->n_free_tris; ++i) {
        const rt_free_triangle& t = scene->free_tris[i];
        for (int k = 0; k < 3; ++k) ftri[3 * i + k] = make_float4(t.verts[k][0], t.verts[k][1], t.verts[k][2], 0.f);
        ftri_n[i] = make_float4(t.norm[0], t.norm[1], t.norm[2], 0.f);
        ftri_mat[i] = make_mat(t.mat, t.rgb);
    }

    pc.mark("refs_dedupe_spheres");
    MeshFlat mf;
    if ((st = flatten_meshes(scene, &mf))) return set_err(c, st, "invalid mesh description");
    pc.mark("flatten_meshes");
    if (mf.tris.size() >= (1u << 30)) return set_err(c, RT_ERR_INVALID_ARG, "too many mesh triangles");
    std::vector<DevPrim> prims(mf.prims.size());
    for (size_t i = 0; i < prims.size(); ++i) {
        const FlatPrim& f = mf.prims[i];
        DevPrim& q = prims[i];
        for (int k = 0; k < 3; ++k) q.base_factor[k] = f.base_factor[k];
        q.base_tex = f.base_tex;
        q.normal_tex = f.normal_tex;
        q.mr_tex = f.mr_tex;
        q.metal = f.metal;
        q.rough = f.rough;
    }
    static_assert(sizeof(DevMeshTri) == sizeof(FlatTri), "mesh triangle record layout");
    std::vector<DevMeshTri> mtri(mf.tris.size());
    if (!mtri.empty()) std::memcpy(mtri.data(), mf.tris.data(), mtri.size() * sizeof(DevMeshTri));
    auto as_f4 = [](const std::vector<float>& v) {
        std::vector<float4> o(v.size() / 4);
        for (size_t i = 0; i < o.size(); ++i) o[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
        return o;
    };
    auto as_f2 = [](const std::vector<float>& v) {
        std::vector<float2> o(v.size() / 2);
        for (size_t i = 0; i < o.size(); ++i) o[i] = make_float2(v[2 * i], v[2 * i + 1]);
        return o;
    };


    DevScene& d = c->sc;
    std::memset(&d, 0, sizeof(d));
    for (uint32_t u = 0; u < tree->n_unconditional; ++u) {
        const Renderable& r = rs[tree->unconditional[u]];
        if (r.kind != RT_KIND_CUBE_MAP) continue;
        const rt_cube_map& cm = scene->cube_maps[r.index];
        for (int f = 0; f < 6; ++f) {
            int ti = cm.face[f].texture;
            if (ti < 0 || (uint32_t)ti >= scene->n_textures) return set_err(c, RT_ERR_INVALID_ARG, "bad cube face texture");
            d.face[f].off = texs[ti].off;
            d.face[f].w = texs[ti].w;
            d.face[f].h = texs[ti].h;
            d.face[f].us = cm.face[f].us;
            d.face[f].vs = cm.face[f].vs;
        }
        d.has_cube = 1;
        break;  // closest_ray_hit over the unconditional list: all hit at +inf, the first wins
    }

    HIPCHK(c, hipSetDevice(c->device));
    pc.mark("host_arrays");
    if ((st = ensure_slot(c, 0))) return st;  // the others on first use (enqueue_queue)
    c->stream = c->slot[0].stream;
    HIPCHK(c, hipEventCreateWithFlags(&c->caller_ev, hipEventDisableTiming));
    HIPCHK(c, hipEventCreate(&c->win_end_ev));
    pc.mark("streams_events");
    if ((st = upload(c, nodes, &d.nodes))) return st;
    if ((st = upload(c, elem_refs, &d.elem_refs))) return st;
    if ((st = upload(c, emit, &d.emit))) return st;
    d.n_elem_refs = (uint32_t)elem_refs.size();
    d.n_emit = (uint32_t)emit.size();
    d.dls = emit.empty() ? 0u : 1u;  // no emitter: the DLS term is exactly zero
    if ((st = upload(c, refs, &d.refs))) return st;
    if ((st = upload(c, sph, &d.sph))) return st;
    if ((st = upload(c, sph_mat, &d.sph_mat))) return st;
    {   // the leaf-test pool: spheres, free triangles, mesh triangles, 3 float4 each
        const size_t n_mesh = mf.tris.size();
        if ((uint64_t)scene->n_spheres + scene->n_free_tris + n_mesh >= (1ull << 30))
            return set_err(c, RT_ERR_INVALID_ARG, "too many primitives");
        tiny = tiny_scene(scene->n_spheres, scene->n_free_tris, n_mesh);
        const uint64_t trav_bytes = nodes.size() * sizeof(uint2) + refs.size() * sizeof(uint32_t) +
                                    3 * sizeof(float4) * ((uint64_t)scene->n_spheres + scene->n_free_tris + n_mesh);
        c->queue_shards = queue_shards(tiny, trav_bytes);
        // A tiny scene (triangles.yml: 6 primitives, ~24 us per item and lane) makes even a 7.2
        // M-sample launch mostly start-up and drain: its launches up to 2^24 samples go to the
        // small-launch pipeline (round 3, tools/gpu_a380_calib.py, 10 spp per launch: 16,600
        // Msamples/s on 2 slots with the full grid, 17,700-18,300 on 4-12 slots with a share).
        if (tiny) c->small_items = 1ull << 24;
        std::vector<float4> pool(3 * ((size_t)scene->n_spheres + scene->n_free_tris + n_mesh), make_float4(0.f, 0.f, 0.f, 0.f));
        for (uint32_t i = 0; i < scene->n_spheres; ++i) pool[3 * (size_t)i] = sph[i];
        std::memcpy(pool.data() + 3 * (size_t)scene->n_spheres, ftri.data(), ftri.size() * sizeof(float4));
        if (n_mesh) std::memcpy(pool.data() + 3 * ((size_t)scene->n_spheres + scene->n_free_tris), mf.verts.data(), 3 * n_mesh * sizeof(float4));
        // triangles as {v0, e1 = v1 - v0, e2 = v2 - v0}: generic.rs:104-105's edges, the same f32
        // subtractions the device would make per test
        for (size_t t = scene->n_spheres; t < pool.size() / 3; ++t) {
            const float4 v0 = pool[3 * t], v1 = pool[3 * t + 1], v2 = pool[3 * t + 2];
            pool[3 * t + 1] = make_float4(v1.x - v0.x, v1.y - v0.y, v1.z - v0.z, 0.f);
            pool[3 * t + 2] = make_float4(v2.x - v0.x, v2.y - v0.y, v2.z - v0.z, 0.f);
        }
        if ((st = upload(c, pool, &d.prim4))) return st;
        d.pool_ftri = scene->n_spheres;
        d.pool_mesh = scene->n_spheres + scene->n_free_tris;
    }
    if ((st = upload(c, ftri_n, &d.ftri_n))) return st;
    if ((st = upload(c, ftri_mat, &d.ftri_mat))) return st;
    if (texel_count) {
        // Textures decoded from 8-bit images hold k / 255 in every channel (image::to_rgb32f,
        // model.rs:204): such a pool is stored as one RGBA8 word per texel (a third of the bytes:
        // biplane 453 -> 151 MB, a380 525 -> 175 MB, under the 256 MB Infinity Cache) and decoded
        // on the device bit for bit.  Any other value keeps the f32 pool, uploaded straight from
        // the caller's arrays.
        pc.mark("uploads");
        if (packer.joinable()) packer.join();
        pc.mark("texel_check_pack (joined)");
        if (t8_ok) {
            void* p = nullptr;
            if (hipMalloc(&p, sizeof(uint32_t) * texel_count) != hipSuccess) return set_err(c, RT_ERR_OOM, "hipMalloc failed");
            c->allocs.push_back(p);
            HIPCHK(c, hipMemcpy(p, t8.data(), sizeof(uint32_t) * texel_count, hipMemcpyHostToDevice));
            d.texels8 = static_cast<const uint32_t*>(p);
        } else {
            void* p = nullptr;
            if (hipMalloc(&p, 3 * sizeof(float) * texel_count) != hipSuccess) return set_err(c, RT_ERR_OOM, "hipMalloc failed");
            c->allocs.push_back(p);
            for (uint32_t i = 0; i < scene->n_textures; ++i) {
                const rt_texture& tx = scene->textures[i];
                HIPCHK(c, hipMemcpy(static_cast<float*>(p) + 3 * (size_t)texs[i].off, tx.rgb,
                                    3 * sizeof(float) * (size_t)tx.width * tx.height, hipMemcpyHostToDevice));
            }
            d.texels = static_cast<const float*>(p);
        }
    }
    pc.mark("texel_upload");
    if ((st = upload(c, texs, &d.tex))) return st;
    if ((st = upload(c, mtri, &d.mtri))) return st;
    if ((st = upload(c, prims, &d.prims))) return st;
    if ((st = upload(c, as_f4(mf.norms), &d.vnorm))) return st;
    if ((st = upload(c, as_f2(mf.base_uv), &d.uv_base))) return st;
    if ((st = upload(c, as_f2(mf.normal_uv), &d.uv_norm))) return st;
    if ((st = upload(c, as_f2(mf.mr_uv), &d.uv_mr))) return st;
    d.n_nodes = tree->n_nodes;
    d.fastdiv = 1;  // see trace.hip div_exact: splits must be 0 or in [2^-70, 2^61)
    for (uint32_t i = 0; i < tree->n_nodes; ++i) {
        if ((tree->nodes[i].b & 3u) == RT_KD_LEAF) continue;
        const uint32_t m = tree->nodes[i].a & 0x7fffffffu;
        if (m != 0u && (m < (57u << 23) || m >= (188u << 23))) d.fastdiv = 0;
    }
    d.stack_depth = tree->max_leaf_depth ? tree->max_leaf_depth : 1u;
    // closest_small (trace.hip) relies on finite sphere roots: every ray origin (camera, lens
    // point, or a point on a sphere) then has |o_i| < 2^59, so |o - c| < 2^60 per component and
    // dot(d, o - c), (o - c).(o - c) - r^2 and the discriminant stay finite for unit d.
    {
        const float lim = 0x1p58f;
        bool ok = true;
        for (uint32_t i = 0; i < scene->n_spheres && ok; ++i) {
            const rt_sphere& sp = scene->spheres[i];
            for (int a = 0; a < 3; ++a) ok = ok && std::fabs(sp.c[a]) + std::fabs(sp.r) < lim;
        }
        float up2 = 0.f;
        for (int a = 0; a < 3; ++a) {
            ok = ok && std::fabs(cam->o[a]) < lim;
            up2 += cam->up[a] * cam->up[a];
        }
        ok = ok && (!cam->has_lens || std::fabs(cam->lens_r) * (std::sqrt(up2) + 2.0f) < lim);
        // in_return_leaf also stands in for the root slab test: every sphere's box
        // [fl(c - r), fl(c + r)] must lie inside the tree's bounds (true for rt_kd_build's trees),
        // and r >= 0 orders its faces
        ok = ok && tree->n_nodes > 0;
        for (uint32_t i = 0; i < scene->n_spheres && ok; ++i) {
            const rt_sphere& sp = scene->spheres[i];
            ok = ok && sp.r >= 0.0f;
            for (int a = 0; a < 3; ++a) {
                const float lo = sp.c[a] - sp.r, hi = sp.c[a] + sp.r;
                ok = ok && tree->bounds[2 * a] <= lo && hi <= tree->bounds[2 * a + 1];
            }
        }
        d.small_ok = ok ? 1u : 0u;
    }
    d.n_spheres = scene->n_spheres;
    // the sphere-only kernel reads every sphere from its LDS table (trace.hip fetch_sphere)
    // (DLS runs in the general kernel)
    d.spheres_only = (scene->n_free_tris == 0 && mf.tris.empty() && scene->n_spheres <= LDS_SPHERES && !d.dls) ? 1u : 0u;
    for (int i = 0; i < 6; ++i) d.bounds[i] = tree->bounds[i];

    // RayCompute::new (generate.rs:13-23)
    const int w = (int)info->width, h = (int)info->height;
    d.x_cf = cam->screen_width / (float)w;
    d.y_cf = cam->screen_height / (float)h;
    {
        float dn = std::sqrt((cam->d[0] * cam->d[0] + cam->d[1] * cam->d[1]) + cam->d[2] * cam->d[2]);
        float nd[3] = {cam->d[0] / dn, cam->d[1] / dn, cam->d[2] / dn};
        const float* up = cam->up;
        float cr[3] = {nd[1] * up[2] - nd[2] * up[1], nd[2] * up[0] - nd[0] * up[2], nd[0] * up[1] - nd[1] * up[0]};
        float cn = std::sqrt((cr[0] * cr[0] + cr[1] * cr[1]) + cr[2] * cr[2]);
        for (int i = 0; i < 3; ++i) d.right[i] = cr[i] / cn;
    }
    d.x_off = (float)w / 2.0f;
    d.y_off = (float)h / 2.0f;
    for (int i = 0; i < 3; ++i) {
        d.cam_d[i] = cam->d[i];
        d.cam_o[i] = cam->o[i];
        d.cam_up[i] = cam->up[i];
    }
    d.has_lens = cam->has_lens ? 1u : 0u;
    d.lens_r = cam->lens_r;
    d.width = info->width;
    d.height = info->height;
    d.assured_depth = info->assured_depth;
    d.debug_single_ray = info->debug_single_ray ? 1u : 0u;
    d.seed = info->seed;

    pc.mark("mesh_uploads");
    const size_t npix = (size_t)info->width * info->height;
    if (hipMalloc(&c->accum, npix * sizeof(float4)) != hipSuccess) return set_err(c, RT_ERR_OOM, "accumulator alloc failed");
    HIPCHK(c, hipMemset(c->accum, 0, npix * sizeof(float4)));
    if (hipMalloc(&c->d_counts, sizeof(DevCounts)) != hipSuccess) return set_err(c, RT_ERR_OOM, "counter alloc failed");
    hipDeviceProp_t prop;
    HIPCHK(c, hipGetDeviceProperties(&prop, c->device));
    c->lane_capacity = (uint64_t)prop.multiProcessorCount * 4 /*SIMD*/ * 7 /*waves*/ * 64;
    pc.mark("accum_props");
    c->n_cu = (uint32_t)prop.multiProcessorCount;
    // RT_DEBUG_SCHED=direct[:K]: the direct schedule (K lanes per pixel, 1/2/4/8; the default K
    // follows the launch's pixels), the tests' second path; "queue" is the default.
    if (const char* e = debug_env("SCHED")) {
        if (!std::strncmp(e, "direct", 6)) {
            c->sched = 1;
            if (e[6] == ':') {
                const unsigned long v = std::strtoul(e + 7, nullptr, 10);
                if (v == 1 || v == 2 || v == 4 || v == 8) c->forced_k = (uint32_t)v;
            }
        } else if (!std::strcmp(e, "queue")) {
            c->sched = 2;
        }
    }
    // Traversal of the queue kernels: the reference's stack (kdtree.rs:66-104) or stackless
    // kd-restart with push-down, bit-identical (trace.hip stack_search_coop).  The stack is faster
    // on the mesh scenes; the sphere-only kernel, which descends for 0.05 nodes
    // per sample, runs stackless and needs no global stack.  RT_DEBUG_KD_RESTART=0/1 overrides.
    // Camera-ray packets in the general queue kernel (trace.hip closest_packet), bit-identical to
    // the cooperative search; RT_DEBUG_PACKET=0 turns them off.  RT_DEBUG_PIX_BLOCK=1 gives the queue the
    // launch pixels in row order instead of 8 x 8 blocks (the same images).
    d.packet = 1u;
    if (const char* e = debug_env("PACKET")) d.packet = std::strcmp(e, "0") ? 1u : 0u;
    c->pix_block = RT_PIX_BLOCK;
    if (const char* e = debug_env("PIX_BLOCK")) {
        const unsigned long v = std::strtoul(e, nullptr, 10);
        if (v >= 1 && v <= 64) c->pix_block = (uint32_t)v;
    }
    d.restart = d.spheres_only ? 1u : 0u;
    if (const char* e = debug_env("KD_RESTART")) d.restart = std::strcmp(e, "0") ? 1u : 0u;
    // Overlapped launches pay off while a launch's drain tail is a sizeable share of it: mesh
    // launches (8-10 ms tails) and small sphere-only ones — walled's ~0.4 ms tail on
    // one rank's 90 M-sample share at N = 8 (9 ms): +3% overlapped, while at 180 M it is neutral
    // and at 360 / 720 M a fold beside the next trace grid costs 1%.  enqueue_queue overlaps
    // launches of at most overlap_max_items (2^27) samples.
    c->overlap = true;
    c->queue_floats = QUEUE_RADIANCE_FLOATS;
    {
        const char* q = std::getenv("GPU_MAX_HW_QUEUES");  // what HIP read when it started
        const int hwq = q && std::atoi(q) > 0 ? std::atoi(q) : 4;
        c->small_slots = slots_for_queues(hwq);
        c->mid_slots = mid_slots_for(c->small_slots);
        // A tiny scene (items of ~24 us) runs its launches of up to 2^24 samples on the
        // small-launch pipeline (above), with the mid-size slot count and half the grid each
        // (round 4, triangles.yml's 7.2 M-sample launches at 16 queues: 12 slots with an eighth of
        // the grid 16,000 Msamples/s, 4 / 6 slots with a half 17,100 / 17,000, 2 slots with the full
        // grid 16,700).
        if (tiny) {
            c->small_slots = c->mid_slots;
            if (c->small_slots >= 4) c->small_div = 2;
        }
    }
    // RT_DEBUG_LAUNCH="key=value,...": the launch pipeline's A/B and test settings (INTEGRATION.md
    // §6): overlap=0|1|2 (never / up to overlap_max_items / always), slots=2..32, grid_div=1..64,
    // small_items=N, group_items=N, shards=1..32, radiance_gib=1..64, radiance_floats=N (tests:
    // force split launches).  Unknown keys are ignored.
    if (const char* e = debug_env("LAUNCH")) {
        for (const char* k = e; *k;) {
            const char* eq = std::strchr(k, '=');
            if (!eq) break;
            const std::string key(k, (size_t)(eq - k));
            char* endp = nullptr;
            const unsigned long long v = std::strtoull(eq + 1, &endp, 10);
            if (key == "overlap") {
                c->overlap = v != 0;
                if (v == 2) c->overlap_max_items = ~0ull;
            } else if (key == "slots" && v >= 2 && v <= (unsigned long long)N_SLOTS) {
                c->n_slots = (uint32_t)v;
            } else if (key == "grid_div" && v >= 1 && v <= 64) {
                c->grid_div = (uint32_t)v;
            } else if (key == "small_items") {
                c->small_items = v;
            } else if (key == "group_items") {
                c->group_items = v;
            } else if (key == "shards" && v >= 1 && v <= 32) {
                c->queue_shards = (uint32_t)v;
            } else if (key == "radiance_gib" && v >= 1 && v <= 64) {
                c->queue_floats = (uint64_t)v << 28;
            } else if (key == "radiance_floats" && v >= 3 && v <= (1ull << 34)) {
                c->queue_floats = (uint64_t)v;
            }
            if (*endp != ',') break;
            k = endp + 1;
        }
    }
    return RT_OK;
}

extern "C" int rt_create(const rt_scene_desc* scene, const rt_camera* cam, const rt_render_info* info,
                         const rt_kd_tree* tree, int device, rt_ctx** out) {
    if (!scene || !cam || !info || !out) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    int total = 0;
    if (hipGetDeviceCount(&total) != hipSuccess || device < 0 || device >= total || !is_gfx950(device))
        return RT_ERR_NO_DEVICE;
    rt_ctx* c = new (std::nothrow) rt_ctx();
    if (!c) return RT_ERR_OOM;
    c->device = device;
    int st = guarded(c, [&] { return create_impl(c, scene, cam, info, tree); });
    if (st) {
        std::fprintf(stderr, "rt_create: %s\n", c->err.c_str());
        destroy_ctx(c);
        return st;
    }
    *out = c;
    return RT_OK;
}

// Drains both pipeline slots and closes the timing window: per-launch trace durations and the
// window's span, from its first trace launch to its last fold.
static int sync_all(rt_ctx* c) {
    for (Slot& sl : c->slot) if (sl.stream) HIPCHK(c, hipStreamSynchronize(sl.stream));
    if (!c->pending) return RT_OK;
    c->pending = false;
    c->trace_ms = 0.f;
    for (uint32_t i = 0; i < c->n_timed; ++i) {
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->lev[2 * i], c->lev[2 * i + 1]));
        c->trace_ms += ms;
    }
    c->last_ms = 0.f;
    if (c->n_timed && c->win_end) HIPCHK(c, hipEventElapsedTime(&c->last_ms, c->lev[0], c->win_end));
    return RT_OK;
}

// Opens a new timing window unless one is pending (async calls extend it).
static void open_window(rt_ctx* c) {
    if (c->pending) return;
    c->pending = true;
    c->n_launch = 0;
    c->n_timed = 0;
    c->win_end = nullptr;
}

// An event from the pool: launch i's start (begin) or stop, recorded on `s`.  Past
// MAX_TIMED_LAUNCHES launches in one window nothing is recorded, except a stop that must end
// the window (`out`), which goes to win_end_ev.
static constexpr uint32_t MAX_TIMED_LAUNCHES = 256;
static int record_launch_event(rt_ctx* c, bool begin, hipStream_t s, hipEvent_t* out = nullptr) {
    if (c->n_timed >= MAX_TIMED_LAUNCHES) {
        if (!begin) {
            c->n_launch++;
            if (out) {
                HIPCHK(c, hipEventRecord(c->win_end_ev, s));
                *out = c->win_end_ev;
            }
        }
        return RT_OK;
    }
    const size_t i = 2 * (size_t)c->n_timed + (begin ? 0 : 1);
    while (c->lev.size() <= i) {
        hipEvent_t e;
        HIPCHK(c, hipEventCreate(&e));
        c->lev.push_back(e);
    }
    HIPCHK(c, hipEventRecord(c->lev[i], s));
    if (out) *out = c->lev[i];
    if (!begin) {
        c->n_launch++;
        c->n_timed++;
    }
    return RT_OK;
}

// Builds the per-launch tile table (and the pixel table) unless the same tiles are already on
// the device; returns the number of output pixels.  New tiles drain the pipeline first, since a
// launch in flight may read the old tables.
static int prepare_tiles(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles, uint32_t K, LaunchArgs* a,
                         uint64_t* n_out) {
    if (!tiles || n_tiles == 0) return set_err(c, RT_ERR_INVALID_ARG, "no tiles");
    std::vector<DevTile> dt(n_tiles);
    uint64_t blocks = 0, pix = 0;
    for (uint32_t i = 0; i < n_tiles; ++i) {
        const rt_tile& t = tiles[i];
        if (t.w == 0 || t.h == 0 || (uint64_t)t.x0 + t.w > c->sc.width || (uint64_t)t.y0 + t.h > c->sc.height)
            return set_err(c, RT_ERR_INVALID_ARG, "tile outside the frame");
        DevTile& d = dt[i];
        d.x0 = t.x0; d.y0 = t.y0; d.w = t.w; d.h = t.h;
        d.out_off = (uint32_t)pix;
        d.block_begin = (uint32_t)blocks;
        d.bx = (t.w + BLOCK_W - 1) / BLOCK_W;
        const uint32_t bh = BLOCK_H / K;
        blocks += (uint64_t)d.bx * ((t.h + bh - 1) / bh);
        pix += (uint64_t)t.w * t.h;
    }
    if (blocks >= (1ull << 31) || pix >= (1ull << 32)) return set_err(c, RT_ERR_INVALID_ARG, "too many pixels");
    const bool same = c->pixmap_tiles.size() == dt.size() &&
                      std::memcmp(c->pixmap_tiles.data(), dt.data(), dt.size() * sizeof(DevTile)) == 0;
    if (!same) {
        int st = sync_all(c);
        if (st) return st;
        if (n_tiles > c->d_tiles_cap) {
            if (c->d_tiles) (void)hipFree(c->d_tiles);
            c->d_tiles = nullptr;
            c->d_tiles_cap = 0;
            if (hipMalloc(&c->d_tiles, n_tiles * sizeof(DevTile)) != hipSuccess) return set_err(c, RT_ERR_OOM, "tile alloc failed");
            c->d_tiles_cap = n_tiles;
        }
        HIPCHK(c, hipMemcpy(c->d_tiles, dt.data(), n_tiles * sizeof(DevTile), hipMemcpyHostToDevice));
        // A per-pixel table replaces the per-item binary search over the tiles (whose dependent
        // loads held back every wave that started a path: rank 0 of 8 with 1-row stripes ran 8%
        // slower) and the divisions by the tile width.
        if (c->sc.width <= 65535u && c->sc.height <= 65535u) {
            std::vector<uint32_t> pm(pix);
            for (const DevTile& d : dt)
                for (uint32_t y = 0; y < d.h; ++y)
                    for (uint32_t x = 0; x < d.w; ++x) pm[d.out_off + (size_t)y * d.w + x] = ((d.y0 + y) << 16) | (d.x0 + x);
            // queue order: RT_PIX_BLOCK x RT_PIX_BLOCK blocks of each tile, row by row
            std::vector<uint4> pq;
            pq.reserve(pix);
            const uint32_t B = c->pix_block;
            for (const DevTile& d : dt)
                for (uint32_t by = 0; by < d.h; by += B)
                    for (uint32_t bx = 0; bx < d.w; bx += B)
                        for (uint32_t y = by; y < std::min(by + B, d.h); ++y)
                            for (uint32_t x = bx; x < std::min(bx + B, d.w); ++x) {
                                const uint32_t o = d.out_off + y * d.w + x;
                                const uint32_t fx = d.x0 + x, fy = d.y0 + y;
                                const uint64_t key = rt_rng_pixel_key(c->sc.seed, fy * c->sc.width + fx);
                                pq.push_back(make_uint4(pm[o], o, (uint32_t)key, (uint32_t)(key >> 32)));
                            }
            if (pix > c->d_pixmap_cap) {
                if (c->d_pixmap) (void)hipFree(c->d_pixmap);
                if (c->d_pixq) (void)hipFree(c->d_pixq);
                c->d_pixmap = nullptr;
                c->d_pixq = nullptr;
                c->d_pixmap_cap = 0;
                if (hipMalloc(&c->d_pixmap, pix * sizeof(uint32_t)) != hipSuccess ||
                    hipMalloc(&c->d_pixq, pix * sizeof(uint4)) != hipSuccess)
                    return set_err(c, RT_ERR_OOM, "pixel map alloc failed");
                c->d_pixmap_cap = pix;
            }
            HIPCHK(c, hipMemcpy(c->d_pixmap, pm.data(), pix * sizeof(uint32_t), hipMemcpyHostToDevice));
            HIPCHK(c, hipMemcpy(c->d_pixq, pq.data(), pix * sizeof(uint4), hipMemcpyHostToDevice));
        }
        c->pixmap_tiles = dt;
    }
    a->pix_xy = (c->sc.width <= 65535u && c->sc.height <= 65535u) ? c->d_pixmap : nullptr;
    a->pix_q = (a->pix_xy && c->pix_block > 1) ? c->d_pixq : nullptr;
    a->sc = c->sc;
    a->tiles = c->d_tiles;
    a->n_tiles = n_tiles;
    a->n_blocks = (uint32_t)blocks;
    a->accum = c->accum;
    a->lanes_per_pixel = K;
    a->n_pix = (uint32_t)pix;
    a->n_pix_magic = pix > 1 ? (uint32_t)((1ull << 32) / pix) : 0u;
    *n_out = pix;
    return RT_OK;
}

static uint64_t tile_pixels(const rt_tile* tiles, uint32_t n) {
    uint64_t p = 0;
    for (uint32_t i = 0; i < n; ++i) p += (uint64_t)tiles[i].w * tiles[i].h;
    return p;
}

// Lanes per pixel: enough (pixel, sample-stream) lanes to fill the chip ~1.5x at the kernel's
// occupancy; 1 whenever the launch has that many pixels (then samples fold in registers).
static uint32_t choose_k(const rt_ctx* c, uint64_t n_pix) {
    if (c->forced_k) return c->forced_k;
    uint32_t k = 1;
    while (k < (uint32_t)BLOCK_H && n_pix * k * 2 < c->lane_capacity * 3) k *= 2;
    return k;
}

// A slot's radiance buffer of at least `floats`; the slot's stream is drained before a
// reallocation (a launch of its own may still be writing the old buffer).
static int ensure_radiance(rt_ctx* c, Slot& sl, uint64_t floats) {
    if (floats <= sl.radiance_cap) return RT_OK;
    HIPCHK(c, hipStreamSynchronize(sl.stream));
    if (sl.radiance) (void)hipFree(sl.radiance);
    sl.radiance = nullptr;
    sl.radiance_cap = 0;
    if (hipMalloc(&sl.radiance, floats * sizeof(float)) != hipSuccess)
        return set_err(c, RT_ERR_OOM, "radiance buffer alloc failed");
    sl.radiance_cap = floats;
    return RT_OK;
}

static constexpr uint32_t SAMPLES_PER_LANE_CHUNK = 64;

// Schedule: the queue (persistent lanes over (pixel, sample) items, tools/variant_bench.py:
// walled 3040 -> 3625, biplane 17 -> 65-70 Msamples/s) unless RT_DEBUG_SCHED=direct[:K]
// asks for the direct one-lane-per-pixel schedule (kept for A/B and as the
// tests' second path).
static bool use_queue(const rt_ctx* c) {
    if (c->forced_k) return false;
    return c->sched != 1;
}

// Queue schedule, asynchronous: each chunk of samples (bounded by the radiance cap) is one
// trace launch on the next pipeline slot, followed on the same stream by its fold.  The trace
// waits only for its slot's previous fold (same stream); the fold also waits for the previous
// chunk's fold (accumulator order, draw_scene.rs:81-83) and, when given, for `after` (the
// caller's stream: its readers of `out` from the previous call).  Returns with the last fold
// in c->last_fold.
//
// Batches (rt_render_batches_device_async, rt_render_to_target): the call's samples are
// consecutive batches of `batch` samples, and batch k's frame goes to outs[k] (nullptr: none).
// The trace launches are the call's, whatever the batches; after each one the fold runs batch by
// batch — one fold kernel per batch part inside the launch, in sample order — and the fold that
// completes batch k writes outs[k].  A fold part reads its rows of the launch's radiance buffer
// ([sample][pixel], so a part is a contiguous block) and continues the running mean exactly where
// the previous part left it: the frames are those of one call per batch, bit for bit.  Chunks of
// a call with several batches hold whole batches when a batch fits the radiance cap.
static int enqueue_queue(rt_ctx* c, LaunchArgs a, uint64_t n_out, uint64_t sample_begin,
                         uint32_t sample_count, hipEvent_t after, uint32_t batch, float4* const* outs) {
    if (batch == 0 || batch > sample_count) batch = sample_count ? sample_count : 1u;
    uint64_t chunk = c->queue_floats / (3 * n_out);
    if (chunk < 1) chunk = 1;
    if (chunk > sample_count) chunk = sample_count ? sample_count : 1;
    int per_cu = 0;  // the queue grid: the resident workgroups of this scene's kernel
    HIPCHK(c, queue_blocks_per_cu(a, &per_cu));
    if (per_cu < 1) per_cu = 1;
    const uint32_t tpb = queue_block_threads(a);  // threads per workgroup of the scene's queue kernel
    const uint64_t lanes = (uint64_t)c->n_cu * (uint64_t)per_cu * tpb;
    // the counter overshoots n_items by at most one grab (<= 1024 = 16 x 64) per wave
    if (n_out * chunk + lanes * 16 >= (1ull << 32)) chunk = ((1ull << 32) - lanes * 16 - 1) / n_out;
    if (chunk < 1) return set_err(c, RT_ERR_INVALID_ARG, "too many pixels for one launch");
    if (sample_count > chunk && batch < sample_count && chunk >= batch) {
        // whole batches per launch, in equal launches of ceil(n_batches / n) batches
        const uint64_t nb = sample_count / batch, per = chunk / batch;
        const uint64_t n = (nb + per - 1) / per;
        chunk = batch * ((nb + n - 1) / n);
    } else if (sample_count > chunk) {  // equal launches: ceil(count / n) samples each
        const uint64_t n = (sample_count + chunk - 1) / chunk;
        chunk = (sample_count + n - 1) / n;
    }
    uint32_t done = 0;
    do {
        a.sample_begin = sample_begin + done;
        a.sample_count = (uint32_t)(sample_count - done < chunk ? sample_count - done : chunk);
        a.n_items = (uint32_t)(n_out * a.sample_count);
        // Without overlap the trace waits for the previous fold: the sphere-only kernel's drain
        // tail is ~0.4 ms, and a fold beside the next persistent trace grid cost walled 2% (its
        // workgroups take slots from that grid).  Mesh launches overlap while the ~10 ms tail is
        // a sizeable share of the launch: up to overlap_max_items samples (a380 at 7.2 M: +19%,
        // spaceship at 18 M: +10%; spaceship 4096^2 at 419 M: -2%, triangles at 720 M: -4%).
        // Overlapped launches alternate slots; a serialized one stays on the last slot's stream,
        // behind its fold, with one radiance buffer.
        const bool overlap = c->overlap && a.n_items <= c->overlap_max_items;
        const bool small = a.n_items <= c->small_items;
        // a small launch behind a launch still running takes a share of the grid (see N_SLOTS)
        bool busy = false;
        if (c->last_fold) {
            const hipError_t q = hipEventQuery(c->last_fold);
            if (q == hipErrorNotReady) {
                busy = true;
                (void)hipGetLastError();  // clear the not-ready status only (every earlier call was checked)
            } else if (q != hipSuccess) {  // e.g. a faulted earlier launch: report it, do not launch
                (void)hipGetLastError();   // reported here, not again by a later call's launch check
                return set_err(c, RT_ERR_HIP, std::string("hipEventQuery(last fold): ") + hipGetErrorString(q));
            }
        }
        const uint32_t n_slots = c->n_slots ? c->n_slots
                                            : (small ? c->small_slots : (a.n_items <= MID_LAUNCH_ITEMS ? c->mid_slots : 2u));
        // the grid share follows the slots this launch rotates over (RT_DEBUG_LAUNCH grid_div overrides)
        const uint32_t grid_div = c->grid_div ? c->grid_div : (c->small_div ? c->small_div : small_grid_div(n_slots));
        if (overlap) c->cur_slot = (c->cur_slot + 1) % n_slots;
        for (uint32_t k = 0; k < (overlap ? n_slots : 1u); ++k) {
            const int e = ensure_slot(c, overlap ? k : c->cur_slot);
            if (e) return e;
        }
        Slot& sl = c->slot[c->cur_slot];
        const uint64_t floats = 3 * n_out * (a.sample_count ? a.sample_count : 1);
        int st = ensure_radiance(c, sl, floats);
        // every slot's buffer at once, so that no allocation lands between overlapped launches
        for (uint32_t k = 0; overlap && !st && k < n_slots; ++k) st = ensure_radiance(c, c->slot[k], floats);
        if (st) return st;
        a.radiance = sl.radiance;
        a.queue = sl.queue;
        a.n_shards = c->queue_shards;
        a.gstack = nullptr;
        if (const size_t gb = queue_gstack_bytes(a, (uint32_t)(lanes / tpb))) {
            if (gb > sl.gstack_cap) {
                HIPCHK(c, hipStreamSynchronize(sl.stream));
                if (sl.gstack) (void)hipFree(sl.gstack);
                sl.gstack = nullptr;
                sl.gstack_cap = 0;
                if (hipMalloc(&sl.gstack, gb) != hipSuccess) return set_err(c, RT_ERR_OOM, "traversal stack alloc failed");
                sl.gstack_cap = gb;
            }
            a.gstack = sl.gstack;
        }
        if (!overlap && c->last_fold && c->last_fold != sl.fold_done)
            HIPCHK(c, hipStreamWaitEvent(sl.stream, c->last_fold, 0));
        if (a.sample_count) {
            HIPCHK(c, hipMemsetAsync(sl.queue, 0, QUEUE_BYTES, sl.stream));
            if ((st = record_launch_event(c, true, sl.stream))) return st;
            uint32_t nb = (uint32_t)(lanes / tpb);
            if (overlap && small && busy && grid_div > 1)
                nb = nb / grid_div > (uint32_t)c->n_cu ? nb / grid_div : (uint32_t)c->n_cu;
            HIPCHK(c, launch_trace_queue(a, nb, sl.stream));
            if ((st = record_launch_event(c, false, sl.stream))) return st;
        }
        if (c->last_fold && c->last_fold != sl.fold_done) HIPCHK(c, hipStreamWaitEvent(sl.stream, c->last_fold, 0));
        if (after) HIPCHK(c, hipStreamWaitEvent(sl.stream, after, 0));
        // the fold, batch part by batch part (one part when the launch is inside one batch)
        const uint64_t cb = a.sample_begin, ce = cb + a.sample_count;
        uint64_t fs = cb;
        do {
            const uint64_t k = (fs - sample_begin) / batch;
            const uint64_t be = sample_begin + (k + 1) * batch;
            const uint64_t fe = ce < be ? ce : be;
            LaunchArgs f = a;
            f.sample_begin = fs;
            f.sample_count = (uint32_t)(fe - fs);
            f.radiance = a.radiance + 3 * n_out * (fs - cb);
            f.out = (fe == be || fe == sample_begin + sample_count) ? outs[k] : nullptr;
            HIPCHK(c, launch_fold(f, sl.stream));
            fs = fe;
        } while (fs < ce);
        HIPCHK(c, hipEventRecord(sl.fold_done, sl.stream));
        c->last_fold = sl.fold_done;
        done += a.sample_count;
    } while (done < sample_count);
    // the window ends at this fold (fold_done carries no timestamp)
    HIPCHK(c, hipEventRecord(c->win_end_ev, c->slot[c->cur_slot].stream));
    c->win_end = c->win_end_ev;
    return RT_OK;
}

// Direct schedule (trace_kernel), synchronous on slot 0 after draining the pipeline.
static int run_direct(rt_ctx* c, LaunchArgs a, uint64_t n_out, uint32_t K, uint64_t sample_begin,
                      uint32_t sample_count) {
    int st = sync_all(c);
    if (st) return st;
    open_window(c);
    Slot& sl = c->slot[0];
    if (K == 1) {
        a.sample_begin = sample_begin;
        a.sample_count = sample_count;
        if ((st = record_launch_event(c, true, sl.stream))) return st;
        HIPCHK(c, launch_trace(a, sl.stream));  // count 0 still (re)writes the accumulators
        if ((st = record_launch_event(c, false, sl.stream, &c->win_end))) return st;
    } else {
        const uint32_t chunk = sample_count < SAMPLES_PER_LANE_CHUNK * K ? sample_count : SAMPLES_PER_LANE_CHUNK * K;
        if ((st = ensure_radiance(c, sl, 3 * n_out * (chunk ? chunk : 1)))) return st;
        a.radiance = sl.radiance;
        uint32_t done = 0;
        do {
            a.sample_begin = sample_begin + done;
            a.sample_count = sample_count - done < chunk ? sample_count - done : chunk;
            if (a.sample_count) {
                if ((st = record_launch_event(c, true, sl.stream))) return st;
                HIPCHK(c, launch_trace(a, sl.stream));
                if ((st = record_launch_event(c, false, sl.stream, &c->win_end))) return st;
            }
            HIPCHK(c, launch_fold(a, sl.stream));
            done += a.sample_count;
        } while (done < sample_count);
    }
    HIPCHK(c, hipEventRecord(sl.fold_done, sl.stream));
    c->last_fold = sl.fold_done;
    c->cur_slot = 0;
    return RT_OK;
}

// Enqueues one rt_render* call.  `after`: an event the output writers must wait for.  `range`:
// the mean over this call's samples alone (rt_render_range), in accum_range.
static int render_impl_(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                        uint32_t sample_count, float4* dev_out, hipEvent_t after, bool range);
static int render_impl(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                       uint32_t sample_count, float4* dev_out, hipEvent_t after, bool range = false) {
    return guarded(c, [&] { return render_impl_(c, tiles, n_tiles, sample_begin, sample_count, dev_out, after, range); });
}
static int render_impl_(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                        uint32_t sample_count, float4* dev_out, hipEvent_t after, bool range) {
    LaunchArgs a{};
    uint64_t n_out = 0;
    const uint32_t K = choose_k(c, tile_pixels(tiles, n_tiles));
    int st = prepare_tiles(c, tiles, n_tiles, use_queue(c) ? 1 : K, &a, &n_out);
    if (st) return st;
    a.out = dev_out;
    if (range) {
        if (!c->accum_range) {
            st = sync_all(c);
            if (st) return st;
            if (hipMalloc(&c->accum_range, (size_t)c->sc.width * c->sc.height * sizeof(float4)) != hipSuccess)
                return set_err(c, RT_ERR_OOM, "range accumulator alloc failed");
        }
        a.accum = c->accum_range;
        a.mean_base = sample_begin;
    }
    if (!use_queue(c)) return run_direct(c, a, n_out, K, sample_begin, sample_count);
    open_window(c);
    return enqueue_queue(c, a, n_out, sample_begin, sample_count, after, sample_count, &dev_out);
}

// n_batches consecutive batches of `batch` samples from sample_begin, batch k's frame into outs[k]
// (enqueue_queue's fold parts); the direct schedule renders them one call at a time.
static int render_batches_impl(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                               uint32_t batch, uint32_t n_batches, float4* const* outs, hipEvent_t after) {
    if (n_batches == 0) return RT_OK;
    if (batch == 0 || (uint64_t)batch * n_batches >= (1ull << 32)) return set_err(c, RT_ERR_INVALID_ARG, "bad batches");
    if (!use_queue(c)) {
        for (uint32_t k = 0; k < n_batches; ++k) {
            const int st = render_impl(c, tiles, n_tiles, sample_begin + (uint64_t)k * batch, batch, outs[k], after);
            if (st) return st;
        }
        return RT_OK;
    }
    return guarded(c, [&]() -> int {
        LaunchArgs a{};
        uint64_t n_out = 0;
        int st = prepare_tiles(c, tiles, n_tiles, 1, &a, &n_out);
        if (st) return st;
        a.out = nullptr;
        open_window(c);
        return enqueue_queue(c, a, n_out, sample_begin, batch * n_batches, after, batch, outs);
    });
}

static int ensure_out(rt_ctx* c, uint64_t n) {
    if (n <= c->d_out_cap) return RT_OK;
    int st = sync_all(c);
    if (st) return st;
    if (c->d_out) (void)hipFree(c->d_out);
    c->d_out = nullptr;
    c->d_out_cap = 0;
    if (hipMalloc(&c->d_out, n * sizeof(float4)) != hipSuccess) return set_err(c, RT_ERR_OOM, "output alloc failed");
    c->d_out_cap = n;
    return RT_OK;
}

extern "C" int rt_render(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                         uint32_t sample_count, float* out_rgba) {
    if (!c || !tiles) return RT_ERR_INVALID_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t n = tile_pixels(tiles, n_tiles);
    int st;
    if (out_rgba && (st = ensure_out(c, n))) return st;
    if ((st = sync_all(c))) return st;  // a synchronous call is its own timing window
    if ((st = render_impl(c, tiles, n_tiles, sample_begin, sample_count, out_rgba ? c->d_out : nullptr, nullptr))) return st;
    if (out_rgba)  // on the stream of the last fold
        HIPCHK(c, hipMemcpyAsync(out_rgba, c->d_out, n * sizeof(float4), hipMemcpyDeviceToHost,
                                 c->slot[c->cur_slot].stream));
    return sync_all(c);
}

// The mean over [sample_begin, sample_begin + sample_count) alone: block_and_get_single_result
// (gpu_utils.rs:681-724) of one batch, whose kernel folds its samples with a running mean that
// starts at zero (trace.wgsl:277-318).  The context's cumulative mean is left alone.
extern "C" int rt_render_range(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                               uint32_t sample_count, float* out_rgba) {
    if (!c || !tiles || !out_rgba) return RT_ERR_INVALID_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t n = tile_pixels(tiles, n_tiles);
    int st;
    if ((st = ensure_out(c, n))) return st;
    if ((st = sync_all(c))) return st;
    if ((st = render_impl(c, tiles, n_tiles, sample_begin, sample_count, c->d_out, nullptr, true))) return st;
    HIPCHK(c, hipMemcpyAsync(out_rgba, c->d_out, n * sizeof(float4), hipMemcpyDeviceToHost,
                             c->slot[c->cur_slot].stream));
    return sync_all(c);
}

extern "C" int rt_render_device_async(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles,
                                      uint64_t sample_begin, uint32_t sample_count, float* out_dev,
                                      void* stream) {
    if (!c || !tiles || !out_dev) return RT_ERR_INVALID_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t cs = static_cast<hipStream_t>(stream);
    // the caller's work enqueued so far (e.g. a gather still reading out_dev) precedes the folds
    HIPCHK(c, hipEventRecord(c->caller_ev, cs));
    int st = render_impl(c, tiles, n_tiles, sample_begin, sample_count, reinterpret_cast<float4*>(out_dev),
                         c->caller_ev);
    if (st) return st;
    // and the caller's later work sees the finished output
    HIPCHK(c, hipStreamWaitEvent(cs, c->last_fold, 0));
    return RT_OK;
}

extern "C" int rt_render_batches_device_async(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles,
                                              uint64_t sample_begin, uint32_t batch, uint32_t n_batches,
                                              float* const* outs_dev, void* stream) {
    if (!c || !tiles || !outs_dev || batch == 0) return RT_ERR_INVALID_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t cs = static_cast<hipStream_t>(stream);
    HIPCHK(c, hipEventRecord(c->caller_ev, cs));
    int st = render_batches_impl(c, tiles, n_tiles, sample_begin, batch, n_batches,
                                 reinterpret_cast<float4* const*>(outs_dev), c->caller_ev);
    if (st) return st;
    if (c->last_fold) HIPCHK(c, hipStreamWaitEvent(cs, c->last_fold, 0));
    return RT_OK;
}

extern "C" int rt_render_device(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles,
                                uint64_t sample_begin, uint32_t sample_count, float* out_dev) {
    if (!c || !tiles || !out_dev) return RT_ERR_INVALID_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    int st = sync_all(c);
    if (st) return st;
    // ordered after the legacy default stream's work (e.g. the caller's allocation / clearing of
    // out_dev), and complete on return
    HIPCHK(c, hipEventRecord(c->caller_ev, nullptr));
    if ((st = render_impl(c, tiles, n_tiles, sample_begin, sample_count, reinterpret_cast<float4*>(out_dev),
                          c->caller_ev)))
        return st;
    return sync_all(c);
}

extern "C" int rt_synchronize(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    return sync_all(c);
}

extern "C" int rt_last_kernel_ms(const rt_ctx* c, float* ms) {
    if (!c || !ms) return RT_ERR_INVALID_ARG;
    *ms = c->last_ms;
    return RT_OK;
}

extern "C" int rt_last_launch_stats(const rt_ctx* c, rt_launch_stats* out) {
    if (!c || !out) return RT_ERR_INVALID_ARG;
    out->render_ms = c->last_ms;
    out->trace_ms = c->trace_ms;
    out->n_trace_launches = c->n_launch;
    out->n_timed_launches = c->n_timed;
    return RT_OK;
}

extern "C" int rt_count_work(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                             uint32_t sample_count, rt_work_counts* out) {
    return rt_count_work_ex(c, tiles, n_tiles, sample_begin, sample_count, RT_COUNT_REFERENCE, out);
}

extern "C" int rt_count_work_ex(rt_ctx* c, const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                                uint32_t sample_count, uint32_t mode, rt_work_counts* out) {
    if (!c || !tiles || !out || mode > RT_COUNT_DEVICE) return RT_ERR_INVALID_ARG;
    HIPCHK(c, hipSetDevice(c->device));
    int st = sync_all(c);
    if (st) return st;
    LaunchArgs a{};
    uint64_t n_out = 0;
    st = prepare_tiles(c, tiles, n_tiles, choose_k(c, tile_pixels(tiles, n_tiles)), &a, &n_out);
    if (st) return st;
    a.sample_begin = sample_begin;
    a.sample_count = sample_count;
    a.counts = c->d_counts;
    a.sc.count_device = mode == RT_COUNT_DEVICE ? 1u : 0u;
    HIPCHK(c, hipMemsetAsync(c->d_counts, 0, sizeof(DevCounts), c->stream));
    if (sample_count) HIPCHK(c, launch_trace_count(a, c->stream));
    DevCounts h{};
    HIPCHK(c, hipMemcpyAsync(&h, c->d_counts, sizeof(DevCounts), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    out->samples = h.samples; out->segments = h.segments; out->nodes = h.nodes;
    out->leaf_refs = h.leaf_refs; out->sphere_tests = h.sphere_tests; out->tri_tests = h.tri_tests;
    out->hits = h.hits; out->mesh_hits = h.mesh_hits;
    return RT_OK;
}

extern "C" const char* rt_last_error(const rt_ctx* c) { return c ? c->err.c_str() : "null context"; }

extern "C" int rt_destroy(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID_ARG;
    destroy_ctx(c);
    return RT_OK;
}

// render_to_target_gpu (draw_scene.rs:17-47) on one device: spp/batch batches over the whole
// frame; after each, the RGBA8 target is refreshed and the update hook runs, in batch order.
// Consecutive batches are traced together (render_batches_impl): a group of G batches is one
// trace launch of at least GROUP_ITEMS samples, folded batch by batch, so a small batch (a380's
// gpu_render_batch of 1 spp: 0.72 M samples, ~2 ms of work against a ~10 ms drain tail) no longer
// needs a pipeline slot, and a hardware queue, of its own: the throughput does not depend on the
// caller's GPU_MAX_HW_QUEUES.  Pipelined: group g + 1 is enqueued before group g's frames are
// read back, converted and handed to the hook, so the device never waits on the host and group
// g + 1's launch fills group g's drain tail.  The frames are those of one launch per batch.
constexpr uint64_t GROUP_ITEMS = 1ull << 24;
extern "C" int rt_render_to_target(const rt_scene_desc* scene, const rt_camera* cam,
                                   const rt_render_info* info, uint32_t spp, uint32_t batch, int device,
                                   uint8_t* target, rt_update_hook hook, void* user) {
    if (!scene || !cam || !info || !target || batch == 0) return RT_ERR_INVALID_ARG;
    if (spp % batch != 0) return RT_ERR_BATCH;
    rt_ctx* c = nullptr;
    int st = rt_create(scene, cam, info, nullptr, device, &c);
    if (st) return st;
    const rt_tile full{0, 0, info->width, info->height};
    const uint64_t npix = (uint64_t)info->width * info->height;
    const uint32_t n_batch = spp / batch;
    const uint64_t per_batch = npix * batch;
    const uint64_t group_items = c->group_items ? c->group_items : GROUP_ITEMS;
    const uint32_t G = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_batch, group_items / per_batch));
    // groups in flight beyond the one being read back: a small group launch rotates over the
    // small-launch slots, a larger one over two
    const uint64_t gitems = per_batch * G;
    const uint32_t ahead = (c->n_slots ? c->n_slots
                                       : (gitems <= c->small_items ? c->small_slots
                                                                   : (gitems <= MID_LAUNCH_ITEMS ? c->mid_slots : 2u))) - 1u;
    const uint32_t ring = (uint32_t)std::min<uint64_t>(n_batch, (uint64_t)G * (ahead + 1));
    std::vector<float4*> dbuf;
    std::vector<hipEvent_t> done;
    auto run = [&]() -> int {
        std::vector<float> rgba(npix * 4);
        dbuf.assign(ring, nullptr);
        done.assign(ring, nullptr);
        for (uint32_t k = 0; k < ring; ++k) {
            if (hipMalloc(&dbuf[k], npix * sizeof(float4)) != hipSuccess) return set_err(c, RT_ERR_OOM, "output alloc failed");
            HIPCHK(c, hipEventCreateWithFlags(&done[k], hipEventDisableTiming));
        }
        uint32_t delivered = 0;
        auto deliver_to = [&](uint32_t end) -> int {  // batches [delivered, end), in order
            for (; delivered < end; ++delivered) {  // batch b's frame: samples [0, (b + 1) * batch)
                const uint32_t k = delivered % ring;
                HIPCHK(c, hipEventSynchronize(done[k]));
                HIPCHK(c, hipMemcpy(rgba.data(), dbuf[k], npix * sizeof(float4), hipMemcpyDeviceToHost));
                rt_rgba_to_u8(rgba.data(), npix, target);
                if (hook) hook(user, (delivered + 1) * batch);
            }
            return RT_OK;
        };
        std::vector<float4*> outs(G);
        for (uint32_t g0 = 0; g0 < n_batch; g0 += G) {
            const uint32_t gn = std::min(G, n_batch - g0);
            // the buffers this group reuses hold batches g0 + gn - 1 - ring and earlier
            int r = deliver_to(g0 + gn > ring ? g0 + gn - ring : 0u);
            if (r) return r;
            for (uint32_t k = 0; k < gn; ++k) outs[k] = dbuf[(g0 + k) % ring];
            if ((r = render_batches_impl(c, &full, 1, (uint64_t)g0 * batch, batch, gn, outs.data(), nullptr))) return r;
            for (uint32_t k = 0; k < gn; ++k) HIPCHK(c, hipEventRecord(done[(g0 + k) % ring], c->slot[c->cur_slot].stream));
        }
        return deliver_to(n_batch);
    };
    st = guarded(c, run);
    if (!st) st = sync_all(c);
    for (size_t k = 0; k < dbuf.size(); ++k) {
        if (done[k]) (void)hipEventDestroy(done[k]);
        if (dbuf[k]) {
            (void)sync_all(c);
            (void)hipFree(dbuf[k]);
        }
    }
    rt_destroy(c);
    return st;
}
