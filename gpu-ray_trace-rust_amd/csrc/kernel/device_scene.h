// device_scene.h — the scene as laid out in HBM for the gfx950 megakernel.
// Shared by the host runtime (upload) and the kernel (reads).  Not part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtd {

constexpr int BLOCK = 128;       // threads per workgroup: 16 x (BLOCK/16) pixels at K = 1
constexpr int LDS_SPHERES = 64;  // the sphere-only kernel's LDS sphere tables (1 KiB each)
constexpr int BLOCK_W = 16;
constexpr int BLOCK_H = BLOCK / BLOCK_W;
constexpr int MAX_STACK = 64;    // deepest KD tree the device path accepts (stack in LDS)

// Leaf node (rt_kd_node {count, (offset << 2) | 3}) on the device: the low 24 bits of the first
// word hold the ref count, the top 8 the number of sphere refs that open the leaf's list (refs
// keep renderable order, where spheres usually precede every triangle; 0 when it does not fit).
constexpr uint32_t LEAF_COUNT_MASK = (1u << 24) - 1u;
constexpr uint32_t LEAF_LEAD_SHIFT = 24;

// Device ref encoding: kind in the top 2 bits, index into the kind's arrays below.
constexpr uint32_t REF_KIND_SHIFT = 30;
constexpr uint32_t REF_INDEX_MASK = (1u << 30) - 1u;
enum : uint32_t { K_SPHERE = 0, K_FREE_TRI = 1, K_MESH_TRI = 2 };

// Shading record of a sphere / free triangle (UniformDiffuseSpec + Coloring).  72 bytes.
struct DevMat {
    float rgb[3];
    float em[3];       // zero when the material has no emissive (sphere.rs:70-75)
    uint32_t divert;   // rt_divert
    float diffp;
    float n_out, n_in;
    // Dielectric constants of refract (interaction.rs:29-59), computed on the host with the
    // same f32 operations: n_out / n_in, n_in / n_out, and r0 = q * q with
    // q = (n1 - n2) / (n1 + n2) — the same value entering or leaving (q changes sign only).
    float over_in, over_out, r0;
    float rgb_atten[3];  // rgb / 0.4 (radiance.rs:44's 1/atten with p = 1), same f32 division
    uint32_t _pad[2];
};

struct DevFace {       // one DistantCubeMap face: texel offset, size, uv scales
    uint32_t off, w, h;
    float us, vs;
};

struct DevTex {        // one UVRgb32FImage in the texel pool (f32 RGB)
    uint32_t off, w, h, _pad;
};

struct DevPrim {       // per glTF primitive (Mesh RgbInfo / NormInfo / PbrMetalRoughInfo)
    float base_factor[3];
    int32_t base_tex;   // -1: factor only
    int32_t normal_tex; // -1: interpolated vertex normals
    int32_t mr_tex;     // -1: metal / rough factors
    float metal, rough;
};

struct DevMeshTri {    // 64 bytes, same layout as rth::FlatTri
    uint32_t prim;
    uint32_t v[3];     // global vertex indices into the vertex pools
    float m[9];        // normal transform, row-major (x normal_scale with a normal map)
    uint32_t _pad[3];
};

struct DevScene {
    // KD tree (rt_kd_node layout), breadth-first
    const uint2* nodes;
    const uint32_t* refs;   // device-encoded refs
    uint32_t n_nodes;
    uint32_t stack_depth;   // traversal stack entries per lane (>= max_leaf_depth, >= 1)
    uint32_t spheres_only;  // no free / mesh triangles: launch the sphere-only kernel
    uint32_t fastdiv;       // every split is 0 or in [2^-70, 2^61): Markstein division allowed
    uint32_t count_device;  // instrumented launch counts the device path (not the reference's)
    uint32_t small_ok;      // closest_small allowed: coordinates below 2^58 (finite roots), r >= 0, sphere boxes inside bounds
    uint32_t restart;       // queue kernels: 0 stack, 1 stackless (kd-restart with push-down)
    uint32_t packet;        // general queue kernel: camera rays may be traced as packets (closest_packet)
    float bounds[6];
    // spheres
    const float4* sph;      // c.xyz, r
    const DevMat* sph_mat;
    uint32_t n_spheres;
    // free triangles
    // Leaf-testable primitives, 3 float4 each, indexed by a device ref's index:
    // [spheres: {c, r}, 0, 0][free triangles: v0, e1, e2][mesh triangles: v0, e1, e2], with the
    // Moller-Trumbore edges e1 = v1 - v0, e2 = v2 - v0 computed on the host by the same f32
    // subtraction generic.rs:104-105 performs per test.
    // A ref's index is its pool position; per-kind arrays below take index - pool_<kind>.
    const float4* prim4;
    uint32_t pool_ftri, pool_mesh;
    // direct-light sampling (dir_light_samp): renderables in renderable order (device refs) and
    // the emissive spheres {sphere index, position in elem_refs}
    const uint32_t* elem_refs;
    const uint2* emit;
    uint32_t n_elem_refs, n_emit, dls;
    const float4* ftri_n;   // uniform normal
    const DevMat* ftri_mat;
    // mesh triangles (src/elements/mesh)
    const DevMeshTri* mtri;
    const DevPrim* prims;
    const float4* vnorm;    // per global vertex
    const float2* uv_base;
    const float2* uv_norm;
    const float2* uv_mr;
    // textures
    const DevTex* tex;
    // The texel pool of every scene texture: f32 RGB (texels), or — when every texel channel is
    // some k / 255 in f32, as image::to_rgb32f makes them (uv_image.rs:9-23, model.rs:204) —
    // one RGBA8 word per texel (texels8, A unused), decoded as k / 255 bit for bit.
    const float* texels;
    const uint32_t* texels8;
    // cube map (first unconditional renderable, distant_cube_map.rs); has_cube == 0: misses are black
    uint32_t has_cube;
    DevFace face[6];
    // camera (RayCompute, generate.rs:13-23, precomputed on host)
    float cam_d[3], cam_o[3], cam_up[3], right[3];
    float x_cf, y_cf, x_off, y_off;
    uint32_t has_lens;
    float lens_r;
    uint32_t width, height;
    int32_t assured_depth;
    uint32_t debug_single_ray;
    uint64_t seed;
};

struct DevTile {
    uint32_t x0, y0, w, h;
    uint32_t out_off;       // first output pixel of the tile
    uint32_t block_begin;   // first workgroup of the tile
    uint32_t bx;            // workgroups per tile row
    uint32_t _pad;
};

struct DevCounts {
    unsigned long long samples, segments, nodes, leaf_refs, sphere_tests, tri_tests, hits, mesh_hits;
};

struct LaunchArgs {
    DevScene sc;
    const DevTile* tiles;
    uint32_t n_tiles;
    const uint32_t* pix_xy; // launch pixel o -> (y << 16) | x; nullptr for frames over 65535 wide/high
    // Queue order of the launch pixels (with pix_xy): the queue kernel's q-th pixel of a sample
    // is {(y << 16) | x, o, key}, 8 x 8 blocks of each tile in turn, so a wave's consecutive items
    // are a compact block of the frame (coherent camera rays for closest_packet); key (low, high
    // word) is the pixel's stream key rt_rng_pixel_key(seed, y * width + x), so a path start
    // makes one SplitMix64 round instead of two.  nullptr: q = o.
    const uint4* pix_q;
    uint32_t n_blocks;
    uint64_t sample_begin;
    uint32_t sample_count;
    // The running mean's n for absolute sample s is s - mean_base: 0 for rt_render's cumulative
    // mean (draw_scene.rs:81-83), the call's first sample for rt_render_range's per-call mean.
    uint64_t mean_base;
    float4* accum;          // width*height running means
    float4* out;            // tile-concatenated output (may alias nothing)
    DevCounts* counts;      // instrumented launch only
    // K lanes per pixel (power of two <= BLOCK_H).  K == 1: each lane folds its pixel's samples
    // in registers.  K > 1: lane k traces samples sample_begin + k + K*j into `radiance`
    // ([sample][launch pixel] x RGB) and fold_kernel applies the running mean in sample order.
    uint32_t lanes_per_pixel;
    uint32_t n_pix;         // pixels of the launch (tiles concatenated)
    uint32_t n_pix_magic;   // floor(2^32 / n_pix) (0 for n_pix = 1): item / n_pix by multiply-high
    float* radiance;
    // Queue schedule (launch_trace_queue): persistent lanes take (pixel, sample) items
    // item = j * n_pix + o (sample j of the launch, output pixel o) in wave-sized grabs from the
    // counters of its n_shards shards (queue[k * 32], one 128-B line each, zeroed before the
    // launch), trace them into `radiance` and fold_kernel folds them in sample order.
    uint32_t* queue;
    uint32_t n_shards;      // 1..32 (runtime.hip queue_shards)
    uint32_t n_items;       // n_pix * sample_count
    // Sphere-only queue kernel: its traversal stack in global memory, [block][stack_depth][BLOCK]
    // (queue_gstack_bytes), so the workgroup's LDS holds only the sphere and material tables.
    uint32_t* gstack;
};

// Launch wrappers (trace.hip).
hipError_t launch_trace(const LaunchArgs& a, hipStream_t s);
hipError_t launch_trace_count(const LaunchArgs& a, hipStream_t s);
hipError_t launch_fold(const LaunchArgs& a, hipStream_t s);
hipError_t launch_trace_queue(const LaunchArgs& a, uint32_t n_blocks, hipStream_t s);
hipError_t queue_blocks_per_cu(const LaunchArgs& a, int* blocks);
size_t queue_gstack_bytes(const LaunchArgs& a, uint32_t n_blocks);  // 0: the stack is in LDS
uint32_t queue_block_threads(const LaunchArgs& a);  // threads per workgroup of the scene's queue kernel

}  // namespace rtd
