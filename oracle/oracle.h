/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's CPU render path (joonhosung/GPU-Ray_Trace-Rust,
 * render_to_target_cpu, src/render/draw_scene.rs:49-101, and everything it calls) used as the
 * parity checker for the HIP device path and as the timed CPU baseline in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product path (gpu-ray_trace-rust_amd/) never links or calls it.
 *
 * Parity pinning: the Rust reference cannot be built here (no rustc/cargo, crates not
 * vendored — SURVEY.md §8c), so the restatement is pinned by the reference's own unit tests
 * (aabb.rs:71-121, hit.rs:94-140, target.rs:23-46, restated in tests/test_oracle_kat.py) and,
 * beyond those, is "parity unpinned" against the Rust binary itself.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>
#include "../include/rt_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Accumulation form of radiance():
 * 0 = recursive, exactly the reference's L = e + f (x) L_next (radiance.rs:44,59);
 * 1 = forward, L += T (x) e; T *= f — the device path's order. */
enum { ORACLE_ACCUM_RECURSIVE = 0, ORACLE_ACCUM_FORWARD = 1 };

typedef struct oracle_counts {
    uint64_t samples, segments;
    uint64_t nodes, leaf_refs;
    uint64_t sphere_tests, tri_tests;
    uint64_t hits, mesh_hits;
} oracle_counts;

/* Renders samples [sample_begin, sample_begin + sample_count) of every pixel in tiles with the
 * reference's per-pixel running mean.  out_rgba (tiles concatenated, row-major RGBA f32) is
 * read as the accumulator when sample_begin > 0 and holds the result on return.
 * threads <= 0: all hardware threads.  counts may be NULL. */
int oracle_render(const rt_scene_desc* scene, const rt_camera* cam, const rt_render_info* info,
                  const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                  uint32_t sample_count, int threads, int accum_mode, float* out_rgba,
                  oracle_counts* counts);

/* oracle_render with the running mean's n = sample - mean_base (mean_base <= sample_begin):
 * mean_base = sample_begin gives the mean over this call's samples alone (one batch of the
 * reference's GPU path, trace.wgsl:277-318); out_rgba is read as the accumulator only when
 * sample_begin > mean_base. */
int oracle_render_ex(const rt_scene_desc* scene, const rt_camera* cam, const rt_render_info* info,
                     const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                     uint32_t sample_count, int threads, int accum_mode, uint64_t mean_base,
                     float* out_rgba, oracle_counts* counts);

/* Shading mix of the counted renders (counts != NULL) since the last reset: continued rays by
 * material branch {spec, diff, diffspec->diff, diffspec->spec, dielectric}, Russian-roulette
 * draws, all draws, mesh continues, positive discriminants, then ORACLE_MIX_DEPTHS bins of branch
 * nodes stepped through per depth: ORACLE_MIX_N entries in all. */
#define ORACLE_MIX_DEPTHS 40
#define ORACLE_MIX_N (9 + ORACLE_MIX_DEPTHS)
void oracle_mix_counts(uint64_t out[ORACLE_MIX_N], int reset);

/* KdTree::build (kdtree.rs:26-56,107-137) as a pointer tree, then a canonical depth-first
 * pre-order dump: per node {is_leaf, axis, split bits | leaf count, first ref}; refs in
 * leaf order.  Returns number of nodes; call with NULL buffers to size. */
int oracle_kd_dump(const rt_scene_desc* scene, uint32_t max_depth, uint32_t* node_rows /*4/node*/,
                   uint32_t node_cap, uint32_t* refs, uint32_t ref_cap, uint32_t* n_refs,
                   float bounds[6]);

/* Per-mesh-triangle normal transform (NormFromMesh::generate_norm_type,
 * mesh/triangle.rs:45-122), row-major 3x3 per triangle in renderable order. */
int oracle_mesh_normal_transforms(const rt_scene_desc* scene, float* out9, uint64_t cap);

/* Known-answer hooks (one reference function each). */
int   oracle_aabb_entry_exit(const float bounds[6], const float d[3], const float o[3],
                             int* min_axis, float* entry, int* max_axis, float* exit_t);
int   oracle_raylen_cmp(float a, float b);                       /* hit.rs:50-76 */
void  oracle_chunk_to_pix(int32_t idx, int32_t width, int32_t* x, int32_t* y); /* target.rs:9-14 */
int   oracle_sphere_intersect(const float c[3], float r, const float d[3], const float o[3],
                              float* l);                          /* sphere.rs:83-105 */
int   oracle_triangle_intersect(const float v[9], const float d[3], const float o[3],
                                float* l, float* u, float* v_out); /* generic.rs:102-137 */
void  oracle_rng_stream(uint64_t seed, uint32_t pixel, uint64_t sample, uint32_t n, float* out);
void  oracle_camera_ray(const rt_camera* cam, uint32_t w, uint32_t h, int32_t x, int32_t y,
                        uint64_t seed, uint64_t sample, float d_out[3], float o_out[3]);
void  oracle_refract(const float d[3], const float n[3], float n_out, float n_in, float u,
                     float d_out[3], float* p);                   /* interaction.rs:29-59 */

#ifdef __cplusplus
}
#endif
#endif
