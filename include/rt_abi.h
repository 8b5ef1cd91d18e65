/*
 * rt_abi.h — C ABI of the MI355X (gfx950) per-pixel path-tracing hot path.
 *
 * This is the drop-in boundary that replaces the reference's wgpu batch dispatcher
 * (joonhosung/GPU-Ray_Trace-Rust):
 *   - render_to_target_gpu            src/render/draw_scene.rs:17-47   -> rt_render_to_target
 *   - GPUState::new                   src/render/gpu_utils.rs:613-640  -> rt_create (device pick)
 *   - GPUState::create_compute_pipeline gpu_utils.rs:642-652 (+ ComputePipeline::new :257-587,
 *     create_mesh_buffers :87-156, create_renderables_buffer :158-254) -> rt_create (upload)
 *   - dispatch_compute_pipeline / submit_compute_pipeline gpu_utils.rs:654-679 -> rt_render
 *   - block_and_get_single_result     gpu_utils.rs:681-724             -> rt_render(out_rgba)
 *   - GPUElements tuple               src/types.rs:7                   -> rt_scene_desc
 *   - scene::Cam                      src/scene.rs:7-15                -> rt_camera
 *   - RenderInfo / RadianceInfo       src/render/cpu_utils.rs:4-15, radiance.rs:8-18 -> rt_render_info
 *   - KdTree::build                   src/accel/kdtree.rs:26-56,107-137 -> rt_kd_build
 *
 * Plain C: fixed-width integers, floats and pointers only, no torch/HIP types, so a Rust
 * caller can bind it unchanged with bindgen.  Nothing throws across
 * the ABI: every entry point returns an rt_status (0 = success, negative = error).
 *
 * Determinism contract (new; the reference's RNG is unseeded, src/lib.rs:25-27):
 * the value of a pixel depends only on (scene, camera, render_info incl. seed, pixel,
 * absolute sample range) — never on tiling, batching, device or device count.
 * The per-(pixel, sample) random stream is defined in rt_rng.h.
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 1

/* ---------------------------------------------------------------- status */
typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = -1,   /* bad pointer / size / index (reference: assert!/expect panics) */
    RT_ERR_OOM = -2,           /* host or device allocation failed */
    RT_ERR_HIP = -3,           /* a HIP runtime call failed (message in rt_last_error) */
    RT_ERR_UNSUPPORTED = -4,   /* beyond the device path (a KD tree deeper than its 64-entry stack) */
    RT_ERR_NO_DEVICE = -5,     /* no gfx950 device / bad device ordinal */
    RT_ERR_BATCH = -6          /* spp % batch != 0 (reference panic, src/renderer.rs:56-57) */
} rt_status;

/* ------------------------------------------------------------- materials */
/* DivertRayMethod, src/material/uniform_diff_spec.rs:13-19 */
typedef enum rt_divert {
    RT_DIVERT_SPEC = 0,
    RT_DIVERT_DIFF = 1,
    RT_DIVERT_DIFFSPEC = 2,    /* DiffSpec { diffp } */
    RT_DIVERT_DIELECTRIC = 3   /* Dielectric { n_out, n_in } */
} rt_divert;

/* UniformDiffuseSpec, src/material/uniform_diff_spec.rs:7-11.  32 bytes. */
typedef struct rt_material {
    float    emissive[3];      /* Option<Vector3<f32>>; ignored unless has_emissive */
    uint32_t has_emissive;
    uint32_t divert;           /* rt_divert */
    float    diffp;            /* DiffSpec */
    float    n_out, n_in;      /* Dielectric */
} rt_material;

/* ------------------------------------------------------------ primitives */
/* Sphere, src/elements/sphere.rs:20-29 (Coloring::Solid).  64 bytes. */
typedef struct rt_sphere {
    float       c[3];
    float       r;
    float       rgb[3];
    uint32_t    _pad0;
    rt_material mat;
} rt_sphere;

/* FreeTriangle, src/elements/triangle/free.rs:7 + builder/inner.rs:44-53.  96 bytes.
 * norm must already be normalised (the reference normalises it at load, inner.rs:48). */
typedef struct rt_free_triangle {
    float       verts[3][3];
    float       norm[3];
    float       rgb[3];
    uint32_t    _pad0;
    rt_material mat;
} rt_free_triangle;

/* UVRgb32FImage, src/material/uv_image.rs:4-23: row-major f32 RGB texels, texel (x, y) at
 * rgb[3 * (y * width + x)], values as produced by image::to_rgb32f (u8 -> x / 255.0). */
typedef struct rt_texture {
    uint32_t     width, height;
    const float* rgb;
} rt_texture;

/* FaceImagewUVScale, src/elements/distant_cube_map.rs:7 */
typedef struct rt_cube_face {
    int32_t texture;           /* index into rt_scene_desc.textures */
    float   us, vs;
} rt_cube_face;

/* DistantCubeMap, src/elements/distant_cube_map.rs:10-17 */
enum { RT_FACE_NEG_X = 0, RT_FACE_POS_X, RT_FACE_NEG_Y, RT_FACE_POS_Y, RT_FACE_NEG_Z, RT_FACE_POS_Z };
typedef struct rt_cube_map {
    rt_cube_face face[6];      /* indexed by RT_FACE_* */
} rt_cube_map;

/* One glTF primitive of a Mesh, src/elements/mesh/mesh.rs:10-25 / builder/pr/model.rs:77-131.
 * Optional arrays are NULL (and textures -1) when the glTF primitive lacks them. */
typedef struct rt_mesh_prim {
    uint32_t        n_verts, n_tris;
    const float*    poses;            /* n_verts*3, already multiplied by trans_mat (model.rs:86-90) */
    const float*    norms;            /* n_verts*3, untransformed (model.rs:121) */
    const uint32_t* indices;          /* n_tris*3 */
    const float*    tangents;         /* n_verts*3 or NULL (model.rs:111) */
    float           base_color_factor[3];
    int32_t         base_color_tex;   /* -1: none */
    const float*    base_color_uv;    /* n_verts*2 or NULL */
    int32_t         normal_tex;       /* -1: no NormInfo */
    float           normal_scale;
    const float*    normal_uv;
    int32_t         metal_rough_tex;  /* -1: none */
    const float*    metal_rough_uv;
    float           metal, rough;     /* PbrMetalRoughInfo factors */
} rt_mesh_prim;

typedef struct rt_mesh {
    float               trans_mat[16];  /* column-major 4x4 (nalgebra storage order) */
    uint32_t            n_prims;
    const rt_mesh_prim* prims;
} rt_mesh;

/* Renderable order (src/render/draw_scene.rs:57-58, 112-130): the non-mesh elements in
 * YAML order, then every mesh triangle (mesh, primitive, triangle). */
enum { RT_ELEM_SPHERE = 0, RT_ELEM_FREE_TRI = 1, RT_ELEM_CUBE_MAP = 2 };
typedef struct rt_elem {
    uint32_t kind;             /* RT_ELEM_* */
    uint32_t index;            /* into the array of that kind */
} rt_elem;

typedef struct rt_scene_desc {
    uint32_t                n_elems;
    const rt_elem*          elems;
    uint32_t                n_spheres;
    const rt_sphere*        spheres;
    uint32_t                n_free_tris;
    const rt_free_triangle* free_tris;
    uint32_t                n_cube_maps;
    const rt_cube_map*      cube_maps;
    uint32_t                n_meshes;
    const rt_mesh*          meshes;
    uint32_t                n_textures;
    const rt_texture*       textures;
} rt_scene_desc;

/* -------------------------------------------------------- camera / info */
/* scene::Cam after From<pr::Cam> (src/builder/pr/cam.rs:19-81) and apply_corrections
 * (src/builder/mod.rs:69-72); use rt_camera_from_scheme to produce it. */
typedef struct rt_camera {
    float    d[3];             /* o -> screen centre, unnormalised (its length sets the FOV) */
    float    o[3];
    float    up[3];
    float    screen_width, screen_height;
    uint32_t has_lens;
    float    lens_r;
} rt_camera;

typedef struct rt_render_info {
    uint32_t width, height;
    uint32_t kd_tree_depth;    /* RenderInfo::kd_tree_depth */
    int32_t  assured_depth;    /* RussianRoullInfo::assured_depth */
    float    max_thres;        /* parsed but unused: radiance.rs:77 uses a static 0.4 */
    uint32_t debug_single_ray; /* RadianceInfo::debug_single_ray */
    uint32_t dir_light_samp;   /* RadianceInfo::dir_light_samp (radiance.rs:46-56,89-120) */
    uint32_t _pad0;
    uint64_t seed;             /* rt_rng.h stream key */
} rt_render_info;

/* A rectangle of pixels; y grows with the reference's row index (target.rs:9-14). */
typedef struct rt_tile {
    uint32_t x0, y0, w, h;
} rt_tile;

/* ------------------------------------------------------------- KD tree */
/* Flattened KdTree (src/accel/kdtree.rs:14-23), 8 bytes per node.
 * Branch: a = bits of split (f32), b = (low_child << 2) | axis; high child = low_child + 1.
 * Leaf:   a = number of refs,       b = (ref_offset << 2) | 3.
 * refs[] hold renderable indices, in renderable order inside each leaf (kdtree.rs:119-127).
 * Node 0 is the root. */
typedef struct rt_kd_node {
    uint32_t a, b;
} rt_kd_node;

#define RT_KD_LEAF 3u

typedef struct rt_kd_tree {
    uint32_t          n_nodes, n_refs;
    uint32_t          max_leaf_depth;  /* deepest leaf (root = 0); traversal stack <= this + 1 */
    uint32_t          n_unconditional; /* renderables without AABB (cube maps) */
    float             bounds[6];       /* root Aabb: x.low, x.high, y.low, y.high, z.low, z.high */
    const rt_kd_node* nodes;
    const uint32_t*   refs;
    const uint32_t*   unconditional;   /* renderable indices, renderable order */
} rt_kd_tree;

/* Device-side work counters (for the roofline's algorithmic bytes). */
typedef struct rt_work_counts {
    uint64_t samples, segments;
    uint64_t nodes, leaf_refs;
    uint64_t sphere_tests, tri_tests;
    uint64_t hits, mesh_hits;
} rt_work_counts;

typedef struct rt_ctx rt_ctx;

/* ----------------------------------------------------------- functions */
int         rt_abi_version(void);
const char* rt_status_string(int status);
int         rt_device_count(int* n);

/* Camera conversion (src/builder/pr/cam.rs:19-81, builder/mod.rs:69-72): up <- normalize(up),
 * R = from_euler_angles(r, p, y) (nalgebra Rotation3), d <- R d, up <- R up. */
int rt_camera_from_scheme(const float d[3], const float o[3], const float up[3],
                          float screen_width, float screen_height,
                          uint32_t has_lens, float lens_r,
                          const float view_eulers[3], rt_camera* out);

/* Host KD build, bit-for-bit KdTree::build(elems_and_aabbs, unconditional, max_depth)
 * (kdtree.rs:26-56,107-137) over the renderables of `scene`.  Free with rt_kd_free. */
int  rt_kd_build(const rt_scene_desc* scene, uint32_t max_depth, rt_kd_tree** out);
void rt_kd_free(rt_kd_tree* tree);

/* Deep-copies the scene (and `tree`, or builds one with info->kd_tree_depth when NULL)
 * to device `device`; the caller may free its inputs on return. */
int rt_create(const rt_scene_desc* scene, const rt_camera* cam, const rt_render_info* info,
              const rt_kd_tree* tree, int device, rt_ctx** out);

/* Advances every pixel of `tiles` from sample `sample_begin` to sample_begin+sample_count.
 * The per-pixel accumulator is the reference's running mean p <- (r + p*n)/(n+1) with n the
 * absolute sample index (draw_scene.rs:81-83), so split batches equal one batch bit-for-bit;
 * sample_begin == 0 resets it.  When out_rgba != NULL the resulting means are copied there as
 * RGBA f32 (alpha 1), tiles concatenated, each row-major.  Synchronous. */
int rt_render(rt_ctx* ctx, const rt_tile* tiles, uint32_t n_tiles,
              uint64_t sample_begin, uint32_t sample_count, float* out_rgba);

/* Same, but the output goes to device memory on the ctx's device (for RCCL gathers); ordered
 * after the work already enqueued on the legacy default stream (the caller's allocation of
 * out_rgba_device, a gather still reading it), and complete on return. */
int rt_render_device(rt_ctx* ctx, const rt_tile* tiles, uint32_t n_tiles,
                     uint64_t sample_begin, uint32_t sample_count, float* out_rgba_device);

/* Asynchronous rt_render_device: enqueues the call and returns.  `stream` is the caller's
 * hipStream_t (NULL: the legacy default stream): what the caller enqueued on it before the call
 * completes before the output is written, and what it enqueues after the call (a gather, a copy)
 * sees the finished output.  Consecutive calls overlap on the device: call i + 1's trace starts
 * while call i's last paths drain (draw_scene.rs:30-44's batches are independent sample ranges;
 * only their running-mean folds are ordered).  Results equal the synchronous calls bit for bit.
 * Stats (rt_last_launch_stats) cover every call since the previous rt_synchronize. */
int rt_render_device_async(rt_ctx* ctx, const rt_tile* tiles, uint32_t n_tiles,
                           uint64_t sample_begin, uint32_t sample_count, float* out_rgba_device,
                           void* stream);

/* The batch loop of render_to_target_gpu (draw_scene.rs:30-44) on the device, asynchronous like
 * rt_render_device_async: n_batches consecutive batches of `batch` samples from sample_begin;
 * after batch k the running mean over [0, sample_begin + (k + 1) * batch) is written to
 * outs_dev[k] (device memory; NULL: that frame is not written, the accumulator still advances).
 * The frames equal n_batches rt_render_device_async calls bit for bit.  The batches are traced by
 * as few launches as the radiance buffer allows and folded batch by batch, so small batches (a
 * 1-spp batch of a 1200x600 frame) keep the GPU busy without one pipeline stream, and HIP
 * hardware queue, per batch in flight (GPU_MAX_HW_QUEUES does not matter). */
int rt_render_batches_device_async(rt_ctx* ctx, const rt_tile* tiles, uint32_t n_tiles,
                                   uint64_t sample_begin, uint32_t batch, uint32_t n_batches,
                                   float* const* outs_dev, void* stream);

/* The mean over samples [sample_begin, sample_begin + sample_count) alone, per pixel of `tiles`
 * (RGBA f32, alpha 1, tiles concatenated): what one batch of the reference's GPU path returns
 * (block_and_get_single_result, gpu_utils.rs:681-724, whose kernel folds the batch with a
 * running mean from zero, trace.wgsl:277-318) before render_to_target_gpu folds batches into its
 * running mean (draw_scene.rs:36).  Uses the same per-(pixel, absolute sample) streams as
 * rt_render; the context's cumulative mean is not touched.  Synchronous. */
int rt_render_range(rt_ctx* ctx, const rt_tile* tiles, uint32_t n_tiles,
                    uint64_t sample_begin, uint32_t sample_count, float* out_rgba);

/* Waits for every enqueued call of the ctx and closes its timing window. */
int rt_synchronize(rt_ctx* ctx);

/* Device time (ms) of the last synchronous rt_render* call (or of the async calls up to the
 * last rt_synchronize), first trace launch to last fold, from HIP events. */
int rt_last_kernel_ms(const rt_ctx* ctx, float* ms);

/* Per-launch breakdown of the last rt_render* call: the trace kernel launches alone (HIP events
 * around each one), their count, and the whole call.  Samples per trace launch follow from the
 * call's pixels x samples / n_trace_launches. */
typedef struct rt_launch_stats {
    float render_ms;            /* same as rt_last_kernel_ms */
    float trace_ms;             /* sum over the trace kernel launches */
    uint32_t n_trace_launches;
    uint32_t n_timed_launches;  /* launches in trace_ms: the first 256 of a window (async calls
                                   without rt_synchronize keep the event pool bounded) */
} rt_launch_stats;
int rt_last_launch_stats(const rt_ctx* ctx, rt_launch_stats* out);

/* Instrumented run: counts work instead of timing it (accumulator untouched).
 * RT_COUNT_REFERENCE: the reference algorithm's work (full stack_search, kdtree.rs:66-104);
 * RT_COUNT_DEVICE: what the device path actually does (e.g. the small-scene bound). */
enum { RT_COUNT_REFERENCE = 0, RT_COUNT_DEVICE = 1 };
int rt_count_work(rt_ctx* ctx, const rt_tile* tiles, uint32_t n_tiles,
                  uint64_t sample_begin, uint32_t sample_count, rt_work_counts* out);
int rt_count_work_ex(rt_ctx* ctx, const rt_tile* tiles, uint32_t n_tiles, uint64_t sample_begin,
                     uint32_t sample_count, uint32_t mode, rt_work_counts* out);

const char* rt_last_error(const rt_ctx* ctx);
int         rt_destroy(rt_ctx* ctx);

/* RGBA f32 -> RGBA8 exactly as rgb_f_to_u8 (draw_scene.rs:104-108): trunc(clamp(f,0,1)*255+0.5),
 * NaN -> 0 (Rust `as u8`), alpha 255. */
int rt_rgba_to_u8(const float* rgba, uint64_t n_pixels, uint8_t* out_rgba8);

/* render_to_target_gpu (draw_scene.rs:17-47): spp/batch launches, RGBA8 written to `target`
 * (width*height*4) after each batch, then hook(user, samples_done).  spp % batch != 0 is
 * RT_ERR_BATCH (renderer.rs:56-57). */
typedef void (*rt_update_hook)(void* user, uint32_t samples_done);
int rt_render_to_target(const rt_scene_desc* scene, const rt_camera* cam,
                        const rt_render_info* info, uint32_t spp, uint32_t batch,
                        int device, uint8_t* target, rt_update_hook hook, void* user);

/* ------------------------------------------- one frame over several devices */
/* New: the reference is single-adapter (gpu_utils.rs:614-637).  The frame's rows are dealt to
 * n contexts as stripes of `stripe_rows` rows, round-robin (stripe i to context i % n; consecutive
 * stripes of one context merge into one tile); every context renders its stripes for the whole
 * sample range on its device, and ONE gather per frame assembles the frame on devices[0]: a
 * context on another device copies its tile radiance there over xGMI (peer copy), then each
 * context's stripes are placed by one strided copy.  A device ordinal may repeat (several contexts
 * on one device).  The frame equals a one-context frame bit for bit (the RNG and the running mean
 * are keyed on the global pixel and the absolute sample).  The caller is the reference's render
 * thread (renderer.rs:43-60 -> render_to_target_gpu, draw_scene.rs:17-47): no torch, no launcher. */
typedef struct rt_frame rt_frame;

/* The tallest stripe S <= 8 rows with height % (S * n_parts) == 0 (equal stripe counts), else 1. */
uint32_t rt_stripe_rows(uint32_t height, uint32_t n_parts);
/* Context `index`'s tiles (x0 = 0, full-width row ranges) of the stripe deal; stripe_rows 0 picks
 * rt_stripe_rows.  *n_tiles is the count; at most `cap` tiles are written (tiles may be NULL). */
int rt_stripe_tiles(uint32_t width, uint32_t height, uint32_t stripe_rows, uint32_t index, uint32_t n_parts,
                    rt_tile* tiles, uint32_t cap, uint32_t* n_tiles);

/* One rt_ctx per entry of devices[] (created side by side, one KD build shared: `tree` or built
 * here), its stripe buffer, and the frame (width * height RGBA f32) on devices[0]. */
int rt_frame_create(const rt_scene_desc* scene, const rt_camera* cam, const rt_render_info* info,
                    const rt_kd_tree* tree, const int* devices, uint32_t n_devices, uint32_t stripe_rows,
                    rt_frame** out);
/* Every context advances its stripes over [sample_begin, sample_begin + sample_count) (the running
 * mean of rt_render); enqueued on the devices, returns at once.  Split calls equal one call. */
int rt_frame_render(rt_frame* frame, uint64_t sample_begin, uint32_t sample_count);
/* The frame-end gather: waits for the enqueued renders, assembles the frame on devices[0] and copies
 * it to out_rgba (host, width * height * 4 floats) and / or out_rgba_device (devices[0] memory);
 * either may be NULL.  Synchronous. */
int rt_frame_gather(rt_frame* frame, float* out_rgba, float* out_rgba_device);
/* Waits for everything enqueued on every context and closes their timing windows. */
int rt_frame_synchronize(rt_frame* frame);
typedef struct rt_frame_stats {
    float    render_ms_max;      /* the slowest context's device window (rt_last_kernel_ms) */
    float    peer_copy_ms_max;   /* the slowest peer copy of the last gather (0: one device) */
    float    place_ms;           /* the last gather's placement on devices[0] */
    uint32_t n_parts, stripe_rows;
    uint32_t n_gathers;          /* gathers since rt_frame_create */
    uint32_t n_peer_copies;      /* peer copies since rt_frame_create */
} rt_frame_stats;
int rt_frame_get_stats(rt_frame* frame, rt_frame_stats* out);   /* synchronizes first */
/* Context `index`: its device, its rt_ctx (owned by the frame: do not destroy) and tile count. */
int rt_frame_part(const rt_frame* frame, uint32_t index, int* device, rt_ctx** ctx, uint32_t* n_tiles);
const char* rt_frame_last_error(const rt_frame* frame);
int rt_frame_destroy(rt_frame* frame);

/* render_to_target_gpu (draw_scene.rs:17-47) over several devices: spp / batch batches, each
 * rendered by every context on its stripes and gathered once; RGBA8 into `target` and
 * hook(user, samples_done) after every batch, in order.  The targets equal rt_render_to_target's. */
int rt_render_to_target_devices(const rt_scene_desc* scene, const rt_camera* cam,
                                const rt_render_info* info, uint32_t spp, uint32_t batch,
                                const int* devices, uint32_t n_devices, uint8_t* target,
                                rt_update_hook hook, void* user);

/* ------------------------------------------------------------ host: the boundary's caller */
/* Scheme loading in C++ (what the reference's builder does before the `use_gpu` switch):
 * Scheme::from_yml + apply_corrections (builder/mod.rs:63-72), member conversion in renderable
 * order (builder/inner.rs:21-64), glTF models (builder/pr/model.rs:19-207) and cube-map images
 * (builder/pr/distant_cube_map.rs:19-23), reading assets from `assets_root`/<dir>.npz (the
 * repo's asset packs).  `text` is the scheme YAML (RT_SCHEME_YAML) or its JSON form
 * (RT_SCHEME_JSON: tags as {"!Tag": value}).  The scheme owns every array its view points
 * into; the view's info / cam may be edited before rt_create (e.g. width / height overrides). */
typedef struct rt_scheme rt_scheme;
enum { RT_SCHEME_YAML = 0, RT_SCHEME_JSON = 1 };
typedef struct rt_scheme_view {
    const rt_scene_desc* scene;
    rt_camera*           cam;
    rt_render_info*      info;
    uint32_t             samps_per_pix;
    uint32_t             gpu_render_batch;   /* 0 when absent (Option<u32>) */
    uint32_t             use_gpu;            /* RenderInfo::use_gpu.unwrap_or(false) */
    uint32_t             animation;          /* RenderInfo::animation.unwrap_or(false) */
} rt_scheme_view;
int         rt_scheme_load(const char* text, uint64_t len, uint32_t format, const char* assets_root,
                           uint64_t seed, rt_scheme** out);
int         rt_scheme_view_get(rt_scheme* scheme, rt_scheme_view* out);
const char* rt_scheme_last_error(void);   /* this thread's last rt_scheme_load failure */

/* Animation (renderer.rs:65-207, builder/inner.rs:113-249): the number of frames of an
 * animated scheme (0 when render_info.animation is off), and frame i as a still scheme whose
 * spheres / models sit at their keyframe-interpolated places (free with rt_scheme_free).  The
 * keyframe crate's easing is restated, not pinned. */
int         rt_scheme_frames(rt_scheme* scheme, uint32_t* n_frames);
int         rt_scheme_frame(rt_scheme* scheme, uint32_t frame, rt_scheme** out);
int         rt_scheme_free(rt_scheme* scheme);

/* process_output_routine (ui_util.rs:37-54): an RGBA8 buffer (width*height*4, row y = pixel
 * row y of the target) saved as an 8-bit RGBA PNG, flipped vertically when flip_vertical. */
int rt_write_png(const char* path, const uint8_t* rgba8, uint32_t width, uint32_t height,
                 uint32_t flip_vertical);

#ifdef __cplusplus
}
#endif
#endif /* RT_ABI_H */
