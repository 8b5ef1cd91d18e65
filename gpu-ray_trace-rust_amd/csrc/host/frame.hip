// frame.hip — one frame over several devices behind the C ABI, for a caller
// without torch: the reference's render thread (src/renderer.rs:43-60 -> render_to_target_gpu,
// src/render/draw_scene.rs:17-47) gets the tile split and the frame-end gather from the library.
//
// The reference is single-adapter (gpu_utils.rs:614-637); this is new.  The frame's rows are
// dealt to the contexts as stripes of a few rows, round-robin (rt_stripe_tiles, the same deal as
// rt_amd/shard.py rank_tiles); each context renders its stripes for the whole sample range into
// one buffer on its own device (rt_render_device_async, its tiles concatenated), and one gather
// per frame assembles the frame on the first device:
//   - a context on another device copies its buffer to a staging buffer on the first device over
//     xGMI (hipMemcpyPeerAsync on a stream of the source device; peer access is enabled where the
//     devices allow it, else HIP stages through the host);
//   - the first device places every context's rows with one strided copy per context
//     (hipMemcpy2DAsync: context k's j-th stripe is frame stripe j * n + k), plus one plain copy
//     for a last, shorter stripe.
// Every copy is ordered by events, not by the host: a context's next render waits (through its
// caller stream) for the gather still reading its buffer, and the gather waits for the render.
// A pixel's value depends only on (pixel, absolute sample range), so the frame equals a
// single-context frame bit for bit, whatever the number of contexts or devices.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/rt_abi.h"

namespace {

constexpr uint32_t STRIPE_MAX = 8;  // rows: the queue hands out a launch's pixels in 8 x 8 blocks

struct Part {                    // one context: its device, stripes and buffers
    int device = 0;
    rt_ctx* ctx = nullptr;
    std::vector<rt_tile> tiles;
    uint64_t npix = 0;
    float* buf = nullptr;        // tiles concatenated, RGBA f32, on `device`
    bool remote = false;         // gathered through staging: on another device (or RT_DEBUG_FRAME_STAGING)
    float* staging = nullptr;    // on the first device, when remote
    hipStream_t stream = nullptr;   // on `device`: the context's caller stream, the peer copy
    hipEvent_t copied = nullptr;    // on `stream`: the buffer is on the first device
    hipEvent_t copy_begin = nullptr, copy_end = nullptr;  // timing of the peer copy
};

}  // namespace

struct rt_frame {
    uint32_t width = 0, height = 0, stripe = 1, n = 0;
    int device0 = 0;
    std::vector<Part> part;
    hipStream_t stream0 = nullptr;  // on the first device: placement and read-back
    hipEvent_t placed = nullptr;    // the last gather's placement is done (contexts may write again)
    hipEvent_t place_begin = nullptr, place_end = nullptr;
    float* frame = nullptr;         // width * height RGBA f32 on the first device
    bool gathered = false;          // a gather has been enqueued (placed / timings valid)
    uint32_t n_gathers = 0, n_peer_copies = 0;
    std::string err;
};

#define FCHK(f, call)                                                               \
    do {                                                                            \
        hipError_t e_ = (call);                                                     \
        if (e_ != hipSuccess) {                                                     \
            (f)->err = std::string(#call) + ": " + hipGetErrorString(e_);           \
            return RT_ERR_HIP;                                                      \
        }                                                                           \
    } while (0)

static int ferr(rt_frame* f, int code, const std::string& msg) {
    f->err = msg;
    return code;
}

// The tallest stripe S <= STRIPE_MAX that deals every context the same number of stripes
// (height % (S * n) == 0), else 1 (rt_amd/shard.py stripe_rows).
extern "C" uint32_t rt_stripe_rows(uint32_t height, uint32_t n_parts) {
    if (n_parts == 0) return 1;
    for (uint32_t s = STRIPE_MAX; s > 1; --s)
        if (height % (s * n_parts) == 0) return s;
    return 1;
}

// Context `index`'s stripes of a width x height frame: stripe i (rows [i * S, i * S + S)) goes to
// context i % n; consecutive stripes of one context merge into one tile.  *n_tiles is always the
// count; at most `cap` tiles are written (tiles may be NULL to ask for the count).
extern "C" int rt_stripe_tiles(uint32_t width, uint32_t height, uint32_t stripe_rows, uint32_t index,
                               uint32_t n_parts, rt_tile* tiles, uint32_t cap, uint32_t* n_tiles) {
    if (!n_tiles || width == 0 || height == 0 || n_parts == 0 || index >= n_parts) return RT_ERR_INVALID_ARG;
    const uint32_t S = stripe_rows ? stripe_rows : rt_stripe_rows(height, n_parts);
    uint32_t n = 0;
    rt_tile last{0, 0, 0, 0};
    for (uint64_t y0 = (uint64_t)index * S; y0 < height; y0 += (uint64_t)n_parts * S) {
        const uint32_t h = (uint32_t)std::min<uint64_t>(S, height - y0);
        if (n && last.y0 + last.h == y0) {
            last.h += h;
        } else {
            if (n && tiles && n - 1 < cap) tiles[n - 1] = last;
            last = rt_tile{0, (uint32_t)y0, width, h};
            ++n;
        }
    }
    if (n && tiles && n - 1 < cap) tiles[n - 1] = last;
    *n_tiles = n;
    return RT_OK;
}

static void destroy_frame(rt_frame* f) {
    if (!f) return;
    for (Part& p : f->part) {
        (void)hipSetDevice(p.device);
        if (p.stream) (void)hipStreamSynchronize(p.stream);
    }
    if (f->stream0) {
        (void)hipSetDevice(f->device0);
        (void)hipStreamSynchronize(f->stream0);
    }
    for (Part& p : f->part) {
        if (p.ctx) rt_destroy(p.ctx);  // drains the context's own streams
        (void)hipSetDevice(p.device);
        if (p.buf) (void)hipFree(p.buf);
        if (p.copied) (void)hipEventDestroy(p.copied);
        if (p.copy_begin) (void)hipEventDestroy(p.copy_begin);
        if (p.copy_end) (void)hipEventDestroy(p.copy_end);
        if (p.stream) (void)hipStreamDestroy(p.stream);
    }
    (void)hipSetDevice(f->device0);
    for (Part& p : f->part)
        if (p.staging) (void)hipFree(p.staging);
    if (f->frame) (void)hipFree(f->frame);
    if (f->placed) (void)hipEventDestroy(f->placed);
    if (f->place_begin) (void)hipEventDestroy(f->place_begin);
    if (f->place_end) (void)hipEventDestroy(f->place_end);
    if (f->stream0) (void)hipStreamDestroy(f->stream0);
    delete f;
}

static int frame_create_impl(rt_frame* f, const rt_scene_desc* scene, const rt_camera* cam,
                             const rt_render_info* info, const rt_kd_tree* tree_in, const int* devices,
                             uint32_t stripe_rows) {
    int total = 0;
    if (hipGetDeviceCount(&total) != hipSuccess) return ferr(f, RT_ERR_NO_DEVICE, "no HIP device");
    for (uint32_t k = 0; k < f->n; ++k)
        if (devices[k] < 0 || devices[k] >= total) return ferr(f, RT_ERR_NO_DEVICE, "bad device ordinal");
    f->width = info->width;
    f->height = info->height;
    f->device0 = devices[0];
    f->stripe = stripe_rows ? stripe_rows : rt_stripe_rows(info->height, f->n);
    f->part.resize(f->n);
    // RT_DEBUG_FRAME_STAGING=1 (tests): every context but the first is gathered as if it were on
    // another device, so the staging buffers, the peer copies and their event hand-offs run on a
    // one-GPU box too (hipMemcpyPeerAsync from a device to itself is a device-to-device copy).
    const char* fs = std::getenv("RT_DEBUG_FRAME_STAGING");
    const bool force_staging = fs && std::strcmp(fs, "0") != 0;
    // one KD build for every context (rt_create deep-copies it to each device)
    rt_kd_tree* built = nullptr;
    const rt_kd_tree* tree = tree_in;
    if (!tree) {
        const int st = rt_kd_build(scene, info->kd_tree_depth, &built);
        if (st) return ferr(f, st, "KD build failed");
        tree = built;
    }
    struct Guard { rt_kd_tree* t; ~Guard() { rt_kd_free(t); } } guard{built};
    // the contexts, created side by side (each uploads the scene to its device)
    std::vector<int> status(f->n, RT_OK);
    {
        std::vector<std::thread> th;
        for (uint32_t k = 0; k < f->n; ++k) {
            f->part[k].device = devices[k];
            th.emplace_back([&, k] { status[k] = rt_create(scene, cam, info, tree, devices[k], &f->part[k].ctx); });
        }
        for (auto& t : th) t.join();
    }
    for (uint32_t k = 0; k < f->n; ++k)
        if (status[k]) return ferr(f, status[k], "rt_create failed for context " + std::to_string(k));
    for (uint32_t k = 0; k < f->n; ++k) {
        Part& p = f->part[k];
        uint32_t nt = 0;
        rt_stripe_tiles(f->width, f->height, f->stripe, k, f->n, nullptr, 0, &nt);
        p.tiles.resize(nt);
        rt_stripe_tiles(f->width, f->height, f->stripe, k, f->n, p.tiles.data(), nt, &nt);
        for (const rt_tile& t : p.tiles) p.npix += (uint64_t)t.w * t.h;
        p.remote = p.device != f->device0 || (force_staging && k > 0);
        FCHK(f, hipSetDevice(p.device));
        FCHK(f, hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking));
        FCHK(f, hipEventCreateWithFlags(&p.copied, hipEventDisableTiming));
        FCHK(f, hipEventCreate(&p.copy_begin));
        FCHK(f, hipEventCreate(&p.copy_end));
        if (p.npix && hipMalloc(&p.buf, p.npix * 4 * sizeof(float)) != hipSuccess)
            return ferr(f, RT_ERR_OOM, "stripe buffer alloc failed");
        if (p.device != f->device0) {
            // the source device writes the first device's memory: its peer mapping, if any
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, p.device, f->device0) == hipSuccess && can) {
                const hipError_t e = hipDeviceEnablePeerAccess(f->device0, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    return ferr(f, RT_ERR_HIP, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
                (void)hipGetLastError();  // an "already enabled" status is no error
            }
        }
    }
    FCHK(f, hipSetDevice(f->device0));
    FCHK(f, hipStreamCreateWithFlags(&f->stream0, hipStreamNonBlocking));
    FCHK(f, hipEventCreateWithFlags(&f->placed, hipEventDisableTiming));
    FCHK(f, hipEventCreate(&f->place_begin));
    FCHK(f, hipEventCreate(&f->place_end));
    const uint64_t fpix = (uint64_t)f->width * f->height;
    if (hipMalloc(&f->frame, fpix * 4 * sizeof(float)) != hipSuccess) return ferr(f, RT_ERR_OOM, "frame alloc failed");
    for (Part& p : f->part)
        if (p.remote && p.npix && hipMalloc(&p.staging, p.npix * 4 * sizeof(float)) != hipSuccess)
            return ferr(f, RT_ERR_OOM, "staging alloc failed");
    return RT_OK;
}

extern "C" int rt_frame_create(const rt_scene_desc* scene, const rt_camera* cam, const rt_render_info* info,
                               const rt_kd_tree* tree, const int* devices, uint32_t n_devices,
                               uint32_t stripe_rows, rt_frame** out) {
    if (!scene || !cam || !info || !devices || !out || n_devices == 0) return RT_ERR_INVALID_ARG;
    *out = nullptr;
    if (info->width == 0 || info->height == 0) return RT_ERR_INVALID_ARG;
    if (n_devices > info->height) return RT_ERR_INVALID_ARG;  // every context gets a stripe
    rt_frame* f = new (std::nothrow) rt_frame();
    if (!f) return RT_ERR_OOM;
    f->n = n_devices;
    int st;
    try {
        st = frame_create_impl(f, scene, cam, info, tree, devices, stripe_rows);
    } catch (const std::bad_alloc&) {
        st = ferr(f, RT_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        st = ferr(f, RT_ERR_OOM, std::string("host runtime: ") + e.what());
    }
    if (st) {
        std::fprintf(stderr, "rt_frame_create: %s\n", f->err.c_str());
        destroy_frame(f);
        return st;
    }
    *out = f;
    return RT_OK;
}

// Every context advances its stripes by [sample_begin, sample_begin + sample_count), enqueued on
// its devices; returns without waiting.  The folds wait for the gather still reading the buffers.
extern "C" int rt_frame_render(rt_frame* f, uint64_t sample_begin, uint32_t sample_count) {
    if (!f) return RT_ERR_INVALID_ARG;
    for (uint32_t k = 0; k < f->n; ++k) {
        Part& p = f->part[k];
        if (!p.npix) continue;
        FCHK(f, hipSetDevice(p.device));
        // the last gather placed (or copied) this buffer before the new fold may write it: the
        // context's folds wait for what its caller stream holds at the call
        if (f->gathered) FCHK(f, hipStreamWaitEvent(p.stream, p.remote ? p.copied : f->placed, 0));
        const int st = rt_render_device_async(p.ctx, p.tiles.data(), (uint32_t)p.tiles.size(), sample_begin,
                                              sample_count, p.buf, p.stream);
        if (st) return ferr(f, st, "context " + std::to_string(k) + ": " + rt_last_error(p.ctx));
    }
    return RT_OK;
}

// The frame-end gather, enqueued: peer copies to the first device, placement of every context's
// stripes into the frame, and (out_host) the read-back.  Ordered after every enqueued render.
static int gather_enqueue(rt_frame* f, float* out_host, float* out_dev) {
    for (Part& p : f->part) {
        if (!p.npix || !p.remote) continue;
        FCHK(f, hipSetDevice(p.device));
        // a staging buffer the previous placement may still read
        if (f->gathered) FCHK(f, hipStreamWaitEvent(p.stream, f->placed, 0));
        FCHK(f, hipEventRecord(p.copy_begin, p.stream));
        FCHK(f, hipMemcpyPeerAsync(p.staging, f->device0, p.buf, p.device, p.npix * 4 * sizeof(float), p.stream));
        FCHK(f, hipEventRecord(p.copy_end, p.stream));
        f->n_peer_copies++;
    }
    for (Part& p : f->part) {
        if (!p.npix) continue;
        FCHK(f, hipSetDevice(p.device));
        FCHK(f, hipEventRecord(p.copied, p.stream));  // local contexts: the render is done
    }
    FCHK(f, hipSetDevice(f->device0));
    for (Part& p : f->part)
        if (p.npix) FCHK(f, hipStreamWaitEvent(f->stream0, p.copied, 0));
    FCHK(f, hipEventRecord(f->place_begin, f->stream0));
    const size_t px = 4 * sizeof(float);
    const size_t row = (size_t)f->width * px;
    const uint32_t S = f->stripe, n = f->n;
    const uint64_t n_stripes = (f->height + S - 1) / S;
    for (uint32_t k = 0; k < n; ++k) {
        Part& p = f->part[k];
        if (!p.npix) continue;
        const char* src = reinterpret_cast<const char*>(p.staging ? p.staging : p.buf);
        // context k's full stripes: its j-th one is frame stripe j * n + k
        uint64_t full = 0;
        for (uint64_t s = k; s < n_stripes; s += n)
            if ((s + 1) * S <= f->height) ++full;
        char* dst = reinterpret_cast<char*>(f->frame) + (size_t)k * S * row;
        if (full)
            FCHK(f, hipMemcpy2DAsync(dst, (size_t)n * S * row, src, (size_t)S * row, (size_t)S * row, full,
                                     hipMemcpyDeviceToDevice, f->stream0));
        // a shorter last stripe of the frame, when it is context k's
        const uint64_t last = n_stripes - 1;
        if (f->height % S && last % n == k) {
            const uint32_t h = f->height % S;
            FCHK(f, hipMemcpyAsync(reinterpret_cast<char*>(f->frame) + (size_t)last * S * row, src + full * S * row,
                                   (size_t)h * row, hipMemcpyDeviceToDevice, f->stream0));
        }
    }
    FCHK(f, hipEventRecord(f->place_end, f->stream0));
    FCHK(f, hipEventRecord(f->placed, f->stream0));
    const size_t bytes = (size_t)f->width * f->height * px;
    if (out_dev) FCHK(f, hipMemcpyAsync(out_dev, f->frame, bytes, hipMemcpyDeviceToDevice, f->stream0));
    if (out_host) FCHK(f, hipMemcpyAsync(out_host, f->frame, bytes, hipMemcpyDeviceToHost, f->stream0));
    f->gathered = true;
    f->n_gathers++;
    return RT_OK;
}

extern "C" int rt_frame_gather(rt_frame* f, float* out_rgba, float* out_rgba_device) {
    if (!f) return RT_ERR_INVALID_ARG;
    int st = gather_enqueue(f, out_rgba, out_rgba_device);
    if (st) return st;
    FCHK(f, hipSetDevice(f->device0));
    FCHK(f, hipStreamSynchronize(f->stream0));
    return RT_OK;
}

extern "C" int rt_frame_synchronize(rt_frame* f) {
    if (!f) return RT_ERR_INVALID_ARG;
    for (uint32_t k = 0; k < f->n; ++k) {
        Part& p = f->part[k];
        const int st = rt_synchronize(p.ctx);
        if (st) return ferr(f, st, "context " + std::to_string(k) + ": " + rt_last_error(p.ctx));
        FCHK(f, hipSetDevice(p.device));
        FCHK(f, hipStreamSynchronize(p.stream));
    }
    FCHK(f, hipSetDevice(f->device0));
    FCHK(f, hipStreamSynchronize(f->stream0));
    return RT_OK;
}

extern "C" int rt_frame_get_stats(rt_frame* f, rt_frame_stats* out) {
    if (!f || !out) return RT_ERR_INVALID_ARG;
    int st = rt_frame_synchronize(f);
    if (st) return st;
    std::memset(out, 0, sizeof(*out));
    out->n_parts = f->n;
    out->stripe_rows = f->stripe;
    out->n_gathers = f->n_gathers;
    out->n_peer_copies = f->n_peer_copies;
    for (Part& p : f->part) {
        float ms = 0.f;
        if (p.ctx && rt_last_kernel_ms(p.ctx, &ms) == RT_OK) out->render_ms_max = std::max(out->render_ms_max, ms);
        if (f->gathered && p.npix && p.remote) {
            FCHK(f, hipSetDevice(p.device));
            FCHK(f, hipEventElapsedTime(&ms, p.copy_begin, p.copy_end));
            out->peer_copy_ms_max = std::max(out->peer_copy_ms_max, ms);
        }
    }
    if (f->gathered) {
        FCHK(f, hipSetDevice(f->device0));
        FCHK(f, hipEventElapsedTime(&out->place_ms, f->place_begin, f->place_end));
    }
    return RT_OK;
}

extern "C" int rt_frame_part(const rt_frame* f, uint32_t index, int* device, rt_ctx** ctx, uint32_t* n_tiles) {
    if (!f || index >= f->n) return RT_ERR_INVALID_ARG;
    if (device) *device = f->part[index].device;
    if (ctx) *ctx = f->part[index].ctx;
    if (n_tiles) *n_tiles = (uint32_t)f->part[index].tiles.size();
    return RT_OK;
}

extern "C" const char* rt_frame_last_error(const rt_frame* f) { return f ? f->err.c_str() : "null frame"; }

extern "C" int rt_frame_destroy(rt_frame* f) {
    if (!f) return RT_ERR_INVALID_ARG;
    destroy_frame(f);
    return RT_OK;
}

// render_to_target_gpu (draw_scene.rs:17-47) over several devices: spp / batch batches, each one
// rendered by every context on its stripes, gathered once, converted to RGBA8 into `target` and
// handed to the hook, in batch order.  Pipelined: batch b + 1 is enqueued before batch b's frame
// is read back and converted (two pinned host frames), so the devices do not wait on the host.
extern "C" int rt_render_to_target_devices(const rt_scene_desc* scene, const rt_camera* cam,
                                           const rt_render_info* info, uint32_t spp, uint32_t batch,
                                           const int* devices, uint32_t n_devices, uint8_t* target,
                                           rt_update_hook hook, void* user) {
    if (!scene || !cam || !info || !target || !devices || n_devices == 0 || batch == 0) return RT_ERR_INVALID_ARG;
    if (spp % batch != 0) return RT_ERR_BATCH;
    rt_frame* f = nullptr;
    int st = rt_frame_create(scene, cam, info, nullptr, devices, n_devices, 0, &f);
    if (st) return st;
    const uint64_t npix = (uint64_t)info->width * info->height;
    const uint32_t n_batch = spp / batch;
    float* host[2] = {nullptr, nullptr};
    hipEvent_t ready[2] = {nullptr, nullptr};
    auto run = [&]() -> int {
        FCHK(f, hipSetDevice(f->device0));
        for (int i = 0; i < 2; ++i) {
            if (hipHostMalloc(reinterpret_cast<void**>(&host[i]), npix * 4 * sizeof(float), hipHostMallocDefault) != hipSuccess)
                return ferr(f, RT_ERR_OOM, "pinned frame alloc failed");
            FCHK(f, hipEventCreateWithFlags(&ready[i], hipEventDisableTiming));
        }
        auto deliver = [&](uint32_t b) -> int {  // batch b's frame: samples [0, (b + 1) * batch)
            FCHK(f, hipEventSynchronize(ready[b & 1]));
            rt_rgba_to_u8(host[b & 1], npix, target);
            if (hook) hook(user, (b + 1) * batch);
            return RT_OK;
        };
        for (uint32_t b = 0; b < n_batch; ++b) {
            int r = rt_frame_render(f, (uint64_t)b * batch, batch);
            if (r) return r;
            if ((r = gather_enqueue(f, host[b & 1], nullptr))) return r;
            FCHK(f, hipSetDevice(f->device0));
            FCHK(f, hipEventRecord(ready[b & 1], f->stream0));
            if (b && (r = deliver(b - 1))) return r;
        }
        return deliver(n_batch - 1);
    };
    try {
        st = run();
    } catch (const std::exception& e) {
        st = ferr(f, RT_ERR_OOM, std::string("host runtime: ") + e.what());
    }
    if (!st) st = rt_frame_synchronize(f);
    if (st) std::fprintf(stderr, "rt_render_to_target_devices: %s\n", f->err.c_str());
    (void)hipSetDevice(f->device0);
    for (int i = 0; i < 2; ++i) {
        if (ready[i]) (void)hipEventDestroy(ready[i]);
        if (host[i]) (void)hipHostFree(host[i]);
    }
    rt_frame_destroy(f);
    return st;
}
