// rt_render — the reference's headless single-frame run (src/main.rs:14-43 with `no_ui`,
// Renderer::consume_and_do renderer.rs:43-60, process_output_routine ui_util.rs:37-54) on the
// MI355X device path, in C++ over the C ABI:
//   scheme YAML -> rt_scheme_load -> rt_render_to_target (spp / gpu_render_batch launches)
//   -> after every batch the RGBA8 target is flipped and saved as a PNG.
// Animated schemes (render_info.animation, renderer.rs:65-207) render every frame to
// <frames-dir>/<n>.png, n from 1 as in the GPU branch; --frames r/N renders frames i with
// i % N == r (frames are independent: N processes on N GPUs need no collective).  The mp4
// muxing of main.rs:54-97 (openh264) is not reproduced.
// --gpus N (devices 0..N-1) or --devices a,b,...: one frame over several devices in this one
// process (rt_render_to_target_devices: row stripes per device, one gather per batch), SURVEY.md
// §8e behind the C ABI; a device may repeat (several contexts on one GPU).
// Usage: rt_render <scheme.yml|scheme.json> [no_ui] [--assets DIR] [--out FILE] [--device N]
//                  [--gpus N | --devices a,b,...] [--seed S] [--width W] [--height H] [--spp N]
//                  [--batch B] [--frames-dir DIR] [--frames r/N] [--max-frames K]
// Assets are read from DIR/<dir>.npz (default: assets_pack next to the library's parent).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sys/stat.h>
#include <sstream>
#include <string>
#include <vector>

#include "../../../include/rt_abi.h"

namespace {

struct Out {
    std::string path;
    const uint8_t* target;
    uint32_t w, h, spp;
    int status = RT_OK;
};

void on_batch(void* user, uint32_t done) {
    Out* o = static_cast<Out*>(user);
    const int st = rt_write_png(o->path.c_str(), o->target, o->w, o->h, 1);
    if (st != RT_OK) o->status = st;
    std::fprintf(stderr, "\r[rt_render] %u / %u samples per pixel -> %s", done, o->spp, o->path.c_str());
}

int usage() {
    std::fprintf(stderr,
                 "usage: rt_render <scheme.yml|scheme.json> [no_ui] [--assets DIR] [--out FILE] [--device N]\n"
                 "                 [--gpus N | --devices a,b,...] [--seed S] [--width W] [--height H]\n"
                 "                 [--spp N] [--batch B]\n"
                 "                 [--frames-dir DIR] [--frames r/N] [--max-frames K]\n");
    return 2;
}

}  // namespace

int main(int argc, char** argv) {
    // the launch pipeline's streams need their own hardware queues (rt_amd/__init__.py): at
    // least 16, set before HIP starts
    {
        const char* q = std::getenv("GPU_MAX_HW_QUEUES");
        if (!q || std::atoi(q) < 16) setenv("GPU_MAX_HW_QUEUES", "16", 1);
    }
    if (argc < 2) return usage();
    std::string scheme_path = argv[1], assets = "assets_pack", out = "render_out.png";
    int device = 0;
    unsigned long long seed = 0x5EED0001ull;
    long width = -1, height = -1, spp = -1, batch = -1, max_frames = -1;
    std::string frames_dir = "anim_frames";
    std::vector<int> devices;  // several: one frame over these devices (rt_render_to_target_devices)
    unsigned frank = 0, fworld = 1;
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        auto val = [&]() -> const char* {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "%s needs a value\n", a.c_str());
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "no_ui" || a == "ui") continue;  // main.rs:20-23: there is no UI here either way
        else if (a == "--assets") assets = val();
        else if (a == "--out") out = val();
        else if (a == "--device") device = std::atoi(val());
        else if (a == "--gpus") {
            const int n = std::atoi(val());
            if (n < 1) return usage();
            devices.clear();
            for (int d = 0; d < n; ++d) devices.push_back(d);
        }
        else if (a == "--devices") {
            devices.clear();
            std::stringstream ds(val());
            std::string tok;
            while (std::getline(ds, tok, ',')) {
                if (tok.empty()) return usage();
                devices.push_back(std::atoi(tok.c_str()));
            }
            if (devices.empty()) return usage();
        }
        else if (a == "--seed") seed = std::strtoull(val(), nullptr, 0);
        else if (a == "--width") width = std::atol(val());
        else if (a == "--height") height = std::atol(val());
        else if (a == "--spp") spp = std::atol(val());
        else if (a == "--batch") batch = std::atol(val());
        else if (a == "--frames-dir") frames_dir = val();
        else if (a == "--max-frames") max_frames = std::atol(val());
        else if (a == "--frames") {
            if (std::sscanf(val(), "%u/%u", &frank, &fworld) != 2 || fworld == 0 || frank >= fworld) return usage();
        }
        else return usage();
    }
    std::ifstream f(scheme_path);
    if (!f) {
        std::fprintf(stderr, "Couldn't open file %s\n", scheme_path.c_str());
        return 1;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    const bool json = scheme_path.size() > 5 && scheme_path.compare(scheme_path.size() - 5, 5, ".json") == 0;
    rt_scheme* sch = nullptr;
    int st = rt_scheme_load(text.data(), text.size(), json ? RT_SCHEME_JSON : RT_SCHEME_YAML, assets.c_str(), seed, &sch);
    if (st != RT_OK) {
        std::fprintf(stderr, "rt_render: %s: %s\n", rt_status_string(st), rt_scheme_last_error());
        return 1;
    }
    rt_scheme_view v{};
    rt_scheme_view_get(sch, &v);
    // one device: rt_render_to_target; several: the same loop over every device's stripes
    auto render = [&](const rt_scheme_view& sv, uint8_t* target, uint32_t n_spp, uint32_t n_batch, Out* o) {
        if (devices.size() > 1)
            return rt_render_to_target_devices(sv.scene, sv.cam, sv.info, n_spp, n_batch, devices.data(),
                                               (uint32_t)devices.size(), target, on_batch, o);
        return rt_render_to_target(sv.scene, sv.cam, sv.info, n_spp, n_batch, devices.empty() ? device : devices[0],
                                   target, on_batch, o);
    };
    if (!v.use_gpu)
        std::fprintf(stderr, "rt_render: use_gpu is false in the scheme; rendering on the device path anyway\n");
    if (width > 0) v.info->width = (uint32_t)width;
    if (height > 0) v.info->height = (uint32_t)height;
    const uint32_t n_spp = spp > 0 ? (uint32_t)spp : v.samps_per_pix;
    const uint32_t n_batch = batch > 0 ? (uint32_t)batch : v.gpu_render_batch;
    if (!n_batch) {
        std::fprintf(stderr, "rt_render: gpu_render_batch needs to be set for GPU mode!\n");  // renderer.rs:55
        rt_scheme_free(sch);
        return 1;
    }
    if (v.animation) {  // consume_and_do_anim (renderer.rs:65-207)
        uint32_t n = 0;
        if ((st = rt_scheme_frames(sch, &n)) != RT_OK) {
            std::fprintf(stderr, "rt_render: %s\n", rt_scheme_last_error());
            rt_scheme_free(sch);
            return 1;
        }
        if (max_frames >= 0 && (uint32_t)max_frames < n) n = (uint32_t)max_frames;
        ::mkdir(frames_dir.c_str(), 0755);
        std::fprintf(stderr, "rt_render: %u frames, rank %u of %u\n", n, frank, fworld);
        for (uint32_t i = frank; i < n; i += fworld) {
            rt_scheme* fr = nullptr;
            if ((st = rt_scheme_frame(sch, i, &fr)) != RT_OK) {
                std::fprintf(stderr, "rt_render: frame %u: %s\n", i, rt_scheme_last_error());
                rt_scheme_free(sch);
                return 1;
            }
            rt_scheme_view fv{};
            rt_scheme_view_get(fr, &fv);
            std::vector<uint8_t> target((size_t)fv.info->width * fv.info->height * 4, 0);
            Out o{frames_dir + "/" + std::to_string(i + 1) + ".png", target.data(), fv.info->width, fv.info->height, n_spp};
            st = render(fv, target.data(), n_spp, n_batch, &o);
            rt_scheme_free(fr);
            std::fprintf(stderr, "\n");
            if (st != RT_OK || o.status != RT_OK) {
                std::fprintf(stderr, "rt_render: frame %u: %s\n", i, rt_status_string(st != RT_OK ? st : o.status));
                rt_scheme_free(sch);
                return 1;
            }
        }
        rt_scheme_free(sch);
        return 0;
    }
    std::vector<uint8_t> target((size_t)v.info->width * v.info->height * 4, 0);
    Out o{out, target.data(), v.info->width, v.info->height, n_spp};
    st = render(v, target.data(), n_spp, n_batch, &o);
    std::fprintf(stderr, "\n");
    rt_scheme_free(sch);
    if (st != RT_OK) {
        std::fprintf(stderr, "rt_render: %s\n", rt_status_string(st));
        return 1;
    }
    if (o.status != RT_OK) {
        std::fprintf(stderr, "rt_render: cannot save %s\n", out.c_str());
        return 1;
    }
    return 0;
}
