// chase_latency.hip — latency of one dependent load on gfx950, by working set, for the chain
// model of the mesh kernel ("What bounds a cooperative round").  One workgroup of
// one wave chases pointers through a random cyclic permutation of 16-B records: every lane its
// own chain (64 random 16-B gathers per step, as a cooperative pass's vertex loads) or all lanes
// the same chain (one address per step, as a packet's scalar-uniform node).  Cycles per step from
// s_memtime (100 MHz constant clock on gfx950, converted with the printed clock rate) and from
// wall time over many steps.
// Build: hipcc --offload-arch=gfx950 -O3 -o lib/chase_latency tools/chase_latency.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void chase(const uint4* __restrict__ t, uint32_t steps, uint32_t same, uint32_t* out,
                      unsigned long long* ticks) {
    uint32_t i = same ? 0u : threadIdx.x * 977u;
    unsigned long long t0 = clock64();
    for (uint32_t s = 0; s < steps; ++s) i = t[i].x;
    unsigned long long t1 = clock64();
    out[threadIdx.x] = i;
    if (threadIdx.x == 0) *ticks = t1 - t0;
}

int main() {
    const size_t sizes[] = {8u << 10, 64u << 10, 1u << 20, 3u << 20, 32u << 20, 192u << 20, 1024u << 20};
    uint4* t = nullptr;
    uint32_t* out = nullptr;
    unsigned long long* ticks = nullptr;
    const size_t maxn = (1024u << 20) / 16;
    if (hipMalloc(&t, maxn * 16) != hipSuccess || hipMalloc(&out, 256) != hipSuccess ||
        hipMalloc(&ticks, 8) != hipSuccess)
        return 1;
    int clk_khz = 0;
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    std::printf("clock64 rate: %d kHz (hipDeviceAttributeClockRate)\n", clk_khz);
    std::vector<uint4> h;
    for (size_t bytes : sizes) {
        const size_t n = bytes / 16;
        // one random cycle through all n records (Sattolo's algorithm)
        std::vector<uint32_t> p(n);
        for (size_t k = 0; k < n; ++k) p[k] = (uint32_t)k;
        uint64_t x = 0x9e3779b97f4a7c15ull;
        for (size_t k = n - 1; k > 0; --k) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            const size_t j = x % k;
            std::swap(p[k], p[j]);
        }
        h.assign(n, make_uint4(0, 0, 0, 0));
        for (size_t k = 0; k < n; ++k) h[p[k]].x = p[(k + 1) % n];
        if (hipMemcpy(t, h.data(), n * 16, hipMemcpyHostToDevice) != hipSuccess) return 2;
        for (uint32_t same = 0; same < 2; ++same) {
            const uint32_t steps = 20000;
            hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, t, 2000, same, out, ticks);  // warm the caches
            if (hipDeviceSynchronize() != hipSuccess) return 3;
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, t, steps, same, out, ticks);
            (void)hipEventRecord(e1, 0);
            if (hipDeviceSynchronize() != hipSuccess) return 4;
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            unsigned long long tk = 0;
            (void)hipMemcpy(&tk, ticks, 8, hipMemcpyDeviceToHost);
            std::printf("{\"working_set_bytes\": %zu, \"lanes\": \"%s\", \"ns_per_step\": %.1f, \"clock64_per_step\": %.1f}\n",
                        bytes, same ? "uniform" : "64 random", ms * 1e6 / steps, (double)tk / steps);
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }
    }
    (void)hipFree(t);
    (void)hipFree(out);
    (void)hipFree(ticks);
    return 0;
}
