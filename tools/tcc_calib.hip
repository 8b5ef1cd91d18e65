// tcc_calib.hip — what one L2 (TCC) request stands for on gfx950, for converting the TCP->TCC
// request counters of the mesh kernels into bytes (DESIGN.md §5, a380's L2 traffic).
// Each pattern is one kernel launch whose lanes gather from random 128-B lines of an L2-resident
// 2 MiB table (L1 misses almost always); run it under
//   rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum -- lib/tcc_calib
// and divide each dispatch's requests by the lane-loads it printed:
//   k=0  one dword per lane at the start of a line
//   k=1  one dwordx4 per lane at the start of a line
//   k=2  two dwordx4 per lane: bytes 0-15 and 64-79 of the same line (two 64-B halves)
//   k=3  two dwordx4 per lane: bytes 0-15 and 16-31 of the same line (one 64-B half)
//   k=4  three dwordx4 per lane: a 48-B record at a 48-B stride (the mesh kernel's triangle)
// Build: hipcc --offload-arch=gfx950 -O3 -o lib/tcc_calib tools/tcc_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr uint32_t LINES = (2u << 20) / 128u;   // 2 MiB table: inside one XCD's 4 MiB L2
constexpr uint32_t THREADS = 256, BLOCKS = 2048, ITERS = 16;

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__global__ void gather(const uint4* __restrict__ t, uint32_t k, uint32_t* out) {
    const uint32_t g = blockIdx.x * THREADS + threadIdx.x;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < ITERS; ++i) {
        const uint32_t line = hash(g * ITERS + i) % LINES;
        const uint4* p = t + line * 8u;  // 8 x 16 B per line
        if (k == 0) {
            acc += reinterpret_cast<const uint32_t*>(p)[0];
        } else if (k == 1) {
            acc += p[0].x;
        } else if (k == 2) {
            const uint4 a = p[0], b = p[4];
            acc += a.x + b.y;
        } else if (k == 3) {
            const uint4 a = p[0], b = p[1];
            acc += a.x + b.y;
        } else {
            const uint32_t rec = hash(g * ITERS + i) % (LINES * 128u / 48u - 1u);
            const uint4* r = t + rec * 3u;
            const uint4 a = r[0], b = r[1], c = r[2];
            acc += a.x + b.y + c.z;
        }
    }
    out[g] = acc;
}

int main() {
    uint4* t = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&t, (size_t)LINES * 128u) != hipSuccess || hipMalloc(&out, (size_t)BLOCKS * THREADS * 4u) != hipSuccess)
        return 1;
    (void)hipMemset(t, 1, (size_t)LINES * 128u);
    const char* what[5] = {"dword", "dwordx4", "2x dwordx4, two 64-B halves", "2x dwordx4, one 64-B half",
                           "3x dwordx4, 48-B record"};
    const uint32_t loads_per_lane[5] = {1, 1, 2, 2, 3};
    for (uint32_t k = 0; k < 5; ++k) {
        for (int rep = 0; rep < 2; ++rep) {  // the first launch warms L2; the profile reads the second
            hipLaunchKernelGGL(gather, dim3(BLOCKS), dim3(THREADS), 0, 0, t, k, out);
            if (hipDeviceSynchronize() != hipSuccess) return 2;
        }
        std::printf("pattern %u (%s): lane-loads per launch %llu, lane line-accesses %llu\n", k, what[k],
                    (unsigned long long)BLOCKS * THREADS * ITERS * loads_per_lane[k],
                    (unsigned long long)BLOCKS * THREADS * ITERS);
    }
    (void)hipFree(t);
    (void)hipFree(out);
    return 0;
}
