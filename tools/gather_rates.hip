// Gather-rate microbenchmark of the vector-memory path on gfx950 (mesh kernels):
// how many records per second the chip returns to VGPRs for the access shapes of a cooperative
// leaf pass (one record per lane, per-lane addresses), by record layout and access pattern.
//   layouts: dword, dwordx2, dwordx3 (12-B records), dwordx4, a triangle as 3 x dwordx4 (48 B)
//            and as 3 x dwordx3 (36 B, 4-B aligned)
//   patterns: "random" (each lane its own record), "runs16" (16-lane groups read 16
//             consecutive records, like the refs of one leaf), "same" (all lanes one record)
//   tables: 16 KiB (L1-resident) and 384 KiB (biplane's vertex pool: L2-resident)
// 8 waves per SIMD on every CU, 4 independent loads per lane in flight per trip.
// Build: hipcc --offload-arch=gfx950 -O3 -o lib/gather_rates tools/gather_rates.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int N_IT = 2048;

struct alignas(4) U3 {
    uint32_t x, y, z;
};

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// record index of load (i, u) for this lane
template <int PAT>
__device__ __forceinline__ uint32_t rec_of(uint32_t i, uint32_t u, uint32_t n_rec, uint32_t seed) {
    const uint32_t lane = threadIdx.x & 63u, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (PAT == 0) return hash32(seed ^ (((wave * 64u + lane) * N_IT + i) * 4u + u)) & (n_rec - 1u);
    if (PAT == 1) return (hash32(seed ^ (((wave * 4u + (lane >> 4)) * N_IT + i) * 4u + u)) + (lane & 15u)) & (n_rec - 1u);
    return hash32(seed ^ ((wave * N_IT + i) * 4u + u)) & (n_rec - 1u);
}

// KIND: 1 dword, 2 dwordx2, 3 dwordx3, 4 dwordx4, 12 = 3 x dwordx4 (48-B record), 9 = 3 x dwordx3 (36 B)
template <int KIND, int PAT>
__global__ __launch_bounds__(256, 2) void k_gather(const uint32_t* __restrict__ tab, uint32_t n_rec,
                                                   uint32_t* __restrict__ out, uint32_t seed) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < (uint32_t)N_IT; ++i) {
        uint32_t v[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            const uint32_t r = rec_of<PAT>(i, u, n_rec, seed);
            if (KIND == 1) {
                v[u] = tab[r];
            } else if (KIND == 2) {
                const uint2 a = reinterpret_cast<const uint2*>(tab)[r];
                v[u] = a.x ^ a.y;
            } else if (KIND == 3) {
                const U3 a = reinterpret_cast<const U3*>(tab)[r];
                v[u] = a.x ^ a.y ^ a.z;
            } else if (KIND == 4) {
                const uint4 a = reinterpret_cast<const uint4*>(tab)[r];
                v[u] = a.x ^ a.y ^ a.z ^ a.w;
            } else if (KIND == 12) {
                const uint4* p = reinterpret_cast<const uint4*>(tab) + 3 * (size_t)r;
                const uint4 a = p[0], b = p[1], c = p[2];
                v[u] = a.x ^ a.y ^ a.z ^ b.x ^ b.y ^ b.z ^ c.x ^ c.y ^ c.z;
            } else {
                const U3* p = reinterpret_cast<const U3*>(tab) + 3 * (size_t)r;
                const U3 a = p[0], b = p[1], c = p[2];
                v[u] = a.x ^ a.y ^ a.z ^ b.x ^ b.y ^ b.z ^ c.x ^ c.y ^ c.z;
            }
        }
        acc += (v[0] ^ v[1]) + (v[2] ^ v[3]);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int KIND, int PAT>
static void run(const char* kind, const char* pat, const uint32_t* tab, size_t tab_bytes, uint32_t* out,
                int blocks) {
    const int rec_b = KIND == 12 ? 48 : KIND == 9 ? 36 : 4 * KIND;
    uint32_t n_rec = 1;
    while ((size_t)(n_rec * 2) * rec_b <= tab_bytes) n_rec *= 2;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_gather<KIND, PAT>), dim3(blocks), dim3(256), 0, 0, tab, n_rec, out, 1u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_gather<KIND, PAT>), dim3(blocks), dim3(256), 0, 0, tab, n_rec, out, 7u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double recs = (double)blocks * 256 * N_IT * 4;
    const int insts = KIND == 12 || KIND == 9 ? 3 : 1;
    std::printf("{\"layout\": \"%s\", \"pattern\": \"%s\", \"table_KiB\": %.0f, \"ms\": %.3f, \"G_records_per_s\": %.2f, "
                "\"G_wave_loads_per_s\": %.3f, \"lane_GB_per_s\": %.0f}\n",
                kind, pat, (double)n_rec * rec_b / 1024.0, ms, recs / ms / 1e6, recs * insts / 64 / ms / 1e6,
                recs * rec_b / ms / 1e6);
}

template <int KIND>
static void run_all(const char* kind, const uint32_t* tab, uint32_t* out, int blocks) {
    for (size_t kib : {16, 384}) {
        run<KIND, 0>(kind, "random", tab, kib * 1024, out, blocks);
        run<KIND, 1>(kind, "runs16", tab, kib * 1024, out, blocks);
        run<KIND, 2>(kind, "same", tab, kib * 1024, out, blocks);
    }
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 2;
    const int blocks = p.multiProcessorCount * 8;  // 8 blocks of 4 waves per CU: 8 waves per SIMD
    uint32_t *tab = nullptr, *out = nullptr;
    if (hipMalloc(&tab, 1 << 20) != hipSuccess || hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 2;
    (void)hipMemset(tab, 0x5a, 1 << 20);
    run_all<1>("dword", tab, out, blocks);
    run_all<2>("dwordx2", tab, out, blocks);
    run_all<3>("dwordx3", tab, out, blocks);
    run_all<4>("dwordx4", tab, out, blocks);
    run_all<12>("tri 3 x dwordx4 (48 B)", tab, out, blocks);
    run_all<9>("tri 3 x dwordx3 (36 B)", tab, out, blocks);
    (void)hipFree(tab);
    (void)hipFree(out);
    return 0;
}
