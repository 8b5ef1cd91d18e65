// Gather-cost sweep of the vector-memory path on gfx950 ("Mesh roofline"): the
// chip-wide rate of wave-loads of a given shape — record size, active lanes A, lanes per group G
// reading G consecutive records from a random start (G = 1: every lane its own random record;
// G = 0: every lane the same record) — from an L1-resident (16 KiB) and an L2-resident (1 MiB)
// table, with every SIMD holding 8 waves that each keep 4 independent loads in flight.  Beside
// each rate: the distinct 128-B lines one such wave-load touches, averaged over 4096 wave-loads of
// the same address function on the host.  tools/mesh_roofline.py prices the mesh kernel's load
// classes (their measured lanes and lines per wave-load) with these curves.
// Build: hipcc --offload-arch=gfx950 -O3 -o lib/gather_sweep tools/gather_sweep.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <set>

constexpr int N_IT = 1024;

__host__ __device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// record of load (i, u) of `lane` in `wave`: groups of G lanes read G consecutive records
__host__ __device__ __forceinline__ uint32_t rec_of(uint32_t wave, uint32_t lane, uint32_t i, uint32_t u, uint32_t G,
                                                    uint32_t n_rec, uint32_t seed) {
    const uint32_t grp = G ? lane / G : 0u, off = G ? lane % G : 0u;
    return (hash32(seed ^ (((wave * 64u + grp) * N_IT + i) * 4u + u)) + off) & (n_rec - 1u);
}

// KIND: 1 dword, 2 dwordx2, 4 dwordx4, 12 = 3 x dwordx4 (48-B record)
template <int KIND>
__global__ __launch_bounds__(256, 2) void k_sweep(const uint32_t* __restrict__ tab, uint32_t n_rec, uint32_t G,
                                                  uint32_t A, uint32_t* __restrict__ out, uint32_t seed) {
    const uint32_t lane = threadIdx.x & 63u, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint32_t acc = 0;
    if (lane < A) {
        for (uint32_t i = 0; i < (uint32_t)N_IT; ++i) {
            uint32_t v[4];
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) {
                const uint32_t r = rec_of(wave, lane, i, u, G, n_rec, seed);
                if (KIND == 1) {
                    v[u] = tab[r];
                } else if (KIND == 2) {
                    const uint2 a = reinterpret_cast<const uint2*>(tab)[r];
                    v[u] = a.x ^ a.y;
                } else if (KIND == 4) {
                    const uint4 a = reinterpret_cast<const uint4*>(tab)[r];
                    v[u] = a.x ^ a.y ^ a.z ^ a.w;
                } else {
                    const uint4* p = reinterpret_cast<const uint4*>(tab) + 3 * (size_t)r;
                    const uint4 a = p[0], b = p[1], c = p[2];
                    v[u] = a.x ^ a.y ^ a.z ^ b.x ^ b.y ^ b.z ^ c.x ^ c.y ^ c.z;
                }
            }
            acc += (v[0] ^ v[1]) + (v[2] ^ v[3]);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

static double lines_per_wave_load(int rec_b, uint32_t G, uint32_t A, uint32_t n_rec) {
    double total = 0;
    for (uint32_t s = 0; s < 4096; ++s) {
        std::set<uint64_t> lines;
        for (uint32_t l = 0; l < A; ++l) lines.insert((uint64_t)rec_of(s / 64, l, s % 64, 0, G, n_rec, 7u) * rec_b / 128);
        total += (double)lines.size();
    }
    return total / 4096.0;
}

template <int KIND>
static void run(const char* kind, size_t tab_bytes, uint32_t G, uint32_t A, const uint32_t* tab, uint32_t* out,
                int blocks) {
    const int rec_b = KIND == 12 ? 48 : 4 * KIND;
    uint32_t n_rec = 1;
    while ((size_t)(n_rec * 2) * rec_b <= tab_bytes) n_rec *= 2;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_sweep<KIND>), dim3(blocks), dim3(256), 0, 0, tab, n_rec, G, A, out, 1u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_sweep<KIND>), dim3(blocks), dim3(256), 0, 0, tab, n_rec, G, A, out, 7u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    const int insts = KIND == 12 ? 3 : 1;
    const double wl = (double)blocks * 4 * N_IT * 4 * insts;  // wave-loads (4 waves per block)
    std::printf("{\"kind\": \"%s\", \"table_KiB\": %.0f, \"group\": %u, \"active_lanes\": %u, "
                "\"lines_per_wave_load\": %.2f, \"ms\": %.3f, \"G_wave_loads_per_s\": %.3f}\n",
                kind, (double)n_rec * rec_b / 1024.0, G, A, lines_per_wave_load(rec_b, G, A, n_rec), ms, wl / ms / 1e6);
    std::fflush(stdout);
}

template <int KIND>
static void sweep(const char* kind, const uint32_t* tab, uint32_t* out, int blocks) {
    for (size_t kib : {16, 1024})
        for (uint32_t A : {64u, 32u, 16u})
            for (uint32_t G : {0u, 64u, 16u, 8u, 4u, 2u, 1u}) {
                if (G > A) continue;
                run<KIND>(kind, kib * 1024, G, A, tab, out, blocks);
            }
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 2;
    const int blocks = p.multiProcessorCount * 8;  // 8 blocks of 4 waves per CU: 8 waves per SIMD
    uint32_t *tab = nullptr, *out = nullptr;
    if (hipMalloc(&tab, 4 << 20) != hipSuccess || hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 2;
    (void)hipMemset(tab, 0x5a, 4 << 20);
    sweep<1>("dword", tab, out, blocks);
    sweep<2>("dwordx2", tab, out, blocks);
    sweep<4>("dwordx4", tab, out, blocks);
    sweep<12>("tri48", tab, out, blocks);
    (void)hipFree(tab);
    (void)hipFree(out);
    return 0;
}
