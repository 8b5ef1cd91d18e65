// include/rt_libm.h on gfx950 against the host C library (glibc sinf, cosf, powf), bit for bit:
// every angle 2*pi*v the renderer forms (v = j * 2^-24), 2^24 hashed floats in [-2 pi, 2 pi],
// and powf(x, 5) on 2^24 hashed x in [0, 1.001] plus 2^20 in [-0.001, 0].  The device computes,
// the host compares.  Prints one JSON line; exit 1 on any mismatch, 2 on a HIP error.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -o check_libm_gpu <this>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "rt_libm.h"

constexpr uint32_t N = 1u << 24;

__host__ __device__ inline uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__host__ __device__ inline float angle(uint32_t j) {
    const float v = (float)j * (1.0f / 16777216.0f);
    return 2.0f * 3.14159265358979323846f * v;
}
__host__ __device__ inline float wide(uint32_t j) {  // hashed float in [-2 pi, 2 pi]
    const uint32_t h = hash(j ^ 0x2545f491u);
    const float m = (float)(h >> 9) * (1.0f / 8388608.0f);
    return (h & 1u ? -1.0f : 1.0f) * m * 6.2831855f;
}
__host__ __device__ inline float pw(uint32_t j) {  // hashed x in [0, 1.001], then [-0.001, 0]
    if (j < N) return (float)(hash(j) >> 8) * (1.001f / 16777216.0f);
    return -(float)(hash(j) >> 8) * (0.001f / 16777216.0f);
}

__global__ void k_sincos(float2* out, int which) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= N) return;
    const float th = which ? wide(j) : angle(j);
    float s = 0.f, c = 0.f;
    if (!rt_sincosf(th, &s, &c)) s = c = __builtin_nanf("");
    out[j] = make_float2(s, c);
}
__global__ void k_pow(float* out, uint32_t n) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    out[j] = rt_powf5(pw(j));
}

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

int main() {
    float2* d2;
    float* d1;
    const uint32_t npow = N + (1u << 20);
    if (hipMalloc(&d2, N * sizeof(float2)) != hipSuccess || hipMalloc(&d1, npow * sizeof(float)) != hipSuccess)
        return 2;
    std::vector<float2> h2(N);
    std::vector<float> h1(npow);
    unsigned long long bad[3] = {0, 0, 0};
    uint32_t first[3] = {0, 0, 0};
    for (int which = 0; which < 2; ++which) {
        hipLaunchKernelGGL(k_sincos, dim3(N / 256), dim3(256), 0, 0, d2, which);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        if (hipMemcpy(h2.data(), d2, N * sizeof(float2), hipMemcpyDeviceToHost) != hipSuccess) return 2;
        for (uint32_t j = 0; j < N; ++j) {
            volatile float th = which ? wide(j) : angle(j);
            const float s = sinf(th), c = cosf(th);
            if (bits(s) != bits(h2[j].x) || bits(c) != bits(h2[j].y)) {
                if (!bad[which]) first[which] = bits(th);
                ++bad[which];
            }
        }
    }
    hipLaunchKernelGGL(k_pow, dim3((npow + 255) / 256), dim3(256), 0, 0, d1, npow);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    if (hipMemcpy(h1.data(), d1, npow * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    for (uint32_t j = 0; j < npow; ++j) {
        volatile float x = pw(j), y = 5.0f;
        const float g = powf(x, y);
        if (bits(g) != bits(h1[j]) && !(std::isnan(g) && std::isnan(h1[j]))) {
            if (!bad[2]) first[2] = bits(x);
            ++bad[2];
        }
    }
    std::printf("{\"device\": \"gfx950\", \"angles_2pi_v\": [%u, %llu, \"0x%08x\"], "
                "\"hashed_pm2pi\": [%u, %llu, \"0x%08x\"], \"powf5\": [%u, %llu, \"0x%08x\"], "
                "\"format\": \"[tested, mismatches vs host glibc, first mismatching input bits]\"}\n",
                N, bad[0], first[0], N, bad[1], first[1], npow, bad[2], first[2]);
    (void)hipFree(d2);
    (void)hipFree(d1);
    return (bad[0] | bad[1] | bad[2]) ? 1 : 0;
}
