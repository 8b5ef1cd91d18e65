// Issue-rate microbenchmark of the VALU instruction classes the trace kernel uses, on gfx950:
// 8 independent register chains per lane, 32 instructions per loop trip (inline asm, so nothing
// is folded), 8 waves per SIMD on every CU.  Prints G wave-instructions/s per class.  This is the
// measured VALU ceiling DESIGN.md §5 prices the sphere-only kernel against.
// Build: hipcc --offload-arch=gfx950 -O3 -o lib/valu_rates tools/valu_rates.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int N_IT = 16384;

#define BODY(INSN, T, CONS)                                                        \
    T a[8];                                                                        \
    const T t = s + (T)1;                                                          \
    for (int j = 0; j < 8; ++j) a[j] = (T)(threadIdx.x * (j + 3)) + s;             \
    for (int i = 0; i < N_IT; ++i) {                                               \
        _Pragma("unroll") for (int r = 0; r < 4; ++r)                             \
        _Pragma("unroll") for (int j = 0; j < 8; ++j)                             \
            asm volatile(INSN : "+v"(a[j]) : CONS(s), CONS(t));                             \
    }                                                                              \
    T acc = 0;                                                                     \
    for (int j = 0; j < 8; ++j) acc += a[j];                                       \
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;

__global__ void k_mul_f32(float* out, float s) { BODY("v_mul_f32 %0, %0, %1 ; %2", float, "v") }
__global__ void k_fma_f32(float* out, float s) { BODY("v_fma_f32 %0, %0, %1, %2", float, "v") }
__global__ void k_add_u32(uint32_t* out, uint32_t s) { BODY("v_add_u32 %0, %0, %1 ; %2", uint32_t, "v") }
__global__ void k_mul_lo_u32(uint32_t* out, uint32_t s) { BODY("v_mul_lo_u32 %0, %0, %1 ; %2", uint32_t, "v") }
__global__ void k_mul_u24(uint32_t* out, uint32_t s) { BODY("v_mul_u32_u24 %0, %0, %1 ; %2", uint32_t, "v") }
__global__ void k_fma_f64(double* out, double s) { BODY("v_fma_f64 %0, %0, %1, %2", double, "v") }
__global__ void k_sqrt_f32(float* out, float s) { BODY("v_sqrt_f32 %0, %0 ; %1 %2", float, "v") }
__global__ void k_fma_f32_same(float* out, float s) { BODY("v_fma_f32 %0, %0, %1, %1 ; %2", float, "v") }
__global__ void k_mul_f32_sq(float* out, float s) { BODY("v_mul_f32 %0, %0, %0 ; %1 %2", float, "v") }
__global__ void k_mul_f32_same(float* out, float s) { BODY("v_mul_f32 %0, %1, %1 ; %2", float, "v") }
__global__ void k_rcp_f32(float* out, float s) { BODY("v_rcp_f32 %0, %0 ; %1 %2", float, "v") }
// packed f32 on 64-bit register pairs (the double only carries the two floats' bits)
__global__ void k_pk_mul_f32(double* out, double s) { BODY("v_pk_mul_f32 %0, %0, %1 ; %2", double, "v") }
__global__ void k_pk_add_f32(double* out, double s) { BODY("v_pk_add_f32 %0, %0, %1 ; %2", double, "v") }
__global__ void k_pk_fma_f32(double* out, double s) { BODY("v_pk_fma_f32 %0, %0, %1, %2", double, "v") }

template <class K, class T>
static void run(const char* name, K k, T* buf, T s, int blocks) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, s);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, s);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double winst = (double)blocks * 256 / 64 * N_IT * 32;
    std::printf("{\"insn\": \"%s\", \"ms\": %.3f, \"G_winst_per_s\": %.1f}\n", name, ms, winst / ms / 1e6);
}

int main() {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 2;
    const int blocks = p.multiProcessorCount * 8;  // 8 blocks of 4 waves: 8 waves per SIMD
    void* buf = nullptr;
    if (hipMalloc(&buf, (size_t)blocks * 256 * 8) != hipSuccess) return 2;
    run("v_mul_f32", k_mul_f32, (float*)buf, 1.0f, blocks);
    run("v_mul_f32 (x * x)", k_mul_f32_sq, (float*)buf, 1.0f, blocks);
    run("v_mul_f32 (d = s * s)", k_mul_f32_same, (float*)buf, 1.0f, blocks);
    run("v_fma_f32", k_fma_f32, (float*)buf, 1.0f, blocks);
    run("v_fma_f32 (b = c)", k_fma_f32_same, (float*)buf, 1.0f, blocks);
    run("v_add_u32", k_add_u32, (uint32_t*)buf, 1u, blocks);
    run("v_mul_lo_u32", k_mul_lo_u32, (uint32_t*)buf, 3u, blocks);
    run("v_mul_u32_u24", k_mul_u24, (uint32_t*)buf, 3u, blocks);
    run("v_fma_f64", k_fma_f64, (double*)buf, 1.0, blocks);
    run("v_sqrt_f32", k_sqrt_f32, (float*)buf, 1.0f, blocks);
    run("v_rcp_f32", k_rcp_f32, (float*)buf, 1.0f, blocks);
    run("v_pk_mul_f32", k_pk_mul_f32, (double*)buf, 1.0, blocks);
    run("v_pk_add_f32", k_pk_add_f32, (double*)buf, 1.0, blocks);
    run("v_pk_fma_f32", k_pk_fma_f32, (double*)buf, 1.0, blocks);
    (void)hipFree(buf);
    return 0;
}
