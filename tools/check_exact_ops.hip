// Exhaustive / large-sample checks, on the GPU, of the fast exact-arithmetic identities the
// trace kernel relies on (trace.hip: rcp_exact, div_exact, sqrt_rn, sincos).  Each compares against the
// IEEE operation the kernel would otherwise issue (hipcc's correctly rounded 1.0f/b, a/b) or
// against the separate ocml calls.  Usage: check_exact_ops  (prints one JSON line; exit 1 on any
// mismatch).  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o check_exact_ops <this>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ float rcp_exact(float b) {
    const float y = __builtin_amdgcn_rcpf(b);
    const float e = fmaf(-b, y, 1.0f);
    return fmaf(e, y, y);
}
__device__ __forceinline__ float div_mk(float a, float b, float r) {
    const float q0 = a * r;
    const float res = fmaf(-q0, b, a);
    return fmaf(res, r, q0);
}

struct Stats {
    unsigned long long tested, bad;
    uint32_t first_bad[8];
};

__device__ void record(Stats* s, uint32_t bits) {
    const unsigned long long k = atomicAdd(&s->bad, 1ull);
    if (k < 8) s->first_bad[k] = bits;
}

// every positive normal b with exponent in [-126+lo, 127-hi]: rcp_exact(b) == 1.0f / b
__global__ void k_rcp(Stats* s, uint32_t e_lo, uint32_t e_hi) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long n = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (1ull << 31); i += stride) {
        const uint32_t bits = (uint32_t)i;
        const uint32_t ex = bits >> 23;
        if (ex < e_lo || ex > e_hi) continue;
        const float b = __uint_as_float(bits);
        ++n;
        if (__float_as_uint(rcp_exact(b)) != __float_as_uint(1.0f / b)) record(s, bits);
        if (__float_as_uint(rcp_exact(-b)) != __float_as_uint(1.0f / -b)) record(s, bits | 0x80000000u);
    }
    atomicAdd(&s->tested, 2 * n);
}

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// random (a, b) pairs, |a| in [2^-60, 2^60) or 0, b in the same range: Markstein quotient with
// the exact reciprocal == a / b
__global__ void k_div(Stats* s, uint32_t rounds) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long n = 0;
    for (uint32_t k = 0; k < rounds; ++k) {
        const uint32_t h1 = hash(t * 2654435761u + k * 0x9e3779b9u + 1u);
        const uint32_t h2 = hash(h1 ^ 0x5bd1e995u);
        // exponents in [127-60, 127+60): bits = sign | exp | mantissa
        const uint32_t ea = 67u + (h1 >> 8) % 120u, eb = 67u + (h2 >> 8) % 120u;
        const float a = __uint_as_float((h1 & 0x80000000u) | (ea << 23) | (hash(h1) & 0x7fffffu));
        const float b = __uint_as_float((h2 & 0x80000000u) | (eb << 23) | (hash(h2) & 0x7fffffu));
        const float q = div_mk(a, b, rcp_exact(b));
        ++n;
        if (__float_as_uint(q) != __float_as_uint(a / b)) record(s, __float_as_uint(a));
    }
    atomicAdd(&s->tested, n);
}

// normalize's quotients: components |a_i| <= n with n = sqrt(dot): a / n for n in [2^-30, 2^30]
// and a = n * u, u in (-1, 1] on a dense grid (the realistic operand distribution)
__global__ void k_norm(Stats* s, uint32_t rounds) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long n = 0;
    for (uint32_t k = 0; k < rounds; ++k) {
        const uint32_t h1 = hash(t * 747796405u + k * 2891336453u + 7u);
        const float nn = __uint_as_float(((97u + (h1 >> 24) % 60u) << 23) | (hash(h1) & 0x7fffffu));
        const float u = (float)(int32_t)hash(h1 ^ 0x1234567u) * 0x1p-31f;
        const float a = nn * u;
        const float q = div_mk(a, nn, rcp_exact(nn));
        ++n;
        if (__float_as_uint(q) != __float_as_uint(a / nn)) record(s, __float_as_uint(a));
    }
    atomicAdd(&s->tested, n);
}

// sqrt_fix(x) = v_sqrt_f32 + the +-1 ulp FMA correction (the kernels' sqrt_rn until round 4),
// without hipcc's denormal scaling and class check: == sqrtf(x) for every x in [lo, +inf] (bit
// patterns), lo = 0 for the full check; the per-range counts locate any failure
__device__ __forceinline__ float sqrt_fix(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u), su = __uint_as_float(__float_as_uint(s) + 1u);
    float r = fmaf(-sd, s, x) <= 0.0f ? sd : s;
    r = fmaf(-su, s, x) > 0.0f ? su : r;
    return r;
}
__global__ void k_sqrt(Stats* s, uint32_t lo_bits) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long n = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (1ull << 31); i += stride) {
        const uint32_t bits = (uint32_t)i;
        const uint32_t ex = bits >> 23;
        if (bits < lo_bits || bits > 0x7f800000u) continue;
        (void)ex;
        const float x = __uint_as_float(bits);
        ++n;
        if (__float_as_uint(sqrt_fix(x)) != __float_as_uint(sqrtf(x))) record(s, bits);
    }
    atomicAdd(&s->tested, n);
}

// sqrt_rn(x) of trace.hip (round 4): the reciprocal square root's Newton correction of
// s = x * rsq(x) with one rounding, s + (x - s^2) * rsq(x) / 2 (Markstein): 5 instructions
// instead of sqrt_fix's 9; == sqrtf(x) for every x in [2^-80, FLT_MAX]
__device__ __forceinline__ float sqrt_rsq(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float s = x * y;
    const float r = fmaf(-s, s, x);
    return fmaf(r, 0.5f * y, s);
}
__global__ void k_sqrt_rsq(Stats* s, uint32_t lo_bits, uint32_t hi_bits) {
    const uint32_t stride = gridDim.x * blockDim.x;
    unsigned long long n = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (1ull << 31); i += stride) {
        const uint32_t bits = (uint32_t)i;
        if (bits < lo_bits || bits > hi_bits) continue;
        const float x = __uint_as_float(bits);
        ++n;
        if (__float_as_uint(sqrt_rsq(x)) != __float_as_uint(sqrtf(x))) record(s, bits);
    }
    atomicAdd(&s->tested, n);
}

// theta = 2*pi*v for every v = j * 2^-24 in [0, 1): sincosf == (sinf, cosf)
__global__ void k_sincos(Stats* s) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= (1u << 24)) return;
    const float v = (float)j * 0x1p-24f;
    const float th = 2.0f * 3.14159265358979323846f * v;
    float sn, cs;
    sincosf(th, &sn, &cs);
    if (__float_as_uint(sn) != __float_as_uint(sinf(th)) || __float_as_uint(cs) != __float_as_uint(cosf(th)))
        record(s, j);
    atomicAdd(&s->tested, 1ull);
}

static int report(const char* name, Stats* d) {
    Stats h;
    (void)hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
    std::printf("\"%s\": {\"tested\": %llu, \"bad\": %llu, \"first_bad\": [", name, h.tested, h.bad);
    for (unsigned k = 0; k < 8 && k < h.bad; ++k) std::printf("%s\"0x%08x\"", k ? ", " : "", h.first_bad[k]);
    std::printf("]}");
    return h.bad ? 1 : 0;
}

int main() {
    Stats* d;
    if (hipMalloc(&d, 9 * sizeof(Stats)) != hipSuccess) return 2;
    (void)hipMemset(d, 0, 9 * sizeof(Stats));
    // reciprocal over |b| in [2^-60, 2^60]: biased exponents 67..187
    hipLaunchKernelGGL(k_rcp, dim3(8192), dim3(256), 0, 0, d + 0, 67u, 187u);
    hipLaunchKernelGGL(k_div, dim3(8192), dim3(256), 0, 0, d + 1, 2048u);
    hipLaunchKernelGGL(k_norm, dim3(8192), dim3(256), 0, 0, d + 2, 1024u);
    hipLaunchKernelGGL(k_sincos, dim3((1u << 24) / 256), dim3(256), 0, 0, d + 3);
    hipLaunchKernelGGL(k_sqrt, dim3(8192), dim3(256), 0, 0, d + 4, 47u << 23);  // [2^-80, inf]
    hipLaunchKernelGGL(k_sqrt, dim3(8192), dim3(256), 0, 0, d + 5, 1u << 23);   // normals
    hipLaunchKernelGGL(k_sqrt, dim3(8192), dim3(256), 0, 0, d + 6, 0u);         // everything >= 0
    hipLaunchKernelGGL(k_sqrt_rsq, dim3(8192), dim3(256), 0, 0, d + 7, 47u << 23, 0x7f7fffffu);  // [2^-80, max]
    hipLaunchKernelGGL(k_sqrt_rsq, dim3(8192), dim3(256), 0, 0, d + 8, 1u << 23, 0x7f7fffffu);   // normals
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    int bad = 0;
    std::printf("{");
    bad |= report("rcp_exact_all_normal_2^-60_2^60", d + 0);
    std::printf(", ");
    bad |= report("markstein_div_random_pairs", d + 1);
    std::printf(", ");
    bad |= report("normalize_quotients", d + 2);
    std::printf(", ");
    bad |= report("sincosf_vs_sinf_cosf", d + 3);
    std::printf(", ");
    bad |= report("sqrt_fix_2^-80_to_inf", d + 4);
    std::printf(", ");
    (void)report("sqrt_fix_normal_to_inf_info", d + 5);  // informational: fails below 2^-80
    std::printf(", ");
    (void)report("sqrt_fix_all_nonneg_info", d + 6);
    std::printf(", ");
    bad |= report("sqrt_rn_rsq_2^-80_to_max", d + 7);
    std::printf(", ");
    (void)report("sqrt_rn_rsq_normal_to_max_info", d + 8);  // informational: fails below 2^-80
    std::printf("}\n");
    (void)hipFree(d);
    return bad;
}
