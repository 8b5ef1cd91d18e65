// stub_hip.cpp — a host-only stand-in for the HIP runtime entry points librt_amd.so imports, for
// CPU tests of the runtime's host logic (tests/test_runtime_stub.py).  LD_PRELOADed, it answers
// every call the library makes: one "gfx950" device, host memory for device allocations, streams
// and events as tokens, kernel launches logged (block, grid, stream) and not run.  hipEventQuery answers what
// stub_hip_set_query() chose, so a test can make the launch pipeline see a failed earlier launch.
// Several devices (stub_hip_set_devices) for the multi-device frame (frame.hip): peer and strided
// copies really copy (host memory) and are logged with their shapes, launches log the current device.
// Test infrastructure only: never on the GPU box, never linked into the product.
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>

namespace {
thread_local hipError_t g_last = hipSuccess;
hipError_t g_query = hipSuccess;
int g_launches = 0;
int g_log[4096];  // block size of every launch, in order (128: a trace kernel, 256: the fold)
int g_log_stream[4096];  // the launch's stream: its token number (streams are numbered as created)
int g_log_grid[4096];    // the launch's workgroups
int g_log_device[4096];  // the current device at the launch
int g_tokens[1024];
int g_ndev = 1;
thread_local int g_dev = 0;
// copies: kind (1 peer, 2 strided, 3 linear async), current device, bytes / width, height, pitches
struct CopyRec { int kind, device; long long bytes, height, dpitch, spitch; };
CopyRec g_copies[4096];
int g_ncopies = 0;
void log_copy(int kind, long long bytes, long long height, long long dpitch, long long spitch) {
    if (g_ncopies < 4096) g_copies[g_ncopies] = CopyRec{kind, g_dev, bytes, height, dpitch, spitch};
    ++g_ncopies;
}
int g_next_token = 0;
dim3 g_grid, g_block;
size_t g_shmem = 0;
hipStream_t g_stream = nullptr;

hipError_t ret(hipError_t e) {
    if (e != hipSuccess) g_last = e;
    return e;
}
void* token() { return &g_tokens[(g_next_token++) & 1023]; }
}  // namespace

extern "C" {
// test controls
void stub_hip_set_query(int e) { g_query = static_cast<hipError_t>(e); }
int stub_hip_launches(void) { return g_launches; }
int stub_hip_launch_log(int* out, int n) {
    const int m = g_launches < 4096 ? g_launches : 4096;
    for (int i = 0; i < m && i < n; ++i) out[i] = g_log[i];
    return m;
}
void stub_hip_set_devices(int n) { g_ndev = n; }
int stub_hip_launch_devices(int* dev, int n) {
    const int m = g_launches < 4096 ? g_launches : 4096;
    for (int i = 0; i < m && i < n; ++i) dev[i] = g_log_device[i];
    return m;
}
// copies as 6 long longs each: kind, device, bytes (strided: width), height, dpitch, spitch
int stub_hip_copy_log(long long* out, int n) {
    const int m = g_ncopies < 4096 ? g_ncopies : 4096;
    for (int i = 0; i < m && i < n; ++i) {
        const CopyRec& c = g_copies[i];
        long long* o = out + 6 * i;
        o[0] = c.kind, o[1] = c.device, o[2] = c.bytes, o[3] = c.height, o[4] = c.dpitch, o[5] = c.spitch;
    }
    return m;
}
int stub_hip_launch_detail(int* stream, int* grid, int n) {
    const int m = g_launches < 4096 ? g_launches : 4096;
    for (int i = 0; i < m && i < n; ++i) stream[i] = g_log_stream[i], grid[i] = g_log_grid[i];
    return m;
}

hipError_t hipGetDeviceCount(int* n) { *n = g_ndev; return hipSuccess; }
hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_t* p, int dev) {
    if (dev < 0 || dev >= g_ndev) return ret(hipErrorInvalidDevice);
    std::memset(p, 0, sizeof(*p));
    std::strcpy(p->name, "stub");
    std::strcpy(p->gcnArchName, "gfx950:sramecc+:xnack-");
    p->multiProcessorCount = 256;
    return hipSuccess;
}
hipError_t hipSetDevice(int d) {
    if (d < 0 || d >= g_ndev) return ret(hipErrorInvalidDevice);
    g_dev = d;
    return hipSuccess;
}
hipError_t hipDeviceCanAccessPeer(int* can, int, int) { *can = 1; return hipSuccess; }
hipError_t hipDeviceEnablePeerAccess(int, unsigned) { return hipSuccess; }
hipError_t hipHostMalloc(void** p, size_t n, unsigned) {
    *p = std::calloc(1, n ? n : 1);
    return *p ? hipSuccess : ret(hipErrorOutOfMemory);
}
hipError_t hipHostFree(void* p) { std::free(p); return hipSuccess; }
hipError_t hipMemcpyPeerAsync(void* d, int, const void* s, int, size_t n, hipStream_t) {
    std::memcpy(d, s, n);
    log_copy(1, (long long)n, 1, 0, 0);
    return hipSuccess;
}
hipError_t hipMemcpy2DAsync(void* d, size_t dpitch, const void* s, size_t spitch, size_t w, size_t h,
                            hipMemcpyKind, hipStream_t) {
    if (w > dpitch || w > spitch) return ret(hipErrorInvalidPitchValue);
    for (size_t r = 0; r < h; ++r)
        std::memcpy(static_cast<char*>(d) + r * dpitch, static_cast<const char*>(s) + r * spitch, w);
    log_copy(2, (long long)w, (long long)h, (long long)dpitch, (long long)spitch);
    return hipSuccess;
}
hipError_t hipMalloc(void** p, size_t n) {
    *p = std::calloc(1, n ? n : 1);
    return *p ? hipSuccess : ret(hipErrorOutOfMemory);
}
hipError_t hipFree(void* p) { std::free(p); return hipSuccess; }
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) { std::memcpy(d, s, n); return hipSuccess; }
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
    std::memcpy(d, s, n);
    log_copy(3, (long long)n, 1, 0, 0);
    return hipSuccess;
}
hipError_t hipMemset(void* d, int v, size_t n) { std::memset(d, v, n); return hipSuccess; }
hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t) { std::memset(d, v, n); return hipSuccess; }
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) { *s = static_cast<hipStream_t>(token()); return hipSuccess; }
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t* e) { *e = static_cast<hipEvent_t>(token()); return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { *e = static_cast<hipEvent_t>(token()); return hipSuccess; }
hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) { *ms = 1.0f; return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return ret(g_query); }
hipError_t hipGetLastError(void) {
    const hipError_t e = g_last;
    g_last = hipSuccess;
    return e;
}
const char* hipGetErrorString(hipError_t e) {
    return e == hipErrorLaunchFailure ? "stub: unspecified launch failure" : "stub error";
}
hipError_t hipOccupancyMaxActiveBlocksPerMultiprocessor(int* n, const void*, int, size_t) { *n = 16; return hipSuccess; }
hipError_t hipLaunchKernel(const void*, dim3 grid, dim3 block, void**, size_t, hipStream_t s) {
    if (g_launches < 4096) {
        g_log[g_launches] = (int)block.x;
        g_log_stream[g_launches] = s ? (int)(static_cast<int*>(static_cast<void*>(s)) - g_tokens) : -1;
        g_log_grid[g_launches] = (int)grid.x;
        g_log_device[g_launches] = g_dev;
    }
    ++g_launches;
    return hipSuccess;
}
hipError_t __hipPushCallConfiguration(dim3 grid, dim3 block, size_t shmem, hipStream_t s) {
    g_grid = grid, g_block = block, g_shmem = shmem, g_stream = s;
    return hipSuccess;
}
hipError_t __hipPopCallConfiguration(dim3* grid, dim3* block, size_t* shmem, hipStream_t* s) {
    *grid = g_grid, *block = g_block, *shmem = g_shmem, *s = g_stream;
    return hipSuccess;
}
void** __hipRegisterFatBinary(const void*) { return reinterpret_cast<void**>(token()); }
void __hipRegisterFunction(void**, const void*, char*, const char*, unsigned, void*, void*, void*, void*, int*) {}
void __hipUnregisterFatBinary(void**) {}
}
