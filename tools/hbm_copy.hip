// hbm_copy.hip -- measured HBM ceilings for bench.py's roofline (a measurement
// probe, not part of libfattn): a global_load_dwordx4 / global_store_dwordx4
// device copy (the form MI355X_MICROARCH.md's 6.29 TB/s "float4 copy" figure is
// quoted for) and a dwordx4 read-only stream, each over buffers far larger than
// the 256 MiB Infinity Cache.  Built into ggml-cuda-experiments_amd/lib/
// libhbmcopy.so; bench.py loads it with ctypes after torch (one HIP runtime).
//
//   int hbm_probe(size_t bytes, int iters, float* copy_gbs, float* read_gbs)
//     copy_gbs: (read + written bytes) / median launch time; read_gbs: bytes /
//     median launch time of the read stream.  Returns 0, or a hipError_t.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kUnroll = 4;  // 16-B loads in flight per lane before the stores

// each workgroup copies one contiguous slice, kUnroll x 4 KiB per iteration
__global__ __launch_bounds__(kThreads) void copy_x4(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                     size_t per_wg) {
    const u32x4* s = src + blockIdx.x * per_wg;
    u32x4* d = dst + blockIdx.x * per_wg;
    for (size_t i = threadIdx.x; i < per_wg; i += kThreads * kUnroll) {
        u32x4 v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++) v[u] = __builtin_nontemporal_load(s + i + u * kThreads);
#pragma unroll
        for (int u = 0; u < kUnroll; u++) __builtin_nontemporal_store(v[u], d + i + u * kThreads);
    }
}

__global__ __launch_bounds__(kThreads) void read_x4(const u32x4* __restrict__ src, size_t per_wg, unsigned* sink) {
    const u32x4* s = src + blockIdx.x * per_wg;
    unsigned acc = 0;
    for (size_t i = threadIdx.x; i < per_wg; i += kThreads * 2 * kUnroll) {
        u32x4 v[2 * kUnroll];
#pragma unroll
        for (int u = 0; u < 2 * kUnroll; u++) v[u] = __builtin_nontemporal_load(s + i + u * kThreads);
#pragma unroll
        for (int u = 0; u < 2 * kUnroll; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the loads alive
}

template <typename F>
static float median_us(F launch, int iters) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return -1.0f;
    std::vector<float> t;
    for (int i = 0; i < iters + 2; i++) {
        (void)hipEventRecord(a, 0);
        launch();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (i >= 2) t.push_back(ms * 1e3f);
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

extern "C" int hbm_probe(size_t bytes, int iters, float* copy_gbs, float* read_gbs) {
    const int wgs = 256 * 8;  // 8 workgroups per CU
    const size_t per_wg = bytes / 16 / wgs / (kThreads * 2 * kUnroll) * (kThreads * 2 * kUnroll);
    const size_t n = per_wg * wgs;
    if (per_wg == 0 || iters < 1) return (int)hipErrorInvalidValue;
    u32x4 *a = nullptr, *b = nullptr;
    unsigned* sink = nullptr;
    hipError_t e = hipMalloc(&a, n * 16);
    if (e == hipSuccess) e = hipMalloc(&b, n * 16);
    if (e == hipSuccess) e = hipMalloc(&sink, 64);
    if (e == hipSuccess) e = hipMemset(a, 1, n * 16);
    if (e == hipSuccess) {
        const float tc = median_us([&] { hipLaunchKernelGGL(copy_x4, dim3(wgs), dim3(kThreads), 0, 0, a, b, per_wg); },
                                   iters);
        const float tr = median_us([&] { hipLaunchKernelGGL(read_x4, dim3(wgs), dim3(kThreads), 0, 0, a, per_wg, sink); },
                                   iters);
        e = hipGetLastError();
        *copy_gbs = (float)(2.0 * n * 16 / (tc * 1e-6) / 1e9);
        *read_gbs = (float)(1.0 * n * 16 / (tr * 1e-6) / 1e9);
    }
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    if (sink) (void)hipFree(sink);
    return (int)e;
}
