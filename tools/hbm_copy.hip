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

// ---------------------------------------------------------------- one-shot
// The decode launch's own read, with nothing else in it: config 3 is ONE launch
// that reads 35.7 MB once (32 kv heads x 8 KV chunks = 256 workgroups, each a
// contiguous `per_wg`-byte slice of the K cache and the same slice of the V
// cache, 69,632 B each), so its ceiling is not a 1 GiB stream's steady state
// but what one such launch achieves, launch ramp and drain included.
//   mode 0: LDS-DMA (buffer_load_dwordx4 ... nt lds, 1 KiB per wave
//           instruction), every wave issues its whole share up front, one
//           vmcnt(0) wait (the LDS holds the workgroup's whole slice)
//   mode 1: LDS-DMA in the split kernel's pattern: per wave 2 steps of K then V
//           pieces, one step in flight, wait, issue the next
//   mode 2: global_load_dwordx4 nt into registers, whole share in flight
// Each launch reads the next of `rot` rotated cache pairs (rot x 2 x wgs x
// per_wg bytes > the 256 MiB Infinity Cache).
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 srd_of(const void* base, unsigned bytes) {
    const unsigned long long p = (unsigned long long)base;
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)p);
    r.y = __builtin_amdgcn_readfirstlane((int)(unsigned)(p >> 32));
    r.z = __builtin_amdgcn_readfirstlane((int)bytes);
    r.w = 0x00020000;
    return r;
}
__device__ __forceinline__ void dma16_nt(const i32x4& srd, unsigned lds, unsigned off) {
    unsigned keep;
    lds = __builtin_amdgcn_readfirstlane(lds);
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen nt lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(off), "s"(srd), "s"(lds)
        : "memory");
}

// per_wg bytes of K and of V per workgroup; NW waves; the LDS holds 2 * per_wg
template <int NW, int MODE>
__global__ __launch_bounds__(NW * 64) void oneshot_read(const unsigned char* __restrict__ k,
                                                        const unsigned char* __restrict__ v, unsigned per_wg,
                                                        unsigned* sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned long long base = (unsigned long long)blockIdx.x * per_wg;
    const unsigned pieces = per_wg / 1024;            // 1-KiB pieces per stream
    const unsigned per_wave = (pieces + NW - 1) / NW;  // this wave's contiguous run of pieces
    const unsigned p0 = wave * per_wave;
    const i32x4 ks = srd_of(k + base, per_wg), vs = srd_of(v + base, per_wg);
    unsigned acc = 0;
    if constexpr (MODE == 0) {
        unsigned char* wb = lds + wave * per_wave * 2048;
        for (unsigned i = 0; i < per_wave; i++)
            dma16_nt(ks, (unsigned)(uintptr_t)(wb + i * 1024), (p0 + i) * 1024 + lane * 16);
        for (unsigned i = 0; i < per_wave; i++)
            dma16_nt(vs, (unsigned)(uintptr_t)(wb + (per_wave + i) * 1024), (p0 + i) * 1024 + lane * 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc = *(const unsigned*)(wb + lane * 4);
    } else if constexpr (MODE == 1) {
        // two steps, each half of the wave's K pieces then half of its V pieces
        unsigned char* wb = lds + wave * per_wave * 2048;
        const unsigned h = (per_wave + 1) / 2;
        for (int s = 0; s < 2; s++) {
            const unsigned a0 = s * h, a1 = s ? per_wave : h;
            for (unsigned i = a0; i < a1; i++)
                dma16_nt(ks, (unsigned)(uintptr_t)(wb + (i - a0) * 1024), (p0 + i) * 1024 + lane * 16);
            for (unsigned i = a0; i < a1; i++)
                dma16_nt(vs, (unsigned)(uintptr_t)(wb + (h + i - a0) * 1024), (p0 + i) * 1024 + lane * 16);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc ^= *(const unsigned*)(wb + lane * 4);
        }
    } else {
        const u32x4* kp = (const u32x4*)(k + base);
        const u32x4* vp = (const u32x4*)(v + base);
        constexpr int U = NW == 4 ? 36 : NW == 8 ? 18 : 10;  // >= 2 x pieces per wave (69,632 B per stream)
        u32x4 r[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            const unsigned pc = p0 + (i >> 1);
            const bool ok = (unsigned)(i >> 1) < per_wave && pc < pieces;
            r[i] = ok ? __builtin_nontemporal_load(((i & 1) ? vp : kp) + pc * 64 + lane) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int i = 0; i < U; i++) acc ^= r[i].x ^ r[i].y ^ r[i].z ^ r[i].w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// us per launch (average over `iters` back-to-back launches, HIP events), or <0 on error
extern "C" float hbm_oneshot(unsigned per_wg, int wgs, int waves, int mode, int rot, int iters) {
    const size_t stream = (size_t)per_wg * wgs;
    std::vector<unsigned char*> bufs(2 * rot, nullptr);
    unsigned* sink = nullptr;
    hipError_t e = hipMalloc(&sink, 64);
    for (auto& p : bufs)
        if (e == hipSuccess && (e = hipMalloc(&p, stream)) == hipSuccess) e = hipMemset(p, 1, stream);
    float us = -1.0f;
    const size_t lds = 2 * (size_t)((per_wg / 1024 + waves - 1) / waves) * 1024 * waves;
    auto launch = [&](int i) {
        const unsigned char* kk = bufs[2 * (i % rot)];
        const unsigned char* vv = bufs[2 * (i % rot) + 1];
        const dim3 g(wgs), b(64 * waves);
        if (waves == 8 && mode == 0) hipLaunchKernelGGL((oneshot_read<8, 0>), g, b, lds, 0, kk, vv, per_wg, sink);
        else if (waves == 8 && mode == 1) hipLaunchKernelGGL((oneshot_read<8, 1>), g, b, lds, 0, kk, vv, per_wg, sink);
        else if (waves == 8) hipLaunchKernelGGL((oneshot_read<8, 2>), g, b, 0, 0, kk, vv, per_wg, sink);
        else if (waves == 16 && mode == 0) hipLaunchKernelGGL((oneshot_read<16, 0>), g, b, lds, 0, kk, vv, per_wg, sink);
        else if (waves == 16 && mode == 1) hipLaunchKernelGGL((oneshot_read<16, 1>), g, b, lds, 0, kk, vv, per_wg, sink);
        else if (waves == 16) hipLaunchKernelGGL((oneshot_read<16, 2>), g, b, 0, 0, kk, vv, per_wg, sink);
        else if (mode == 0) hipLaunchKernelGGL((oneshot_read<4, 0>), g, b, lds, 0, kk, vv, per_wg, sink);
        else if (mode == 1) hipLaunchKernelGGL((oneshot_read<4, 1>), g, b, lds, 0, kk, vv, per_wg, sink);
        else hipLaunchKernelGGL((oneshot_read<4, 2>), g, b, 0, 0, kk, vv, per_wg, sink);
    };
    if (e == hipSuccess && lds > 160 * 1024 && mode != 2) e = hipErrorInvalidValue;
    if (e == hipSuccess && (waves == 4 || waves == 8 || waves == 16) && per_wg % 1024 == 0 && iters > 0 &&
        (waves != 4 || per_wg / 1024 / 4 <= 20) && (waves != 8 || per_wg / 1024 / 8 <= 20) &&
        (waves != 16 || per_wg / 1024 / 16 <= 20)) {
        for (auto* f : {(const void*)oneshot_read<4, 0>, (const void*)oneshot_read<4, 1>, (const void*)oneshot_read<8, 0>,
                        (const void*)oneshot_read<8, 1>, (const void*)oneshot_read<16, 0>,
                        (const void*)oneshot_read<16, 1>})
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        for (int i = 0; i < 2 * rot; i++) launch(i);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a, 0);
        for (int i = 0; i < iters; i++) launch(i);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        e = hipGetLastError();
        if (e == hipSuccess) us = ms * 1e3f / iters;
    } else if (e == hipSuccess) {
        e = hipErrorInvalidValue;
    }
    for (auto* p : bufs)
        if (p) (void)hipFree(p);
    if (sink) (void)hipFree(sink);
    return e == hipSuccess ? us : -(float)e;
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
