// hbm_probe.hip -- calibration probe: how fast can one launch stream B bytes
// from HBM on this MI355X, as a function of grid shape and load form?
// (Diagnostic tool, not part of libfattn.)  Sets the practical ceiling the
// decode kernel's roofline fraction should be read against.
//
//   vgpr : global_load_dwordx4 into registers, U loads in flight per lane
//   dma  : global_load_lds_dwordx4 (1 KiB per wave instruction) into LDS,
//          U pieces in flight per wave, like fattn_split_kernel's step copy
//
// Each workgroup (256 threads) streams a contiguous slice of the buffer; the
// buffer is one of R rotated copies (R * B > 256 MiB Infinity Cache).
// Output: one line per configuration: us per launch (hipEvent over L launches)
// and GB/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void vgpr_read(const u32x4* __restrict__ src, size_t per_wg, unsigned* sink) {
    const u32x4* p = src + blockIdx.x * (per_wg / 16);
    const size_t n = per_wg / 16;
    unsigned acc = 0;
    for (size_t i = threadIdx.x; i < n; i += 256 * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t j = i + (size_t)u * 256;
            v[u] = j < n ? p[j] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int U>
__global__ __launch_bounds__(256) void dma_read(const unsigned char* __restrict__ src, size_t per_wg, unsigned* sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned char* p = src + blockIdx.x * per_wg;
    const size_t pieces = per_wg / 1024;  // 1 KiB per wave instruction
    unsigned char* wb = lds + wave * U * 1024;
    unsigned acc = 0;
    for (size_t i = wave; i < pieces; i += 4 * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t pc = i + (size_t)u * 4;
            const size_t off = (pc < pieces ? pc : i) * 1024 + lane * 16;
            __builtin_amdgcn_global_load_lds((const void*)(p + off), (void*)(wb + u * 1024), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc ^= *(const unsigned*)(wb + lane * 4);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// NW waves per workgroup, U pieces (1 KiB) in flight per wave before each wait
template <int NW, int U>
__global__ __launch_bounds__(NW * 64) void dma_read_w(const unsigned char* __restrict__ src, size_t per_wg, unsigned* sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned char* p = src + blockIdx.x * per_wg;
    const size_t pieces = per_wg / 1024;
    unsigned char* wb = lds + wave * U * 1024;
    unsigned acc = 0;
    for (size_t i = wave; i < pieces; i += NW * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t pc = i + (size_t)u * NW;
            const size_t off = (pc < pieces ? pc : i) * 1024 + lane * 16;
            __builtin_amdgcn_global_load_lds((const void*)(p + off), (void*)(wb + u * 1024), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc ^= *(const unsigned*)(wb + lane * 4);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <typename K>
static float time_it(K launch, int L) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 5; i++) launch(i);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, 0));
    for (int i = 0; i < L; i++) launch(i);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ms * 1e3f / L;
}

int main(int argc, char** argv) {
    const size_t B = argc > 1 ? strtoull(argv[1], nullptr, 10) : 35692544ull;  // config-3 bytes
    const int R = 16, L = 200;
    std::vector<unsigned char*> bufs(R);
    for (auto& p : bufs) {
        CHECK(hipMalloc(&p, B + (1 << 20)));
        CHECK(hipMemset(p, 1, B + (1 << 20)));
    }
    unsigned* sink;
    CHECK(hipMalloc(&sink, 64));
    printf("bytes per launch %zu, %d rotated buffers\n", B, R);
    const int wgs_list[] = {256, 512, 1024, 2048, 4096};
    for (int wgs : wgs_list) {
        const size_t per = (B / wgs) / 4096 * 4096;
        const double bytes = (double)per * wgs;
        auto v4 = [&](int i) { hipLaunchKernelGGL(vgpr_read<4>, dim3(wgs), dim3(256), 0, 0, (const u32x4*)bufs[i % R], per, sink); };
        auto v8 = [&](int i) { hipLaunchKernelGGL(vgpr_read<8>, dim3(wgs), dim3(256), 0, 0, (const u32x4*)bufs[i % R], per, sink); };
        auto d4 = [&](int i) { hipLaunchKernelGGL(dma_read<4>, dim3(wgs), dim3(256), 4 * 4 * 1024, 0, bufs[i % R], per, sink); };
        auto d8 = [&](int i) { hipLaunchKernelGGL(dma_read<8>, dim3(wgs), dim3(256), 4 * 8 * 1024, 0, bufs[i % R], per, sink); };
        auto d16 = [&](int i) { hipLaunchKernelGGL(dma_read<16>, dim3(wgs), dim3(256), 4 * 16 * 1024, 0, bufs[i % R], per, sink); };
        const float t_v4 = time_it(v4, L), t_v8 = time_it(v8, L), t_d4 = time_it(d4, L), t_d8 = time_it(d8, L),
                    t_d16 = time_it(d16, L);
        printf("wgs %5d per_wg %7zu B | vgpr U4 %6.2f us %6.0f GB/s | vgpr U8 %6.2f us %6.0f GB/s | "
               "dma U4 %6.2f us %6.0f GB/s | dma U8 %6.2f us %6.0f GB/s | dma U16 %6.2f us %6.0f GB/s\n",
               wgs, per, t_v4, bytes / t_v4 * 1e-3, t_v8, bytes / t_v8 * 1e-3, t_d4, bytes / t_d4 * 1e-3, t_d8,
               bytes / t_d8 * 1e-3, t_d16, bytes / t_d16 * 1e-3);
    }
    // 256 workgroups of NW waves (one per CU): U pieces in flight per wave
    {
        const int wgs = 256;
        const size_t per = (B / wgs) / 1024 * 1024;
        const double bytes = (double)per * wgs;
        auto w16u2 = [&](int i) { hipLaunchKernelGGL((dma_read_w<16, 2>), dim3(wgs), dim3(1024), 16 * 2 * 1024, 0, bufs[i % R], per, sink); };
        auto w16u4 = [&](int i) { hipLaunchKernelGGL((dma_read_w<16, 4>), dim3(wgs), dim3(1024), 16 * 4 * 1024, 0, bufs[i % R], per, sink); };
        auto w16u9 = [&](int i) { hipLaunchKernelGGL((dma_read_w<16, 9>), dim3(wgs), dim3(1024), 16 * 9 * 1024, 0, bufs[i % R], per, sink); };
        auto w8u4 = [&](int i) { hipLaunchKernelGGL((dma_read_w<8, 4>), dim3(wgs), dim3(512), 8 * 4 * 1024, 0, bufs[i % R], per, sink); };
        auto w8u8 = [&](int i) { hipLaunchKernelGGL((dma_read_w<8, 8>), dim3(wgs), dim3(512), 8 * 8 * 1024, 0, bufs[i % R], per, sink); };
        auto w8u17 = [&](int i) { hipLaunchKernelGGL((dma_read_w<8, 17>), dim3(wgs), dim3(512), 8 * 17 * 1024, 0, bufs[i % R], per, sink); };
        CHECK(hipFuncSetAttribute((const void*)dma_read_w<16, 9>, hipFuncAttributeMaxDynamicSharedMemorySize, 16 * 9 * 1024));
        CHECK(hipFuncSetAttribute((const void*)dma_read_w<8, 17>, hipFuncAttributeMaxDynamicSharedMemorySize, 8 * 17 * 1024));
        const float a1 = time_it(w16u2, L), a2 = time_it(w16u4, L), a3 = time_it(w16u9, L);
        const float b1 = time_it(w8u4, L), b2 = time_it(w8u8, L), b3 = time_it(w8u17, L);
        printf("wgs 256 x 16 waves per_wg %zu B | U2 %6.2f us %6.0f GB/s | U4 %6.2f us %6.0f GB/s | U9 (all) %6.2f us %6.0f GB/s\n",
               per, a1, bytes / a1 * 1e-3, a2, bytes / a2 * 1e-3, a3, bytes / a3 * 1e-3);
        printf("wgs 256 x  8 waves per_wg %zu B | U4 %6.2f us %6.0f GB/s | U8 %6.2f us %6.0f GB/s | U17 (all) %6.2f us %6.0f GB/s\n",
               per, b1, bytes / b1 * 1e-3, b2, bytes / b2 * 1e-3, b3, bytes / b3 * 1e-3);
    }
    // empty-kernel launch floor
    auto e = [&](int i) { hipLaunchKernelGGL(vgpr_read<1>, dim3(1024), dim3(256), 0, 0, (const u32x4*)bufs[i % R], 0, sink); };
    printf("empty 1024-WG launch: %.2f us\n", time_it(e, L));
    return 0;
}
