// Test-only probes of gfx950 primitives used by the attention kernels
// (built into tests/_build/libprims.so by `make tests-hip`; never linked into libfattn).
#include <hip/hip_runtime.h>
#include "../../ggml-cuda-experiments_amd/csrc/fattn_common.h"

using namespace fattn;

__global__ void permlane_probe(const float* in, float* out) {
    const int l = threadIdx.x;
    const float x = in[l];
    float a16 = x, b16 = x, a32 = x, b32 = x;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a16), "+v"(b16));
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a32), "+v"(b32));
    out[0 * 64 + l] = a16;
    out[1 * 64 + l] = b16;
    out[2 * 64 + l] = a32;
    out[3 * 64 + l] = b32;
    out[4 * 64 + l] = grp4_max(x);
    out[5 * 64 + l] = grp4_sum(x);
}

extern "C" int prims_permlane(const float* in, float* out) {
    hipLaunchKernelGGL(permlane_probe, dim3(1), dim3(64), 0, 0, in, out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

// LDS-DMA with a partial EXEC mask: lanes < nact load 16 B each into a
// lane-linear LDS image that is pre-filled with 0xAB; the whole image is
// dumped so the test can see which bytes the instruction wrote.
typedef __attribute__((address_space(3))) void lds_void_t;
__global__ void dma_partial_probe(const uint8_t* src, uint8_t* out, int nact, int use_buffer) {
    __shared__ __attribute__((aligned(16))) uint8_t img[2048];
    const int l = threadIdx.x;
    for (int i = l; i < 2048; i += 64) img[i] = 0xAB;
    __syncthreads();
    if (use_buffer == 2) {
        // every lane issues; lanes >= nact point past the descriptor's range
        auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 4096, 0x00020000);
        const unsigned off = l < nact ? l * 16 : 0xFFFFFF00u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(img + 256), 16, off, 0, 0, 0);
    } else if (l < nact) {
        if (use_buffer) {
            auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 4096, 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)(img + 256), 16, l * 16, 0, 0, 0);
        } else {
            __builtin_amdgcn_global_load_lds((const void*)(src + l * 16), (void*)(img + 256), 16, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = l; i < 2048; i += 64) out[i] = img[i];
}

extern "C" int prims_dma_partial(const uint8_t* src, uint8_t* out, int nact, int use_buffer) {
    hipLaunchKernelGGL(dma_partial_probe, dim3(1), dim3(64), 0, 0, src, out, nact, use_buffer);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
