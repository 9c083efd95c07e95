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
