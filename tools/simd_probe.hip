// simd_probe.hip -- which SIMD does each wave of a 512-thread workgroup run on?
// (diagnostic tool, not part of libfattn)  Reads HW_REG_HW_ID (gfx9: WAVE_ID
// [3:0], SIMD_ID [5:4], CU_ID [11:8]) from lane 0 of every wave.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void probe(unsigned* out) {
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = id;
}

int main() {
    unsigned* d;
    hipMalloc(&d, 64 * 8 * 4);
    hipLaunchKernelGGL(probe, dim3(64), dim3(512), 0, 0, d);
    unsigned h[64 * 8];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int b = 0; b < 4; b++) {
        printf("block %d:", b);
        for (int w = 0; w < 8; w++) printf(" w%d->simd%u(wave%u,cu%u)", w, (h[b * 8 + w] >> 4) & 3, h[b * 8 + w] & 15,
                                           (h[b * 8 + w] >> 8) & 15);
        printf("\n");
    }
    return 0;
}
