// atomic_probe.hip -- calibration probe (not part of libfattn): latency of one
// agent-scope atomic add per workgroup when `per` workgroups share a counter
// (each counter on its own 256-B line), all workgroups arriving together.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void probe(unsigned* cnt, unsigned long long* lat, int per, int mode) {
    __shared__ unsigned long long t0;
    if (threadIdx.x == 0) {
        unsigned* c = cnt + (blockIdx.x / per) * 64;
        const unsigned long long a = __builtin_amdgcn_s_memrealtime();
        unsigned v;
        if (mode == 0) {
            v = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            unsigned long long* c64 = (unsigned long long*)c;
            v = (unsigned)__hip_atomic_fetch_add(c64, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const unsigned long long b = __builtin_amdgcn_s_memrealtime();
        lat[blockIdx.x] = (b - a) | ((unsigned long long)v << 40);
        t0 = a;
    }
}

int main() {
    const int G = 1024;
    unsigned* cnt;
    unsigned long long* lat;
    CHECK(hipMalloc(&cnt, G * 256));
    CHECK(hipMalloc(&lat, G * 8));
    unsigned long long h[G];
    for (int mode = 0; mode < 2; mode++) {
        for (int per : {1, 8, 32, 128, 1024}) {
            double mx = 0, sum = 0;
            for (int rep = 0; rep < 3; rep++) {
                CHECK(hipMemset(cnt, 0, G * 256));
                hipLaunchKernelGGL(probe, dim3(G), dim3(256), 0, 0, cnt, lat, per, mode);
                CHECK(hipDeviceSynchronize());
                CHECK(hipMemcpy(h, lat, G * 8, hipMemcpyDeviceToHost));
                for (int i = 0; i < G; i++) {
                    const double l = (double)(h[i] & ((1ull << 40) - 1)) * 0.01;
                    if (l > mx) mx = l;
                    sum += l;
                }
            }
            printf("%s atomics, %4d workgroups per counter: max %.2f us  mean %.2f us\n", mode ? "64-bit" : "32-bit",
                   per, mx, sum / (3 * G));
        }
    }
    return 0;
}
