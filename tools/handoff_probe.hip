// handoff_probe.hip -- calibration probe (not part of libfattn): how long until
// a value stored by one workgroup is seen by another workgroup that is
// polling it, for different store / poll forms.  Block 0 (producer) and block
// 1 (consumer) are dealt to different XCDs by the round-robin dispatcher; the
// consumer reads the line BEFORE the producer writes (its L2 may then hold a
// stale copy).  s_memrealtime (100 MHz) stamps give the latency.
//
// poll modes: 0 = global_load sc1, 1 = global_load sc0 sc1, 2 = atomic RMW
//             (fetch_add 0, agent scope), 3 = global_load sc1 nt
// store modes: 0 = global_store sc1, 1 = atomic store (agent), 2 = global_store sc0 sc1
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__device__ __forceinline__ unsigned poll_load(unsigned* p, int mode) {
    unsigned v;
    if (mode == 0) {
        asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    } else if (mode == 1) {
        asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    } else if (mode == 2) {
        v = __hip_atomic_fetch_add(p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        asm volatile("global_load_dword %0, %1, off sc1 nt\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    }
    return v;
}

__global__ void probe(unsigned* flag, unsigned long long* t, int poll_mode, int store_mode, int delay_iters) {
    if (threadIdx.x != 0) return;
    if (blockIdx.x == 1) {
        // consumer: warm its caches with the old value, then poll
        unsigned v = poll_load(flag, poll_mode);
        t[2] = v;
        unsigned long long n = 0;
        while (poll_load(flag, poll_mode) != 1u) {
            if (++n > (1ull << 20)) break;
        }
        t[1] = __builtin_amdgcn_s_memrealtime();
        t[3] = n;
    } else if (blockIdx.x == 0) {
        for (int i = 0; i < delay_iters; i++) __builtin_amdgcn_s_sleep(127);
        t[0] = __builtin_amdgcn_s_memrealtime();
        if (store_mode == 0) {
            asm volatile("global_store_dword %0, %1, off sc1" ::"v"(flag), "v"(1u) : "memory");
        } else if (store_mode == 1) {
            __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(flag), "v"(1u) : "memory");
        }
    }
}

int main() {
    unsigned* flag;
    unsigned long long* t;
    CHECK(hipMalloc(&flag, 4096));
    CHECK(hipMalloc(&t, 64));
    const char* pn[] = {"load sc1", "load sc0 sc1", "atomic rmw", "load sc1 nt"};
    const char* sn[] = {"store sc1", "atomic store", "store sc0 sc1"};
    for (int sm = 0; sm < 3; sm++) {
        for (int pm = 0; pm < 4; pm++) {
            double lat[5];
            unsigned long long polls = 0, stale = 0;
            for (int rep = 0; rep < 5; rep++) {
                CHECK(hipMemset(flag, 0, 4096));
                CHECK(hipMemset(t, 0, 64));
                CHECK(hipDeviceSynchronize());
                hipLaunchKernelGGL(probe, dim3(2), dim3(64), 0, 0, flag, t, pm, sm, 200);
                CHECK(hipDeviceSynchronize());
                unsigned long long h[4];
                CHECK(hipMemcpy(h, t, 32, hipMemcpyDeviceToHost));
                lat[rep] = (double)(long long)(h[1] - h[0]) * 0.01;
                polls += h[3];
                stale += h[2];
            }
            printf("%-14s poll %-13s latency us:", sn[sm], pn[pm]);
            for (double l : lat) printf(" %7.2f", l);
            printf("   polls/rep %llu  warm-read %llu\n", polls / 5, stale);
        }
    }
    return 0;
}
