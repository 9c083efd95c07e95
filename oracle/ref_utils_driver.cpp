// ref_utils_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Builds the reference's own CPU oracle, /root/reference/src/utils.h, from the
// file where it lies (it is never copied into this repo), into
// oracle/_ref/libref_utils.so, and exposes its functions through a C ABI so
// that tests can pin the restatement in oracle/fattn_oracle.c bit-for-bit and
// bench.py can time the reference's own loops as the CPU baseline.
//
// utils.h uses `half`, `__half2float`, `__float2half` from cuda_fp16.h; here
// they come from ROCm's hip/hip_fp16.h (host-side round-to-nearest-even
// conversions, part of this image -- not a stand-in written for this build).
// The include path for utils.h is passed on the command line by
// oracle/Makefile (-include /root/reference/src/utils.h).
#include <hip/hip_fp16.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include REF_UTILS_H

extern "C" {

void ref_mulmat_f32(const float* A, const float* B, const float* mask, float* C, uint32_t M, uint32_t N,
                    uint32_t K, float scale, int B_transposed) {
    mulmat_cpu(A, B, mask, C, M, N, K, scale, B_transposed != 0);
}

void ref_mulmat_f16(const float* A, const uint16_t* B, const uint16_t* mask, float* C, uint32_t M, uint32_t N,
                    uint32_t K, float scale, int B_transposed) {
    mulmat_cpu(A, reinterpret_cast<const half*>(B), reinterpret_cast<const half*>(mask), C, M, N, K, scale,
               B_transposed != 0);
}

void ref_softmax(float* scores, int kv_size, int batch_size) { softmax(scores, kv_size, batch_size, 0); }

void ref_random(float* arr, uint32_t count) { random(arr, count); }

void ref_srand(unsigned seed) { srand(seed); }

void ref_fill_buffer(float* arr, float val, uint32_t count) { fill_buffer(arr, val, count); }

uint16_t ref_float2half(float x) {
    half h = __float2half(x);
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
}

float ref_half2float(uint16_t u) {
    half h;
    std::memcpy(&h, &u, 2);
    return __half2float(h);
}

// src/kernel_test.h:50-62, calling the reference's functions in the same
// order. n_threads > 1 splits the heads over std::threads (heads are
// independent: each call touches only its own scores/out slices), which is the
// "heads-parallel" CPU baseline of BASELINE.md.
void ref_kernel_test_cpu(const float* query, const float* key, const float* value, const float* mask, float* out,
                         int kv_size, int head_dim, int num_heads, int num_kv_heads, float scale, int n_threads) {
    const int r_kv_heads = num_heads / num_kv_heads;
    std::vector<float> scores((size_t)kv_size * num_heads);
    auto run = [&](int h0, int h1) {
        for (int h = h0; h < h1; h++) {
            mulmat_cpu(query + (size_t)h * head_dim, key + (size_t)(h / r_kv_heads) * head_dim * kv_size, mask,
                       scores.data() + (size_t)h * kv_size, 1, kv_size, head_dim, scale, true);
            softmax(scores.data() + (size_t)h * kv_size, kv_size, 1, h);
        }
        for (int h = h0; h < h1; h++) {
            mulmat_cpu(scores.data() + (size_t)h * kv_size, value + (size_t)(h / r_kv_heads) * head_dim * kv_size,
                       (const float*)nullptr, out + (size_t)h * head_dim, 1, head_dim, kv_size, 1.0f);
        }
    };
    if (n_threads <= 1) {
        run(0, num_heads);
        return;
    }
    std::vector<std::thread> th;
    const int per = (num_heads + n_threads - 1) / n_threads;
    for (int t = 0; t < n_threads; t++) {
        const int h0 = t * per, h1 = std::min(num_heads, h0 + per);
        if (h0 < h1) th.emplace_back(run, h0, h1);
    }
    for (auto& t : th) t.join();
}

}  // extern "C"
