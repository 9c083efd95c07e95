// kernel_test.cpp -- MI355X counterpart of the reference's launch/verify harness
// (src/kernel_test.h:1-249, entered from main() in src/flash-matrix.cu:341-346).
//
// Same flags and the same flow: synthetic inputs from rand() in the order
// Q, K, V, mask (kernel_test.h:45-48; srand never called -> glibc seed 1),
// a CPU reference with the reference's arithmetic (kernel_test.h:50-62: operands
// rounded through fp16, fp32 accumulation, single-pass online softmax), the GPU
// path through the C ABI (include/fattn.h), a timed launch and the max-diff
// report (kernel_test.h:201-234).  Differences from the reference harness, all
// additive: a pass/fail threshold and exit code (the reference prints a diff
// with no threshold), warmup + repeated timing (median), and K/V types.
//
//   --no-kv-parallel     the flash_attn_ext branch (kernel_test.h:180-199): the call goes
//                        through fattn_ext_f16_launch with kernel_test.h:191-198's argument
//                        list -- 32-row padded mask (row 0 = the mask, kernel_test.h:74-85),
//                        ne31 = 32, nb31 = kv_size*2, nb01 = nb02 = head_dim*4, V not
//                        transposed.  The default branch is flash_attn_row + fa_reduce
//                        (kernel_test.h:161-162): fattn_row with V transposed.
//   --n-warps N          accepted for compatibility (kernel_test.h:9-13); the gfx950
//                        kernels pick their own wave counts
//   --kv-size N          KV length, min 256 on the GPU path (kernel_test.h:14-18)
//   --kv-type T          f16 (default, as the reference) | q8_0 | q4_0
//   --cpu-only           the CPU reference alone (BASELINE config 1: no GPU is touched,
//                        any kv_size); with --dump FILE its f32 output is written raw
//   --head-dim D --heads H --kv-heads Hkv --iters I --tol T
//   --n-q N              query rows (the reference's batch / ne01, flash-llama.h:7-32;
//                        src/flash-matrix.cu:76): Q [n_q][H][D], mask [rows >= n_q, padded
//                        to 32][N'], dst [n_q][H][D]; n_q > 1 takes the ext branch
//   --mask random|zero|none   mask values (default random, kernel_test.h:48)
//   --check-rows R       verify R query rows at the start, middle and end of the
//                        sequence (all rows when n_q <= 3R; the CPU reference is slow)
//   --config N           BASELINE.json's configs: 1 (CPU only: 1 head, D 64, N 128),
//                        2 (f16, 32 heads, D 128, N 2048, flash_attn_row), 3 (Q8_0,
//                        32 heads, N 4096), 4 (Q4_0, 32 q / 8 kv heads, N 8192), 5 (Q8_0,
//                        n_q 64, N 4096); "prefill" (Q8_0, n_q = N = 4096, 32 heads,
//                        zero mask: SURVEY 8(d)'s MFMA shape); later flags override
//   --ngpu G             head-shard over G GPUs of this host (kv heads Hkv/G and their q
//                        heads per device, fattn_ext on each, one RCCL all-gather of the
//                        outputs, permuted into the ggml dst layout): BASELINE config 5's
//                        multi-GPU form, timed as kernel + gather
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fattn.h"

#define HIP_CHECK(x)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "HIP error %s at %s:%d (%s)\n", hipGetErrorString(e_), __FILE__, __LINE__, #x); \
            exit(2);                                                                              \
        }                                                                                         \
    } while (0)

namespace {

// ---- host fp16 (round to nearest even), the conversions utils.h relies on
uint16_t f2h(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u, ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);
    if (ax < 0x38800000u) {
        if (ax <= 0x33000000u) return (uint16_t)sign;
        const uint32_t e = ax >> 23, m = (ax & 0x7fffffu) | 0x800000u, sh = 126u - e;
        uint32_t q = m >> sh;
        const uint32_t rem = m & ((1u << sh) - 1u), half = 1u << (sh - 1u);
        if (rem > half || (rem == half && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t h = ((((ax >> 23) - 112u) << 10) | ((ax & 0x7fffffu) >> 13));
    const uint32_t rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}
float h2f(uint16_t h) {
    const uint32_t sign = ((uint32_t)h & 0x8000u) << 16, e = (h >> 10) & 0x1fu;
    uint32_t m = h & 0x3ffu, x;
    if (e == 0) {
        if (m == 0) {
            x = sign;
        } else {
            int ee = -1;
            do {
                ee++;
                m <<= 1;
            } while (!(m & 0x400u));
            x = sign | ((uint32_t)(112 - ee) << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (e == 31) {
        x = sign | 0x7f800000u | (m << 13);
    } else {
        x = sign | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &x, 4);
    return f;
}
float rh(float x) { return h2f(f2h(x)); }

// kernel_test.h:45-48 / utils.h:57-61
void random_fill(std::vector<float>& a) {
    for (auto& x : a) x = 1.0f - ((float)rand() * 1.0f / (float)RAND_MAX) * 2.0f;
}

// kernel_test.h:50-62 with utils.h:5-49 arithmetic, per (query row, head):
// q [NQ][H][D], k / v [Hkv][N][D], mask [NQ][N], out [NQ][H][D]; only the rows
// listed (all of them for the reference's n_q = 1), heads over threads (the
// per-head arithmetic and its order are the reference's, so the bits are too)
void cpu_reference(const std::vector<float>& q, const std::vector<float>& k, const std::vector<float>& v,
                   const std::vector<float>& mask, std::vector<float>& out, int N, int D, int H, int Hkv, float scale,
                   const std::vector<int>& rows, int threads = 1) {
    const int r = H / Hkv;
    std::vector<float> qh(q.size()), kh(k.size()), vh(v.size());
    for (size_t i = 0; i < q.size(); i++) qh[i] = rh(q[i]);
    for (size_t i = 0; i < k.size(); i++) kh[i] = rh(k[i]);
    for (size_t i = 0; i < v.size(); i++) vh[i] = rh(v[i]);
    auto head = [&](int h) {
        std::vector<float> s(N);
        const float* kk = kh.data() + (size_t)(h / r) * D * N;
        const float* vv = vh.data() + (size_t)(h / r) * D * N;
        for (int row : rows) {
            const float* qq = qh.data() + ((size_t)row * H + h) * D;
            const float* mrow = mask.data() + (size_t)row * N;
            for (int c = 0; c < N; c++) {
                float acc = 0.0f;
                for (int i = 0; i < D; i++) {
                    const float p = qq[i] * kk[(size_t)c * D + i];
                    acc = acc + p;
                }
                s[c] = acc * scale + mrow[c];
            }
            float M = -INFINITY, S = 0.0f;
            for (int i = 0; i < N; i++) {
                if (s[i] > M) {
                    S = 1.0f + S * expf(M - s[i]);
                    M = s[i];
                } else {
                    S += expf(s[i] - M);
                }
            }
            for (int i = 0; i < N; i++) s[i] = expf(s[i] - M) / S;
            float* o = out.data() + ((size_t)row * H + h) * D;
            for (int c = 0; c < D; c++) {
                float acc = 0.0f;
                for (int i = 0; i < N; i++) {
                    const float p = rh(s[i]) * vv[(size_t)i * D + c];
                    acc = acc + p;
                }
                o[c] = acc;
            }
        }
    };
    threads = std::max(1, std::min(threads, H));
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++)
        pool.emplace_back([&, t] {
            for (int h = t; h < H; h += threads) head(h);
        });
    for (auto& th : pool) th.join();
}

void print_array(const char* name, const float* a, int count) {  // utils.h:63-71
    printf("---------------- %s ------------------\n", name);
    for (int i = 0; i < count; i++) printf("%0.4ff, ", a[i]);
    printf("\n");
}

int parse_type(const std::string& s) {
    if (s == "f16") return FATTN_TYPE_F16;
    if (s == "q8_0") return FATTN_TYPE_Q8_0;
    if (s == "q4_0") return FATTN_TYPE_Q4_0;
    fprintf(stderr, "unknown --kv-type %s\n", s.c_str());
    exit(2);
}

}  // namespace

#define RCCL_CHECK(x)                                                                             \
    do {                                                                                          \
        ncclResult_t r_ = (x);                                                                    \
        if (r_ != ncclSuccess) {                                                                  \
            fprintf(stderr, "RCCL error %s at %s:%d (%s)\n", ncclGetErrorString(r_), __FILE__, __LINE__, #x); \
            exit(2);                                                                              \
        }                                                                                         \
    } while (0)

int main(int argc, const char* argv[]) {
    int kv_size = 512, num_warps = 8, head_dim = 128, num_heads = 32, num_kv_heads = 8, iters = 20;
    int kv_type = FATTN_TYPE_F16, n_q = 1, check_rows = 64, ngpu = 1;
    bool parallel_kv = true, cpu_only = false;
    std::string mask_kind = "random";
    const char* dump = nullptr;
    float tol = 1e-3f;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (++i >= argc) {
                fprintf(stderr, "missing value for %s\n", a.c_str());
                exit(2);
            }
            return argv[i];
        };
        if (a == "--no-kv-parallel") parallel_kv = false;
        else if (a == "--n-warps") num_warps = atoi(next());
        else if (a == "--kv-size") kv_size = atoi(next());
        else if (a == "--cpu-only") cpu_only = true;
        else if (a == "--dump") dump = next();
        else if (a == "--kv-type") kv_type = parse_type(next());
        else if (a == "--head-dim") head_dim = atoi(next());
        else if (a == "--heads") num_heads = atoi(next());
        else if (a == "--kv-heads") num_kv_heads = atoi(next());
        else if (a == "--iters") iters = std::max(1, atoi(next()));
        else if (a == "--tol") tol = (float)atof(next());
        else if (a == "--n-q") n_q = atoi(next());
        else if (a == "--check-rows") check_rows = std::max(1, atoi(next()));
        else if (a == "--ngpu") ngpu = atoi(next());
        else if (a == "--mask") {
            mask_kind = next();
            if (mask_kind != "random" && mask_kind != "zero" && mask_kind != "none") {
                fprintf(stderr, "--mask random|zero|none\n");
                return 2;
            }
        } else if (a == "--config") {
            // BASELINE.json configs[N - 1] (and SURVEY 8(d)'s prefill shape)
            const std::string c = next();
            if (c == "1") {
                cpu_only = true, num_heads = num_kv_heads = 1, head_dim = 64, kv_size = 128;
            } else if (c == "2") {
                kv_type = FATTN_TYPE_F16, num_heads = num_kv_heads = 32, head_dim = 128, kv_size = 2048;
            } else if (c == "3") {
                parallel_kv = false, kv_type = FATTN_TYPE_Q8_0, num_heads = num_kv_heads = 32, kv_size = 4096;
            } else if (c == "4") {
                parallel_kv = false, kv_type = FATTN_TYPE_Q4_0, num_heads = 32, num_kv_heads = 8, kv_size = 8192;
            } else if (c == "5") {
                parallel_kv = false, kv_type = FATTN_TYPE_Q8_0, num_heads = num_kv_heads = 32, kv_size = 4096,
                n_q = 64;
            } else if (c == "prefill") {
                parallel_kv = false, kv_type = FATTN_TYPE_Q8_0, num_heads = num_kv_heads = 32, kv_size = 4096,
                n_q = 4096, mask_kind = "zero";
            } else {
                fprintf(stderr, "--config 1|2|3|4|5|prefill\n");
                return 2;
            }
        } else {
            fprintf(stderr, "unknown flag %s\n", a.c_str());
            return 2;
        }
    }
    if (num_warps != 8 && num_warps != 4 && num_warps != 2 && num_warps != 1)
        printf("invalid num_warps, should be 2, 4, 8\n");  // kernel_test.h:176-178 (informational)
    if (!cpu_only) kv_size = std::max(256, kv_size);      // kernel_test.h:14-18
    if (n_q > 1 || ngpu > 1) parallel_kv = false;        // flash_attn_row is one query row on one device

    const int D = head_dim, H = num_heads, Hkv = num_kv_heads, N = kv_size, NQ = n_q;
    const float scale = 1.0f / sqrtf((float)D);
    if (H <= 0 || Hkv <= 0 || N <= 0 || D <= 0 || NQ <= 0 || H % Hkv) {
        fprintf(stderr, "heads must be a positive multiple of kv-heads\n");
        return 2;
    }
    if (ngpu < 1 || Hkv % ngpu) {
        fprintf(stderr, "--ngpu must divide the kv heads (%d)\n", Hkv);
        return 2;
    }
    // the rand() stream in kernel_test.h:45-48's order: Q, K, V, then the mask
    // (n_q rows; row 0 is the reference's one mask row)
    std::vector<float> query((size_t)D * H * NQ), key((size_t)D * N * Hkv), value((size_t)D * N * Hkv),
        mask((size_t)N * NQ);
    random_fill(query);
    random_fill(key);
    random_fill(value);
    random_fill(mask);
    if (mask_kind != "random") std::fill(mask.begin(), mask.end(), 0.0f);  // "none": zeros on the CPU, no mask on the GPU
    // the query rows the CPU reference checks: all of them, or check_rows at
    // the start, middle and end of the sequence
    std::vector<int> rows;
    if (NQ <= 3 * check_rows) {
        for (int i = 0; i < NQ; i++) rows.push_back(i);
    } else {
        for (int b : {0, NQ / 2 - check_rows / 2, NQ - check_rows})
            for (int i = 0; i < check_rows; i++) rows.push_back(b + i);
    }
    const int threads = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));

    if (cpu_only) {  // BASELINE config 1: kernel_test.h:50-66 on the host, nothing else
        std::vector<float> out((size_t)D * H * NQ);
        cpu_reference(query, key, value, mask, out, N, D, H, Hkv, scale, rows, threads);
        print_array("Reference", out.data(), std::min(16, D * H));
        if (dump) {
            FILE* f = fopen(dump, "wb");
            if (!f || fwrite(out.data(), sizeof(float), out.size(), f) != out.size()) {
                fprintf(stderr, "cannot write %s\n", dump);
                return 2;
            }
            fclose(f);
        }
        return 0;
    }

    int ndev = 0;
    HIP_CHECK(hipGetDeviceCount(&ndev));
    if (ngpu > ndev) {
        fprintf(stderr, "--ngpu %d but %d devices\n", ngpu, ndev);
        return 2;
    }
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, 0));
    printf("GPU: %s (%s), CUs: %d, LDS/block max: %zu KB, HBM: %zu MB%s\n", prop.name, prop.gcnArchName,
           prop.multiProcessorCount, prop.sharedMemPerBlock / 1024, prop.totalGlobalMem >> 20,
           ngpu > 1 ? " (x --ngpu)" : "");

    // K/V values as the kernels see them: f16 rounding on the host, or Q8_0 /
    // Q4_0 quantised on device 0 (fattn_quantize) and dequantised back for the
    // CPU reference (fattn_dequantize)
    const size_t rb = fattn_row_size(kv_type, D);
    std::vector<float> kref = key, vref = value;
    std::vector<uint8_t> kbytes(rb * N * Hkv), vbytes(rb * N * Hkv);
    const bool vtrans = parallel_kv && kv_type == FATTN_TYPE_F16;
    {
        HIP_CHECK(hipSetDevice(0));
        hipStream_t st0;
        HIP_CHECK(hipStreamCreate(&st0));
        if (kv_type == FATTN_TYPE_F16) {
            uint16_t* k16 = (uint16_t*)kbytes.data();
            uint16_t* v16 = (uint16_t*)vbytes.data();
            for (size_t i = 0; i < key.size(); i++) k16[i] = f2h(key[i]);
            for (int h = 0; h < Hkv; h++)
                for (int n = 0; n < N; n++)
                    for (int d = 0; d < D; d++) {
                        const size_t src = ((size_t)h * N + n) * D + d;
                        const size_t dst = vtrans ? ((size_t)h * D + d) * N + n : src;
                        v16[dst] = f2h(value[src]);
                    }
        } else {
            float *d_kf, *d_vf;
            void *d_kq, *d_vq;
            HIP_CHECK(hipMalloc(&d_kf, sizeof(float) * key.size()));
            HIP_CHECK(hipMalloc(&d_vf, sizeof(float) * value.size()));
            HIP_CHECK(hipMalloc(&d_kq, kbytes.size()));
            HIP_CHECK(hipMalloc(&d_vq, vbytes.size()));
            HIP_CHECK(hipMemcpyAsync(d_kf, key.data(), 4 * key.size(), hipMemcpyHostToDevice, st0));
            HIP_CHECK(hipMemcpyAsync(d_vf, value.data(), 4 * value.size(), hipMemcpyHostToDevice, st0));
            int rc = fattn_quantize(kv_type, d_kf, d_kq, D, (int64_t)N * Hkv, st0);
            rc = rc ? rc : fattn_quantize(kv_type, d_vf, d_vq, D, (int64_t)N * Hkv, st0);
            rc = rc ? rc : fattn_dequantize(kv_type, d_kq, d_kf, D, (int64_t)N * Hkv, st0);
            rc = rc ? rc : fattn_dequantize(kv_type, d_vq, d_vf, D, (int64_t)N * Hkv, st0);
            if (rc) {
                fprintf(stderr, "quantize failed: %s\n", fattn_strerror(rc));
                return 2;
            }
            HIP_CHECK(hipMemcpyAsync(kref.data(), d_kf, 4 * key.size(), hipMemcpyDeviceToHost, st0));
            HIP_CHECK(hipMemcpyAsync(vref.data(), d_vf, 4 * value.size(), hipMemcpyDeviceToHost, st0));
            HIP_CHECK(hipMemcpyAsync(kbytes.data(), d_kq, kbytes.size(), hipMemcpyDeviceToHost, st0));
            HIP_CHECK(hipMemcpyAsync(vbytes.data(), d_vq, vbytes.size(), hipMemcpyDeviceToHost, st0));
            HIP_CHECK(hipStreamSynchronize(st0));
            HIP_CHECK(hipFree(d_kf));
            HIP_CHECK(hipFree(d_vf));
            HIP_CHECK(hipFree(d_kq));
            HIP_CHECK(hipFree(d_vq));
        }
        HIP_CHECK(hipStreamSynchronize(st0));
        HIP_CHECK(hipStreamDestroy(st0));
    }

    // CPU reference (kernel_test.h:50-66) on the checked rows
    std::vector<float> qkv((size_t)D * H * NQ, 0.0f), qkv_gpu((size_t)D * H * NQ);
    cpu_reference(query, kref, vref, mask, qkv, N, D, H, Hkv, scale, rows, threads);
    print_array("Reference", qkv.data(), 16);

    // ---- per device: its head shard (kv heads [g Hkv/G, (g+1) Hkv/G) and their
    // q heads; G = 1: everything), inputs, workspace, stream
    const int G = ngpu, Hl = H / G, Hkvl = Hkv / G;
    // mask f16: one row for flash_attn_row; rows padded to a multiple of 32
    // (row i = query i's mask, the rest zeros) for flash_attn_ext
    // (kernel_test.h:74-85), each padded to an even length (ggml pads to
    // GGML_KQ_MASK_PAD; the kernels read rows in dword pieces)
    const bool has_mask = mask_kind != "none";
    const int mask_rows = parallel_kv ? 1 : (NQ + 31) / 32 * 32;
    const int Np = parallel_kv ? N : N + (N & 1);
    std::vector<uint16_t> mask16((size_t)Np * mask_rows, f2h(0.0f));
    for (int r = 0; r < NQ && r < mask_rows; r++)
        for (int i = 0; i < N; i++) mask16[(size_t)r * Np + i] = f2h(mask[(size_t)r * N + i]);
    struct Dev {
        hipStream_t st;
        float *q, *out, *gather;
        void *k, *v, *mask, *ws;
        size_t ws_bytes;
        fattn_params p;
    };
    std::vector<Dev> dv(G);
    const int r_kv_heads = H / Hkv;
    for (int g = 0; g < G; g++) {
        Dev& d = dv[g];
        HIP_CHECK(hipSetDevice(g));
        HIP_CHECK(hipStreamCreate(&d.st));
        // this shard's Q [NQ][Hl][D] and K / V rows [Hkvl][N][row]
        std::vector<float> qs((size_t)NQ * Hl * D);
        for (int r = 0; r < NQ; r++)
            std::memcpy(&qs[(size_t)r * Hl * D], &query[((size_t)r * H + g * Hl) * D], sizeof(float) * Hl * D);
        HIP_CHECK(hipMalloc(&d.q, sizeof(float) * qs.size()));
        HIP_CHECK(hipMalloc(&d.out, sizeof(float) * NQ * Hl * D));
        HIP_CHECK(hipMalloc(&d.gather, sizeof(float) * NQ * H * D));
        const size_t kvb = rb * N * Hkvl;
        HIP_CHECK(hipMalloc(&d.k, kvb));
        HIP_CHECK(hipMalloc(&d.v, kvb));
        HIP_CHECK(hipMalloc(&d.mask, 2 * mask16.size()));
        HIP_CHECK(hipMemcpyAsync(d.q, qs.data(), 4 * qs.size(), hipMemcpyHostToDevice, d.st));
        HIP_CHECK(hipMemcpyAsync(d.k, kbytes.data() + kvb * g, kvb, hipMemcpyHostToDevice, d.st));
        HIP_CHECK(hipMemcpyAsync(d.v, vbytes.data() + kvb * g, kvb, hipMemcpyHostToDevice, d.st));
        HIP_CHECK(hipMemcpyAsync(d.mask, mask16.data(), 2 * mask16.size(), hipMemcpyHostToDevice, d.st));
        // the ext plan: the flash_attn_ext argument list of kernel_test.h:191-198
        // (n_q = 1) or its ne01 = n_q form, as a fattn_params view
        std::memset(&d.p, 0, sizeof(d.p));
        const int64_t eb = kv_type == FATTN_TYPE_F16 ? 2 : (int64_t)fattn_row_size(kv_type, 32);
        d.p.q = {d.q, FATTN_TYPE_F32, 0, {D, NQ, Hl, 1}, {4, (int64_t)Hl * D * 4, D * 4, (int64_t)NQ * Hl * D * 4}};
        d.p.k = {d.k, kv_type, 0, {D, N, Hkvl, 1}, {eb, (int64_t)rb, (int64_t)rb * N, (int64_t)rb * N * Hkvl}};
        d.p.v = {d.v, kv_type, 0, {D, N, Hkvl, 1}, {eb, (int64_t)rb, (int64_t)rb * N, (int64_t)rb * N * Hkvl}};
        if (has_mask)
            d.p.mask = {d.mask, FATTN_TYPE_F16, 0, {Np, mask_rows, 1, 1},
                        {2, (int64_t)Np * 2, (int64_t)Np * 2 * mask_rows, (int64_t)Np * 2 * mask_rows}};
        d.p.dst = d.out;
        d.p.scale = scale;
        d.ws_bytes = parallel_kv ? fattn_row_workspace_size(D, N, H) : fattn_workspace_size(&d.p);
        d.ws_bytes = std::max<size_t>(d.ws_bytes, 16);
        HIP_CHECK(hipMalloc(&d.ws, d.ws_bytes));
        if (int zr = fattn_workspace_init(d.ws, d.ws_bytes, d.st)) {
            fprintf(stderr, "fattn_workspace_init failed: %s\n", fattn_strerror(zr));
            return 2;
        }
        d.p.workspace = d.ws;
        d.p.workspace_bytes = d.ws_bytes;
    }
    if (parallel_kv && kv_type != FATTN_TYPE_F16) {
        fprintf(stderr, "the flash_attn_row branch takes f16 K/V (use --no-kv-parallel for %s)\n",
                kv_type == FATTN_TYPE_Q8_0 ? "q8_0" : "q4_0");
        return 2;
    }
    std::vector<ncclComm_t> comms(G);
    if (G > 1) {
        std::vector<int> devs(G);
        for (int g = 0; g < G; g++) devs[g] = g;
        RCCL_CHECK(ncclCommInitAll(comms.data(), G, devs.data()));
    }
    // one step: every device's attention (flash_attn_row with V transposed,
    // kernel_test.h:161-162; the positional flash_attn_ext call of
    // kernel_test.h:191-198 when n_q = 1 on one device; the fattn_params form
    // otherwise), then with G > 1 one all-gather of the shards' outputs
    auto launch = [&]() -> int {
        for (int g = 0; g < G; g++) {
            Dev& d = dv[g];
            HIP_CHECK(hipSetDevice(g));
            int rc;
            if (parallel_kv)
                rc = fattn_row(d.q, d.k, d.v, d.mask, d.ws, d.ws_bytes, d.out, D, N, H, scale, D * N, r_kv_heads, d.st);
            else if (NQ == 1 && G == 1 && has_mask)
                rc = fattn_ext_f16_launch(d.q, d.k, d.v, d.mask, d.out, scale,
                                          D, 1, H, 1,
                                          D, N, Hkv, 1,
                                          mask_rows, Np * 2,
                                          D * 4, D * 4, D * H * 4,
                                          (int)rb, (int)rb * N, (int)rb * N * Hkv,
                                          D, H, 1, 1,
                                          kv_type, kv_type, d.ws, d.ws_bytes, d.st);
            else
                rc = fattn_ext(&d.p, d.st);
            if (rc) return rc;
        }
        if (G > 1) {
            RCCL_CHECK(ncclGroupStart());
            for (int g = 0; g < G; g++)
                RCCL_CHECK(ncclAllGather(dv[g].out, dv[g].gather, (size_t)NQ * Hl * D, ncclFloat, comms[g], dv[g].st));
            RCCL_CHECK(ncclGroupEnd());
        }
        return 0;
    };
    auto sync_all = [&] {
        for (int g = 0; g < G; g++) {
            HIP_CHECK(hipSetDevice(g));
            HIP_CHECK(hipStreamSynchronize(dv[g].st));
        }
    };
    int rc = launch();
    if (rc) {
        fprintf(stderr, "launch failed: %s\n", fattn_strerror(rc));
        return 2;
    }
    sync_all();
    // timing on device 0's stream (G > 1: events around every device's step,
    // device 0's span; the gather makes the devices wait for each other)
    HIP_CHECK(hipSetDevice(0));
    hipEvent_t start, stop;
    HIP_CHECK(hipEventCreate(&start));
    HIP_CHECK(hipEventCreate(&stop));
    std::vector<float> times;
    for (int it = 0; it < iters; it++) {
        HIP_CHECK(hipSetDevice(0));
        HIP_CHECK(hipEventRecord(start, dv[0].st));
        rc = launch();
        HIP_CHECK(hipSetDevice(0));
        HIP_CHECK(hipEventRecord(stop, dv[0].st));
        HIP_CHECK(hipEventSynchronize(stop));
        sync_all();
        if (rc) {
            fprintf(stderr, "launch failed: %s\n", fattn_strerror(rc));
            return 2;
        }
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, start, stop));
        times.push_back(ms);
    }
    std::sort(times.begin(), times.end());
    const float millis = times[times.size() / 2];
    // the output in the ggml dst layout [n_q][H][D]: device 0's gather buffer
    // [G][n_q][Hl][D] permuted (G > 1), or its output
    HIP_CHECK(hipSetDevice(0));
    if (G > 1) {
        std::vector<float> gath((size_t)NQ * H * D);
        HIP_CHECK(hipMemcpy(gath.data(), dv[0].gather, 4 * gath.size(), hipMemcpyDeviceToHost));
        for (int g = 0; g < G; g++)
            for (int r = 0; r < NQ; r++)
                std::memcpy(&qkv_gpu[((size_t)r * H + g * Hl) * D], &gath[(((size_t)g * NQ + r) * Hl) * D],
                            sizeof(float) * Hl * D);
    } else {
        HIP_CHECK(hipMemcpy(qkv_gpu.data(), dv[0].out, 4 * qkv_gpu.size(), hipMemcpyDeviceToHost));
    }
    print_array(parallel_kv ? "Parallel KV HIP" : "No paralell KV HIP", qkv_gpu.data(), 16);

    // kernel_test.h:215-234 (+ a normwise relative error -- the max |diff| over
    // the max |reference| -- and a threshold), over the checked rows
    float max_diff = 0.0f, max_ref = 0.0f;
    int row_idx = 0, head_idx = 0, dim_idx = 0;
    for (int r : rows)
        for (int h = 0; h < H; h++) {
            const size_t o = ((size_t)r * H + h) * D;
            for (int i = 0; i < D; i++) {
                const float dd = fabsf(qkv[o + i] - qkv_gpu[o + i]);
                max_ref = std::max(max_ref, fabsf(qkv[o + i]));
                if (dd > max_diff || std::isnan(dd)) {
                    max_diff = std::isnan(dd) ? INFINITY : dd;
                    row_idx = r, head_idx = h, dim_idx = i;
                }
            }
        }
    const float worst_rel = max_diff / std::max(max_ref, 1e-30f);
    const double bytes = (double)D * H * NQ * 4 * 2 + 2.0 * rb * N * Hkv + (has_mask ? 2.0 * N * NQ : 0.0);
    const double flops = 4.0 * N * D * H * NQ;
    printf("\ncuda time: %.4f ms  (%.1f GB/s, %.3f TFLOP/s; median of %d%s)\n", millis, bytes / millis / 1e6,
           flops / millis / 1e9, iters, G > 1 ? ", kernel + all-gather" : "");
    printf("R (%.4f) CUDA(%.4f) diff: %.4f - row = %d, head = %d, dim = %d\n",
           qkv[((size_t)row_idx * H + head_idx) * D + dim_idx], qkv_gpu[((size_t)row_idx * H + head_idx) * D + dim_idx],
           max_diff, row_idx, head_idx, dim_idx);
    printf("checked %zu of %d query rows x %d heads; n_q %d, %d GPU(s)\n", rows.size(), NQ, H, NQ, G);
    printf("normwise rel err %.3g (tol %.1g): %s\n", worst_rel, tol, worst_rel <= tol ? "PASS" : "FAIL");
    for (int g = 0; g < G; g++) {
        if (G > 1) RCCL_CHECK(ncclCommDestroy(comms[g]));
    }
    return worst_rel <= tol ? 0 : 1;
}
