/*
 * fattn_oracle.c -- CPU restatement of the reference attention oracle.
 * TEST INFRASTRUCTURE ONLY (see fattn_oracle.h).  Compiled with
 * -ffp-contract=off so that `acc += a*b` is a rounded multiply followed by a
 * rounded add, exactly as src/utils.h:10-11 is evaluated without FMA.
 */
#include "fattn_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ fp16 */

uint16_t orc_f32_to_f16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) { /* inf / nan */
        return (uint16_t)(sign | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u));
    }
    if (ax >= 0x477ff000u) { /* >= 65520 rounds to inf */
        return (uint16_t)(sign | 0x7c00u);
    }
    if (ax < 0x38800000u) { /* below 2^-14: fp16 subnormal or zero */
        if (ax <= 0x33000000u) return (uint16_t)sign; /* <= 2^-25 rounds to 0 (tie to even) */
        const uint32_t e = ax >> 23;
        const uint32_t m = (ax & 0x7fffffu) | 0x800000u;
        const uint32_t shift = 126u - e; /* 14..24 */
        uint32_t q = m >> shift;
        const uint32_t rem = m & ((1u << shift) - 1u);
        const uint32_t half = 1u << (shift - 1u);
        if (rem > half || (rem == half && (q & 1u))) q++;
        return (uint16_t)(sign | q);
    }
    uint32_t h = ((((ax >> 23) - 112u) << 10) | ((ax & 0x7fffffu) >> 13));
    const uint32_t rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}

float orc_f16_to_f32(uint16_t hv) {
    const uint32_t sign = ((uint32_t)hv & 0x8000u) << 16;
    const uint32_t e = (hv >> 10) & 0x1fu;
    uint32_t m = hv & 0x3ffu;
    uint32_t x;
    if (e == 0) {
        if (m == 0) {
            x = sign;
        } else { /* subnormal: normalise */
            int ee = -1;
            do {
                ee++;
                m <<= 1;
            } while ((m & 0x400u) == 0);
            x = sign | ((uint32_t)(127 - 15 - ee) << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (e == 31) {
        x = sign | 0x7f800000u | (m << 13);
    } else {
        x = sign | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

float orc_round_f16(float x) { return orc_f16_to_f32(orc_f32_to_f16(x)); }

void orc_f32_to_f16_n(const float* x, uint16_t* y, int64_t n) {
    for (int64_t i = 0; i < n; i++) y[i] = orc_f32_to_f16(x[i]);
}
void orc_f16_to_f32_n(const uint16_t* x, float* y, int64_t n) {
    for (int64_t i = 0; i < n; i++) y[i] = orc_f16_to_f32(x[i]);
}

/* ------------------------------------------------------- src/utils.h:5-61 */

/* src/utils.h:5-16.  Loop order c, r, k as in the reference; both operands
 * rounded through fp16; fp32 accumulate in k order; mask added unrounded. */
void orc_mulmat_f32(const float* A, const float* B, const float* mask, float* C,
                    uint32_t M, uint32_t N, uint32_t K, float scale, int B_transposed) {
    for (uint32_t c = 0; c < N; c++) {
        for (uint32_t r = 0; r < M; r++) {
            float acc = 0.0f;
            for (uint32_t k = 0; k < K; k++) {
                const float a = orc_round_f16(A[(size_t)r * K + k]);
                const float b = orc_round_f16(B[B_transposed ? ((size_t)c * K + k) : ((size_t)k * N + c)]);
                const float p = a * b;
                acc = acc + p;
            }
            C[(size_t)r * N + c] = acc * scale + (mask != NULL ? mask[c] : 0.0f);
        }
    }
}

/* src/utils.h:18-28.  A unrounded, B f16, mask f16 indexed [r*N + c]. */
void orc_mulmat_f16(const float* A, const uint16_t* B, const uint16_t* mask, float* C,
                    uint32_t M, uint32_t N, uint32_t K, float scale, int B_transposed) {
    for (uint32_t c = 0; c < N; c++) {
        for (uint32_t r = 0; r < M; r++) {
            float acc = 0.0f;
            for (uint32_t k = 0; k < K; k++) {
                const float b = orc_f16_to_f32(B[B_transposed ? ((size_t)c * K + k) : ((size_t)k * N + c)]);
                const float p = A[(size_t)r * K + k] * b;
                acc = acc + p;
            }
            C[(size_t)r * N + c] = acc * scale + (mask != NULL ? orc_f16_to_f32(mask[(size_t)r * N + c]) : 0.0f);
        }
    }
}

/* src/utils.h:30-49.  NOTE (faithful quirk): a row whose FIRST score is -inf
 * makes S NaN (expf(-inf - -inf)), exactly like the reference. */
void orc_softmax(float* scores, int kv_size, int batch_size) {
    for (int b = 0; b < batch_size; b++) {
        float Mx = -INFINITY;
        float S = 0.0f;
        for (int i = 0; i < kv_size; i++) {
            const float s = scores[(size_t)b * kv_size + i];
            if (s > Mx) {
                S = 1.0f + S * expf(Mx - s);
                Mx = s;
            } else {
                S += expf(s - Mx);
            }
        }
        for (int i = 0; i < kv_size; i++) {
            scores[(size_t)b * kv_size + i] = expf(scores[(size_t)b * kv_size + i] - Mx) / S;
        }
    }
}

/* src/utils.h:51-55: ignores val, always 0 */
void orc_fill_buffer(float* arr, float val, uint32_t count) {
    (void)val;
    for (uint32_t i = 0; i < count; ++i) arr[i] = 0.0f;
}

/* src/utils.h:57-61 */
void orc_random(float* arr, uint32_t count) {
    for (uint32_t i = 0; i < count; ++i) {
        arr[i] = 1.0f - ((float)rand() * 1.0f / (float)RAND_MAX) * 2.0f;
    }
}

void orc_srand(unsigned seed) { srand(seed); }

/* src/kernel_test.h:50-62 */
void orc_kernel_test_cpu(const float* query, const float* key, const float* value,
                         const float* mask, float* out, int kv_size, int head_dim,
                         int num_heads, int num_kv_heads, float scale) {
    const int r_kv_heads = num_heads / num_kv_heads;
    float* scores = (float*)malloc(sizeof(float) * (size_t)kv_size * num_heads);
    for (int h = 0; h < num_heads; h++) {
        orc_mulmat_f32(query + (size_t)h * head_dim, key + (size_t)(h / r_kv_heads) * head_dim * kv_size, mask,
                       scores + (size_t)h * kv_size, 1, kv_size, head_dim, scale, 1);
        orc_softmax(scores + (size_t)h * kv_size, kv_size, 1);
    }
    for (int h = 0; h < num_heads; h++) {
        orc_mulmat_f32(scores + (size_t)h * kv_size, value + (size_t)(h / r_kv_heads) * head_dim * kv_size, NULL,
                       out + (size_t)h * head_dim, 1, head_dim, kv_size, 1.0f, 0);
    }
    free(scores);
}

/* ------------------------------------------------- ggml Q8_0 / Q4_0 (upstream) */

#define QK 32

/* ggml quantize_row_q8_0_ref: amax -> d = amax/127, id = d ? 1/d : 0,
 * qs = roundf(x*id), stored d = fp16(d). */
void orc_quantize_row_q8_0(const float* x, void* vy, int64_t k) {
    uint8_t* y = (uint8_t*)vy;
    const int64_t nb = k / QK;
    for (int64_t i = 0; i < nb; i++) {
        float amax = 0.0f;
        for (int j = 0; j < QK; j++) {
            const float v = x[i * QK + j];
            const float av = fabsf(v);
            amax = amax > av ? amax : av;
        }
        const float d = amax / ((1 << 7) - 1);
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        const uint16_t dh = orc_f32_to_f16(d);
        uint8_t* blk = y + i * 34;
        memcpy(blk, &dh, 2);
        for (int j = 0; j < QK; ++j) {
            const float x0 = x[i * QK + j] * id;
            const int8_t q = (int8_t)roundf(x0);
            blk[2 + j] = (uint8_t)q;
        }
    }
}

/* ggml dequantize_row_q8_0: y = qs * fp32(d) (exact in f32) */
void orc_dequantize_row_q8_0(const void* vx, float* y, int64_t k) {
    const uint8_t* x = (const uint8_t*)vx;
    const int64_t nb = k / QK;
    for (int64_t i = 0; i < nb; i++) {
        const uint8_t* blk = x + i * 34;
        uint16_t dh;
        memcpy(&dh, blk, 2);
        const float d = orc_f16_to_f32(dh);
        for (int j = 0; j < QK; ++j) {
            y[i * QK + j] = (float)(int8_t)blk[2 + j] * d;
        }
    }
}

/* ggml quantize_row_q4_0_ref: max = signed value of largest |x|, d = max/-8,
 * q = min(15, (int8)(x*id + 8.5)); low nibble = elements 0..15, high = 16..31 */
void orc_quantize_row_q4_0(const float* x, void* vy, int64_t k) {
    uint8_t* y = (uint8_t*)vy;
    const int64_t nb = k / QK;
    for (int64_t i = 0; i < nb; i++) {
        float amax = 0.0f;
        float mx = 0.0f;
        for (int j = 0; j < QK; j++) {
            const float v = x[i * QK + j];
            if (amax < fabsf(v)) {
                amax = fabsf(v);
                mx = v;
            }
        }
        const float d = mx / -8;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        const uint16_t dh = orc_f32_to_f16(d);
        uint8_t* blk = y + i * 18;
        memcpy(blk, &dh, 2);
        for (int j = 0; j < QK / 2; ++j) {
            const float x0 = x[i * QK + 0 + j] * id;
            const float x1 = x[i * QK + QK / 2 + j] * id;
            const int8_t t0 = (int8_t)(x0 + 8.5f);
            const int8_t t1 = (int8_t)(x1 + 8.5f);
            const uint8_t xi0 = (uint8_t)(t0 < 15 ? t0 : 15);
            const uint8_t xi1 = (uint8_t)(t1 < 15 ? t1 : 15);
            blk[2 + j] = (uint8_t)(xi0 | (xi1 << 4));
        }
    }
}

/* ggml dequantize_row_q4_0: y[j] = ((qs[j] & 15) - 8) * d, y[j+16] = ((qs[j] >> 4) - 8) * d */
void orc_dequantize_row_q4_0(const void* vx, float* y, int64_t k) {
    const uint8_t* x = (const uint8_t*)vx;
    const int64_t nb = k / QK;
    for (int64_t i = 0; i < nb; i++) {
        const uint8_t* blk = x + i * 18;
        uint16_t dh;
        memcpy(&dh, blk, 2);
        const float d = orc_f16_to_f32(dh);
        for (int j = 0; j < QK / 2; ++j) {
            const int x0 = (blk[2 + j] & 0x0F) - 8;
            const int x1 = (blk[2 + j] >> 4) - 8;
            y[i * QK + j + 0] = (float)x0 * d;
            y[i * QK + j + QK / 2] = (float)x1 * d;
        }
    }
}

size_t orc_row_size(int type, int64_t k) {
    switch (type) {
        case ORC_TYPE_F32: return (size_t)k * 4;
        case ORC_TYPE_F16: return (size_t)k * 2;
        case ORC_TYPE_Q8_0: return (k % QK) ? 0 : (size_t)(k / QK) * 34;
        case ORC_TYPE_Q4_0: return (k % QK) ? 0 : (size_t)(k / QK) * 18;
        default: return 0;
    }
}

int orc_to_f32_row(int type, const void* x, float* y, int64_t k) {
    switch (type) {
        case ORC_TYPE_F32: memcpy(y, x, (size_t)k * 4); return 0;
        case ORC_TYPE_F16: {
            const uint8_t* p = (const uint8_t*)x;
            for (int64_t i = 0; i < k; i++) {
                uint16_t h;
                memcpy(&h, p + 2 * i, 2);
                y[i] = orc_f16_to_f32(h);
            }
            return 0;
        }
        case ORC_TYPE_Q8_0: if (k % QK) return -1; orc_dequantize_row_q8_0(x, y, k); return 0;
        case ORC_TYPE_Q4_0: if (k % QK) return -1; orc_dequantize_row_q4_0(x, y, k); return 0;
        default: return -1;
    }
}

/* ------------------------------------------------------- FLASH_ATTN_EXT */

static int type_size(int type) {
    return type == ORC_TYPE_F32 ? 4 : type == ORC_TYPE_F16 ? 2 : 0;
}

/* gather K or V of (kv head ih, kv seq is) into f32 [N][D] */
static int gather_kv(const orc_tensor* t, int64_t ih, int64_t is, float* out) {
    const int64_t D = t->ne[0], N = t->ne[1];
    const uint8_t* base = (const uint8_t*)t->data + ih * t->nb[2] + is * t->nb[3];
    const int ts = type_size(t->type);
    if (ts != 0 && t->nb[0] != ts) {
        /* transposed / strided element layout (f16 / f32 only) */
        for (int64_t n = 0; n < N; n++) {
            for (int64_t d = 0; d < D; d++) {
                const uint8_t* p = base + n * t->nb[1] + d * t->nb[0];
                if (t->type == ORC_TYPE_F32) {
                    memcpy(&out[n * D + d], p, 4);
                } else {
                    uint16_t h;
                    memcpy(&h, p, 2);
                    out[n * D + d] = orc_f16_to_f32(h);
                }
            }
        }
        return 0;
    }
    for (int64_t n = 0; n < N; n++) {
        if (orc_to_f32_row(t->type, base + n * t->nb[1], out + n * D, D) != 0) return -1;
    }
    return 0;
}

typedef struct {
    const orc_tensor *q, *k, *v, *mask;
    float* dst;
    float scale;
    int64_t next; /* work counter */
    pthread_mutex_t mu;
    int err;
} ext_job;

static void ext_one(ext_job* J, int64_t iq3, int64_t iq2, float* kf, float* vf, float* qrow,
                    float* scores, float* mrow, float* orow) {
    const orc_tensor *q = J->q, *k = J->k, *v = J->v, *mask = J->mask;
    const int64_t D = q->ne[0], NQ = q->ne[1], H = q->ne[2];
    const int64_t N = k->ne[1];
    /* GQA / seq broadcast: flash-llama.h:128-140 */
    const int64_t rk2 = q->ne[2] / k->ne[2], rk3 = q->ne[3] / k->ne[3];
    const int64_t rv2 = q->ne[2] / v->ne[2], rv3 = q->ne[3] / v->ne[3];
    if (gather_kv(k, iq2 / rk2, iq3 / rk3, kf) != 0 || gather_kv(v, iq2 / rv2, iq3 / rv3, vf) != 0) {
        J->err = -1;
        return;
    }
    for (int64_t iq1 = 0; iq1 < NQ; iq1++) {
        const uint8_t* qp = (const uint8_t*)q->data + iq1 * q->nb[1] + iq2 * q->nb[2] + iq3 * q->nb[3];
        memcpy(qrow, qp, (size_t)D * 4);
        const float* mp = NULL;
        if (mask != NULL && mask->data != NULL) {
            const uint8_t* m = (const uint8_t*)mask->data + iq1 * mask->nb[1];
            for (int64_t n = 0; n < N; n++) {
                uint16_t h;
                memcpy(&h, m + 2 * n, 2);
                mrow[n] = orc_f16_to_f32(h);
            }
            mp = mrow;
        }
        /* scores = h(q).h(k) * scale + mask  (utils.h:5-16, B transposed) */
        orc_mulmat_f32(qrow, kf, mp, scores, 1, (uint32_t)N, (uint32_t)D, J->scale, 1);
        orc_softmax(scores, (int)N, 1);
        /* O = h(P).h(v)  (utils.h:5-16, V [N][D]) */
        orc_mulmat_f32(scores, vf, NULL, orow, 1, (uint32_t)D, (uint32_t)N, 1.0f, 0);
        /* dst[(iq3*ne2*ne1 + iq2 + iq1*ne1)*D + i], ne1 = H, ne2 = NQ (flash-llama.h:434) */
        memcpy(J->dst + ((iq3 * NQ + iq1) * H + iq2) * D, orow, (size_t)D * 4);
    }
}

static void* ext_worker(void* arg) {
    ext_job* J = (ext_job*)arg;
    const int64_t D = J->q->ne[0], N = J->k->ne[1], H = J->q->ne[2], S = J->q->ne[3];
    float* kf = (float*)malloc(sizeof(float) * (size_t)(N * D));
    float* vf = (float*)malloc(sizeof(float) * (size_t)(N * D));
    float* scores = (float*)malloc(sizeof(float) * (size_t)N);
    float* mrow = (float*)malloc(sizeof(float) * (size_t)N);
    float* qrow = (float*)malloc(sizeof(float) * (size_t)D);
    float* orow = (float*)malloc(sizeof(float) * (size_t)D);
    for (;;) {
        pthread_mutex_lock(&J->mu);
        const int64_t w = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (w >= H * S || J->err) break;
        ext_one(J, w / H, w % H, kf, vf, qrow, scores, mrow, orow);
    }
    free(kf); free(vf); free(scores); free(mrow); free(qrow); free(orow);
    return NULL;
}

int orc_flash_attn_ext(const orc_tensor* q, const orc_tensor* k, const orc_tensor* v,
                       const orc_tensor* mask, float* dst, float scale, int n_threads) {
    if (q->type != ORC_TYPE_F32) return -1;
    if (k->ne[0] != q->ne[0] || v->ne[0] != q->ne[0] || k->ne[1] != v->ne[1]) return -1;
    if (q->ne[2] % k->ne[2] || q->ne[2] % v->ne[2] || q->ne[3] % k->ne[3] || q->ne[3] % v->ne[3]) return -1;
    ext_job J;
    J.q = q; J.k = k; J.v = v; J.mask = mask; J.dst = dst; J.scale = scale;
    J.next = 0; J.err = 0;
    pthread_mutex_init(&J.mu, NULL);
    if (n_threads <= 1) {
        ext_worker(&J);
    } else {
        pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
        for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, ext_worker, &J);
        for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
        free(th);
    }
    pthread_mutex_destroy(&J.mu);
    return J.err;
}
