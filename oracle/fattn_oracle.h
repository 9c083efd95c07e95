/*
 * fattn_oracle.h -- CPU restatement of the reference's attention oracle.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (libfattn.so, the
 * kernel_test harness, the Python host package) links or calls this code.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / CPU baseline.
 *
 * What it restates (reference = FSSRepo/ggml-cuda-experiments, /root/reference):
 *   orc_mulmat_f32     src/utils.h:5-16   (operands rounded through fp16, fp32 acc)
 *   orc_mulmat_f16     src/utils.h:18-28  (A f32, B f16, mask f16 per row)
 *   orc_softmax        src/utils.h:30-49  (single-pass online max/sum, expf)
 *   orc_fill_buffer    src/utils.h:51-55  (always writes 0, ignores val)
 *   orc_random         src/utils.h:57-61  (1 - 2*rand()/RAND_MAX in float)
 *   orc_kernel_test_cpu  src/kernel_test.h:50-62 (per-head QK^T, softmax, PV)
 *   orc_flash_attn_ext   the same arithmetic applied to the ggml FLASH_ATTN_EXT
 *                        argument convention of src/flash-llama.h:5-32,120-140,
 *                        151,194,434 (ne/nb strides, GQA broadcast, mask rows,
 *                        permuted dst)
 * and, because the reference has NO quantized code, the ggml
 * block formats from upstream ggml (ggml-quants.c, quantize_row_q8_0_ref /
 * quantize_row_q4_0_ref / dequantize_row_q8_0 / dequantize_row_q4_0; ggml is
 * not vendored and has no pinned version in the reference -- see DESIGN.md).
 *
 * Parity pinning: the fp16 conversion, mulmat, softmax and random restatements
 * are checked bit-for-bit against the reference's own src/utils.h compiled in
 * this container (oracle/_ref, see oracle/Makefile) and against the hand-written
 * known-answer test in src/misc/flash-attn.cu:202-295.
 */
#ifndef FATTN_ORACLE_H
#define FATTN_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ggml type ids (same numbering as ggml_type) */
enum { ORC_TYPE_F32 = 0, ORC_TYPE_F16 = 1, ORC_TYPE_Q4_0 = 2, ORC_TYPE_Q8_0 = 8 };

/* fp16 <-> fp32, round-to-nearest-even, identical to cuda_fp16 __float2half /
 * __half2float which src/utils.h:10-11,23,25 use. */
uint16_t orc_f32_to_f16(float x);
float orc_f16_to_f32(uint16_t h);
float orc_round_f16(float x);
void orc_f32_to_f16_n(const float* x, uint16_t* y, int64_t n);
void orc_f16_to_f32_n(const uint16_t* x, float* y, int64_t n);

/* src/utils.h:5-16 */
void orc_mulmat_f32(const float* A, const float* B, const float* mask, float* C,
                    uint32_t M, uint32_t N, uint32_t K, float scale, int B_transposed);
/* src/utils.h:18-28 */
void orc_mulmat_f16(const float* A, const uint16_t* B, const uint16_t* mask, float* C,
                    uint32_t M, uint32_t N, uint32_t K, float scale, int B_transposed);
/* src/utils.h:30-49 */
void orc_softmax(float* scores, int kv_size, int batch_size);
/* src/utils.h:51-55 */
void orc_fill_buffer(float* arr, float val, uint32_t count);
/* src/utils.h:57-61 (glibc rand(); orc_srand wraps srand) */
void orc_random(float* arr, uint32_t count);
void orc_srand(unsigned seed);

/* src/kernel_test.h:50-62 -- CPU reference of the harness: query [H][D] f32,
 * key/value [Hkv][N][D] f32, mask [N] f32, out [H][D] f32. */
void orc_kernel_test_cpu(const float* query, const float* key, const float* value,
                         const float* mask, float* out, int kv_size, int head_dim,
                         int num_heads, int num_kv_heads, float scale);

/* ggml block formats (upstream ggml, restated). Q8_0: {fp16 d; int8 qs[32]},
 * 34 B. Q4_0: {fp16 d; uint8 qs[16]}, 18 B. k must be a multiple of 32. */
void orc_quantize_row_q8_0(const float* x, void* y, int64_t k);
void orc_dequantize_row_q8_0(const void* x, float* y, int64_t k);
void orc_quantize_row_q4_0(const float* x, void* y, int64_t k);
void orc_dequantize_row_q4_0(const void* x, float* y, int64_t k);
/* bytes of one row of k elements of a ggml type (0 for unsupported) */
size_t orc_row_size(int type, int64_t k);
/* dequantize/convert one contiguous row of `type` to f32 */
int orc_to_f32_row(int type, const void* x, float* y, int64_t k);

/* ggml-style tensor view (ne = elements per dim, nb = byte strides) */
typedef struct orc_tensor {
    const void* data;
    int32_t type;
    int64_t ne[4];
    int64_t nb[4];
} orc_tensor;

/* FLASH_ATTN_EXT with the reference arithmetic:
 *   scores = mulmat_cpu(h(q), h(deq(k))) * scale + mask   (utils.h:5-16 semantics)
 *   P      = softmax(scores)                               (utils.h:30-49)
 *   O      = mulmat_cpu(h(P), h(deq(v)))                   (utils.h:5-16)
 * q: f32 [D, n_q, H, S]; k/v: [D, N, Hkv, S_kv] f16/q8_0/q4_0/f32 (row-contiguous
 * or, for f16/f32 v only, transposed: nb[0] != type size); mask: f16 [N, rows]
 * (row = query index iq1, broadcast over heads/seqs) or data==NULL;
 * dst: contiguous f32 [D, H, n_q, S] (flash-llama.h:434).
 * n_threads > 1 parallelises over (seq, head). Returns 0 on success. */
int orc_flash_attn_ext(const orc_tensor* q, const orc_tensor* k, const orc_tensor* v,
                       const orc_tensor* mask, float* dst, float scale, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
