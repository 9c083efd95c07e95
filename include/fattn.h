/*
 * fattn.h -- C ABI of the MI355X (gfx950) flash-attention-with-quantized-KV
 * kernels.  Plain C: device pointers, sizes, ggml ne/nb conventions, an opaque
 * hipStream_t.  No torch / HIP C++ types cross this boundary.
 *
 * What each entry point replaces in FSSRepo/ggml-cuda-experiments
 * (/root/reference, read-only):
 *
 *   fattn_ext()          <- flash_attn_ext_f16<D,Q,C><<<...>>>, the ggml
 *                           GGML_OP_FLASH_ATTN_EXT kernel, src/flash-llama.h:5-32
 *                           (launched at src/kernel_test.h:191-198 and
 *                           src/flash-matrix.cu:198-206).  Same argument meaning
 *                           (q/k/v/mask as ggml ne/nb views, f32 dst in the
 *                           permuted [seq][n_q][H][D] layout of flash-llama.h:434),
 *                           extended with K/V element types F16 / Q8_0 / Q4_0.
 *   fattn_ext_f16_launch()  the positional argument list of flash-llama.h:7-32,
 *                           verbatim (ne00..ne03, ne10..ne13, ne31, nb31,
 *                           nb01..nb03, nb11..nb13, ne0..ne3), for call sites
 *                           that pass it that way; K/V types added at the end.
 *   fattn_row()          <- flash_attn_row<128,nw,2,256> + fa_reduce<128,nw>
 *                           (src/flash_row_float.h:4-6, 415-416; launched at
 *                           src/kernel_test.h:161-162, src/flash-matrix.cu:226-227):
 *                           decode with query f32 [H][D], key f16 [Hkv][N][D],
 *                           value f16 TRANSPOSED [Hkv][D][N], mask f16 [N],
 *                           out f32 [H][D]; `tmp` is the caller-owned split-KV
 *                           scratch exactly like d_temporal (kernel_test.h:155).
 *   fattn_workspace_size()  the size of that scratch (kernel_test.h:155 computes
 *                           it inline).
 *   fattn_dequantize() / fattn_quantize()   ggml Q8_0 / Q4_0 row conversion on the
 *                           GPU (bit-exact with upstream ggml; absent from the
 *                           reference) -- the KV-cache write side.
 *
 * Conventions:
 *   - every pointer is a device pointer the caller allocated; the library never
 *     allocates on the hot path; `stream` is a hipStream_t (NULL = default).
 *   - return value: FATTN_OK (0) or a negative fattn_status; nothing is launched
 *     when an error is returned.  fattn_strerror() names the code.
 *   - stream-ordered and asynchronous; thread-compatible.  Global state: a
 *     per-device CU count cache, a launch-epoch counter that stamps the split-KV
 *     arrival words (monotonic; any thread may advance it), and the planner
 *     overrides of fattn_debug.h (tests, benchmarks; all off by default).
 *   - this header lists the drop-in entry points only; the diagnostics (planner
 *     overrides, the plan as text, an event-bracketed launch) are declared in
 *     fattn_debug.h, exported by the same library.
 */
#ifndef FATTN_H
#define FATTN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element types: the ggml_type numbering */
enum fattn_type {
    FATTN_TYPE_F32 = 0,
    FATTN_TYPE_F16 = 1,
    FATTN_TYPE_Q4_0 = 2,
    FATTN_TYPE_Q8_0 = 8,
};

enum fattn_status {
    FATTN_OK = 0,
    FATTN_ERR_INVALID_ARG = -1,     /* NULL pointer, bad shape, ne not divisible */
    FATTN_ERR_UNSUPPORTED_TYPE = -2,
    FATTN_ERR_UNSUPPORTED_HEAD_DIM = -3,  /* D must be 64, 80 (f16 K/V only), 96, 128 or 256 */
    FATTN_ERR_BAD_STRIDE = -4,       /* layout the kernels cannot address */
    FATTN_ERR_WORKSPACE = -5,        /* workspace too small */
    FATTN_ERR_LAUNCH = -6,           /* HIP launch failure */
    FATTN_ERR_ALIGNMENT = -7,
};

/* A ggml tensor view: ne[i] elements along dim i, nb[i] byte stride of dim i. */
typedef struct fattn_tensor {
    const void* data;
    int32_t type;
    int32_t pad_;
    int64_t ne[4];
    int64_t nb[4];
} fattn_tensor;

/* GGML_OP_FLASH_ATTN_EXT:
 *   q    f32  ne = [D, n_q, H, S]        (any nb with nb[0] == 4)
 *   k    F16/Q8_0/Q4_0  ne = [D, N, Hkv, Skv]  rows contiguous (nb[0] = type size)
 *   v    F16/Q8_0/Q4_0  ne = [D, N, Hkv, Skv]; rows contiguous, or for F16 only
 *        transposed (nb[1] == 2, nb[0] == N*2 style strides).  v's type may
 *        differ from k's (llama.cpp's separate K / V cache types) at D = 64,
 *        128 and 256: the split-KV kernel takes every such pair
 *   mask F16 ne = [N', rows >= n_q] with N' >= N rounded up to even (ggml pads
 *        mask rows to GGML_KQ_MASK_PAD), 4-byte aligned rows; row = query
 *        index, broadcast over heads and sequences; or data == NULL for no mask
 *   dst  f32 contiguous [S][n_q][H][D]
 *   H % Hkv == 0 (GQA broadcast), S % Skv == 0.
 *   softmax(scale * q.k^T + mask) . v per (seq, head, query row).  A row whose
 *   mask is -inf everywhere yields NaN, as the reference's softmax does
 *   (src/utils.h:30-49). */
typedef struct fattn_params {
    fattn_tensor q, k, v, mask;
    float* dst;
    float scale;
    int32_t kv_chunk;      /* split-KV chunk length in positions; 0 = auto */
    void* workspace;       /* split-KV scratch, >= fattn_workspace_size() bytes.  Zero a new
                              allocation once (fattn_workspace_init): a launch stamps its
                              arrival words with a fresh epoch by atomic max, which
                              supersedes any word an earlier launch left (re-armed, or
                              mid-count after an abort) and any word whose top 8 bits are
                              not all ones -- but an uninitialised word that happens to
                              read 0xFF in its top bits with an epoch field ahead of the
                              launch's would outrank the stamp.  No re-zeroing is needed
                              between launches.  Launches that share one workspace must be
                              ordered on one stream */
    size_t workspace_bytes;
} fattn_params;

size_t fattn_workspace_size(const fattn_params* p);
/* Zero a workspace (hipMemsetAsync on `stream`); call once per allocation.  The
 * split-KV chunks of a tile meet through 64-bit arrival words kept at the front
 * of the workspace, [0xFF | epoch:32 | generation:8 | count:16]; each launch
 * stamps them with its own epoch (atomic max) before counting, so memory left by
 * an earlier or an aborted launch is superseded -- but not a never-initialised
 * word whose top 8 bits are all ones with an epoch above the current one (e.g.
 * 0xFF fill), which this call clears.  The last arriver re-arms a word (count 0,
 * generation + 1), so a replayed graph finds it clean. */
int fattn_workspace_init(void* workspace, size_t workspace_bytes, void* stream);
int fattn_ext(const fattn_params* p, void* stream);

/* flash-llama.h:7-32 argument list (K and V share nb11..nb13, flash-llama.h:123-125;
 * mask rows padded to ne31, nb31 bytes per row). */
int fattn_ext_f16_launch(const void* q, const void* k, const void* v, const void* mask, float* dst, float scale,
                         int ne00, int ne01, int ne02, int ne03, int ne10, int ne11, int ne12, int ne13, int ne31,
                         int nb31, int nb01, int nb02, int nb03, int nb11, int nb12, int nb13, int ne0, int ne1,
                         int ne2, int ne3, int k_type, int v_type, void* workspace, size_t workspace_bytes,
                         void* stream);

/* flash_attn_row + fa_reduce (flash_row_float.h): query f32 [H][D], key f16
 * [Hkv][N][D] (head_stride = D*N elements), value f16 [Hkv][D][N], mask f16 [N],
 * qkv f32 [H][D]; r_kv_heads = H / Hkv.  tmp: >= fattn_row_workspace_size(),
 * its arrival words are epoch-stamped per launch (as for fattn_params.workspace). */
size_t fattn_row_workspace_size(int head_dim, int kv_size, int num_heads);
int fattn_row(const float* query, const void* key, const void* value, const void* mask, void* tmp,
              size_t tmp_bytes, float* qkv, int head_dim, int kv_size, int num_heads, float scale,
              int head_stride, int r_kv_heads, void* stream);

/* ggml row conversions on the GPU (n_rows rows of k elements each, contiguous).
 * dequantize: Q8_0/Q4_0/F16 -> f32 (bit-exact with ggml dequantize_row_*).
 * quantize:   f32 -> Q8_0/Q4_0 (bit-exact with ggml quantize_row_*_ref). */
int fattn_dequantize(int type, const void* src, float* dst, int64_t k, int64_t n_rows, void* stream);
int fattn_quantize(int type, const float* src, void* dst, int64_t k, int64_t n_rows, void* stream);

/* GGML_OP_CPY f32 -> F16 / Q8_0 / Q4_0 into a strided view: the KV-cache write
 * (quantize-on-write; upstream ggml cpy_f32_q /
 * cpy_f32_f16, absent from the reference).  src: f32, nb[0] = 4; dst: same ne,
 * nb[0] = element / block bytes, any nb[1..3] -- e.g. one token's Hkv rows
 * written into a [Hkv][N][row] cache (nb1 = N * row bytes) or a [N][Hkv][row]
 * cache (nb1 = row bytes).  ne[0] a multiple of 32 for Q8_0 / Q4_0.  Values
 * bit-exact with ggml quantize_row_*_ref / f16 round-to-nearest-even. */
int fattn_cpy(const fattn_tensor* src, const fattn_tensor* dst, void* stream);

const char* fattn_strerror(int status);
/* bytes of one row of k elements (0 if unsupported) */
size_t fattn_row_size(int type, int64_t k);
/* library version string */
const char* fattn_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FATTN_H */
