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
 *   - stream-ordered and asynchronous; thread-compatible.  Global state: the
 *     process-wide planner overrides of fattn_set_option (tests, benchmarks), a
 *     per-device CU count cache, and a launch-epoch counter that stamps the
 *     split-KV arrival words (monotonic; any thread may advance it).
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

/* Same as fattn_ext, additionally recording the hipEvent_t `ev_begin` / `ev_end`
 * on `stream` immediately before the first and after the last kernel of the
 * plan -- the attention kernel, plus the chunk-merge kernel when the plan
 * merges its split-KV partials in a second launch (fattn_describe names both),
 * plus the prefill mask-flags pass before it -- so a caller can time the whole
 * attention op on the device with hipEventElapsedTime.  Either event may be NULL. */
int fattn_ext_events(const fattn_params* p, void* stream, void* ev_begin, void* ev_end);

/* Planner overrides (tests, benchmarks).  They are PROCESS-WIDE: one call changes
 * the plans of every later fattn_ext / fattn_describe / fattn_workspace_size on
 * every host thread (stored in atomics, so never torn, but a thread that sets an
 * option while another plans races with it).  Set them before launching, or from
 * one thread.  Option ids of removed experiments are not reused.  Returns
 * FATTN_OK or FATTN_ERR_INVALID_ARG. */
enum {
    FATTN_OPT_MQ_ROWS_PER_WAVE = 1, /* multi-query kernel: 0 = auto, 16 (4 waves x 16 rows), 32 (8 waves x 32 rows) */
    FATTN_OPT_MQ_DISABLE = 2,       /* 1 = never pick the multi-query kernel (split-KV kernel only) */
    FATTN_OPT_SPLIT_STEPS = 3,      /* split kernel: 32-position steps per wave (0 = auto, 1..64) */
    FATTN_OPT_SPLIT_INFLIGHT = 4,   /* split kernel: steps in flight per wave (0 = auto, 1..4; LDS permitting) */
    FATTN_OPT_PF = 5,               /* prefill kernel: 0 = auto, 1 = never, 2 = whenever eligible (even if the
                                       workgroups do not fill the chip) */
    FATTN_OPT_PF_STAGGER = 6,       /* prefill kernel, bit 1 (default on): waves 4-7 at s_setprio 1; bit 2:
                                       XCD-grouped workgroup order (the query tiles of a kv head on one XCD);
                                       bit 0 (a phase stagger of SIMD partners) was removed and is rejected */
    FATTN_OPT_SPLIT_WAVE_MERGE = 10 /* split kernel, one-row tiles with <= 32 wave partials: 0 = every wave
                                       publishes and the last-arriving wave merges (default), 1 = the
                                       workgroup-level merge used for all other tiles */,
    FATTN_OPT_SPLIT_PRIO = 11       /* split kernel wave priorities: 0 = staggered 3/2/1/0 (default), 1 = none,
                                       2 = staggered only while the first steps are issued */,
    FATTN_OPT_PF_SKIP = 12          /* masked prefill: 0 = a pre-pass flags the blocks with any key above -inf
                                       and the kernel walks only the live KV range, longest query tiles
                                       first (default; the workspace holds n_qt * N/64 flag bytes),
                                       1 = no pre-pass (every tile fetched; all -inf wave blocks still skipped) */,
    FATTN_OPT_MQ_MIN_ROWS = 13,     /* multi-query kernel only from this many packed (query x head) rows per kv
                                       head (0 = the default, 64; minimum 32); fewer rows take the split-KV kernel.
                                       An explicit value (64 included) also lifts the default's rule that every
                                       KV chunk hold two 128-key tiles */
    FATTN_OPT_SPLIT_WAVES = 19,     /* split kernel waves per workgroup: 0 = auto, 4, 8 or 16 (16-B row path;
                                       16 needs the Q8_0/Q4_0 register budget, else clamped to 8) */
    FATTN_OPT_SPLIT_SKIP = 20       /* split kernel, masked: 0 = steps whose mask is -inf for every key and row
                                       of the tile are neither loaded nor computed (default; the mask words are
                                       read beside Q), 1 = every step loaded and computed */,
    FATTN_OPT_SPLIT_MERGE = 21,     /* split kernel, tiles of several packed rows: 0 = with 4+ chunks the partials
                                       merge one wave per (tile, row), in a second launch or in-kernel
                                       (FATTN_OPT_MERGE_IN_KERNEL) (default), 1 = the last-arriving workgroup merges
                                       the whole tile (combine_tile) */
    FATTN_OPT_BD = 22               /* batched-decode kernels (64-row workgroups, 16-B rows): the compute /
                                       build-role form fattn_bdp_kernel for Q8_0 / Q4_0 K/V at D = 64, 96, 128;
                                       the all-waves form fattn_bd_kernel for Q8_0 / Q4_0 at D = 128 (value 2
                                       only) and for f16 K/V at D = 64, 96, 128 (always: f16 has no role form).
                                       0 = auto (from 64 packed rows per kv head, below the prefill shapes),
                                       1 = never, 2 = the all-waves form whenever eligible (quantised D = 64 / 96:
                                       the multi-query kernel instead), 3 = the role form whenever eligible --
                                       on f16 K/V 3 runs the all-waves form */,
    /* 23: a removed experiment (one-row partials as data-tagged granules), rejected */
    FATTN_OPT_MERGE_IN_KERNEL = 24  /* chunk partials of multi-row tiles (split kernel with 4+ chunks, batched-
                                       decode kernel): 0 = merged in a second launch (default); 1 = inside the
                                       launch when the whole grid is co-resident -- the tile's workgroups wait
                                       for each other, then each merges a share of the rows (0.6-1.5 us slower).
                                       Co-residency is judged from CU count, LDS and launch bounds only: on a
                                       device shared with other streams or processes (or CU-masked) a waiting
                                       workgroup's bounded poll can give up, and it then writes NaN rows while
                                       fattn_ext has returned FATTN_OK.  Diagnostics only; keep 0 in production */,
    FATTN_OPT_BD_XCD = 25           /* batched-decode kernels: workgroup order. 0 = auto (XCD-grouped), 1 = plain
                                       (chunk fastest), 2 = XCD-grouped: each of the 8 XCDs takes whole (kv head x
                                       row tile)s, so a tile's Q rows come from HBM once, not once per chunk
                                       (needs a grid of a multiple of 8 workgroups; otherwise plain) */,
    FATTN_OPT_SPLIT_XCD = 26        /* split kernel: workgroup order. 0 = auto (XCD-grouped for one-row tiles merged
                                       in the launch, e.g. config 3; plain otherwise), 1 = plain, 2 = XCD-grouped:
                                       a tile's chunk workgroups on one XCD (grid a multiple of 8 workgroups) */,
    /* 27: a removed experiment (speculative granule merge of one-row tiles: slower), rejected */
    FATTN_OPT_PF_STAGE = 28         /* prefill kernel over Q8_0 / Q4_0 K/V: 0 = auto (staged), 1 = dequantised in
                                       the kernel, tile by tile, once per 256-row query tile; 2 = staged: the rows
                                       converted once to f16 in the workspace (kv_stage_f16, + 2 * Skv * Hkv * N *
                                       D * 2 bytes of fattn_workspace_size), then the f16 prefill kernel */,
    FATTN_OPT_PF_FORM = 29          /* prefill body over f16 rows (native or staged) at D = 128: 0 = auto (5), 1 =
                                       the 8-wave form (fattn_pf_kernel), 2 = one wave per SIMD (fattn_pf4_kernel),
                                       3 = the same with the rebalanced phase schedule, 4 = the same pipelined
                                       (two 32-MFMA phases per tile, P.V one tile behind S), 5 = pipelined and
                                       balanced (each phase carries one row block's exponentials and the other's
                                       scores / max, interleaved over its 32 steps) */
};
int fattn_set_option(int option, int value);

/* Diagnostic: the kernel(s) fattn_ext would launch for `p` and the plan's
 * grid / LDS / chunk / workspace, as text (NUL-terminated, at most cap bytes).
 * Returns FATTN_OK or the error fattn_ext would return. */
int fattn_describe(const fattn_params* p, char* out, size_t cap);

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
