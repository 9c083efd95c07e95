// fattn_quant.h -- ggml Q8_0 / Q4_0 row conversions on gfx950.
//
// The reference has no quantized code at all; these follow the
// published upstream-ggml algorithms (ggml-quants.c quantize_row_q8_0_ref,
// quantize_row_q4_0_ref, dequantize_row_q8_0, dequantize_row_q4_0), restated in
// oracle/fattn_oracle.c, and are bit-exact with that restatement: every
// multiply/add is a separately rounded IEEE op (contraction off + barriers),
// divisions are correctly rounded (hipcc default), f32->f16 is round-to-nearest-even.
//
// Layout: one thread per 32-element block; a wave covers 64 consecutive blocks,
// so the block reads/writes of a wave are contiguous.  These are the
// KV-cache write side (ggml cpy f32 -> q8_0/q4_0) and the dequant unit check.
#pragma once

#include "fattn_common.h"

namespace fattn {

// hipcc contracts a*b+c into FMA by default (even written as __fmul_rn /
// __fadd_rn) and folds f16(a*b) into v_fma_mix with a +0 addend (losing -0);
// ggml's reference evaluates each op separately.  The pragma and this barrier
// keep every operation individually rounded.
__device__ __forceinline__ float opaque(float x) {
    asm volatile("" : "+v"(x));
    return x;
}

static __global__ __launch_bounds__(256) void dequant_q8_0_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst,
                                                           int64_t nblocks) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblocks) return;
    const uint8_t* blk = src + i * kQ8Bytes;
    const float d = (float)__builtin_bit_cast(f16, (uint16_t)(blk[0] | (blk[1] << 8)));
    float* y = dst + i * QK;
#pragma unroll
    for (int j = 0; j < QK; j += 4) {
        f32x4 v;
        v.x = (float)(int8_t)blk[2 + j] * d;
        v.y = (float)(int8_t)blk[3 + j] * d;
        v.z = (float)(int8_t)blk[4 + j] * d;
        v.w = (float)(int8_t)blk[5 + j] * d;
        *(f32x4*)(y + j) = v;
    }
}

static __global__ __launch_bounds__(256) void dequant_q4_0_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst,
                                                           int64_t nblocks) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblocks) return;
    const uint8_t* blk = src + i * kQ4Bytes;
    const float d = (float)__builtin_bit_cast(f16, (uint16_t)(blk[0] | (blk[1] << 8)));
    float* y = dst + i * QK;
#pragma unroll
    for (int j = 0; j < QK / 2; j++) {
        const int b = blk[2 + j];
        y[j] = (float)((b & 0x0F) - 8) * d;
        y[j + QK / 2] = (float)((b >> 4) - 8) * d;
    }
}

static __global__ __launch_bounds__(256) void dequant_f16_kernel(const uint16_t* __restrict__ src, float* __restrict__ dst,
                                                          int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dst[i] = (float)__builtin_bit_cast(f16, src[i]);
}

// One ggml block of 32 values -> Q8_0 {f16 d; int8 qs[32]} (quantize_row_q8_0_ref)
__device__ __forceinline__ void quant_block_q8_0(const float (&xv)[QK], uint8_t* blk) {
#pragma clang fp contract(off)
    float amax = 0.0f;
#pragma unroll
    for (int j = 0; j < QK; j++) amax = fmaxf(amax, fabsf(xv[j]));
    const float d = amax / 127.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    const uint16_t dh = __builtin_bit_cast(uint16_t, (f16)opaque(d));
    blk[0] = dh & 0xff;
    blk[1] = dh >> 8;
#pragma unroll
    for (int j = 0; j < QK; j++) blk[2 + j] = (uint8_t)(int8_t)roundf(xv[j] * id);
}

// One ggml block of 32 values -> Q4_0 {f16 d; u8 qs[16]} (quantize_row_q4_0_ref)
__device__ __forceinline__ void quant_block_q4_0(const float (&xv)[QK], uint8_t* blk) {
#pragma clang fp contract(off)
    float amax = 0.0f, mx = 0.0f;
#pragma unroll
    for (int j = 0; j < QK; j++) {
        if (amax < fabsf(xv[j])) {
            amax = fabsf(xv[j]);
            mx = xv[j];
        }
    }
    const float d = mx * -0.125f;  // == mx / -8 exactly (power of two), keeps -0.0
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    const uint16_t dh = __builtin_bit_cast(uint16_t, (f16)opaque(d));
    blk[0] = dh & 0xff;
    blk[1] = dh >> 8;
#pragma unroll
    for (int j = 0; j < QK / 2; j++) {
        const int8_t t0 = (int8_t)(opaque(xv[j] * id) + 8.5f);
        const int8_t t1 = (int8_t)(opaque(xv[j + QK / 2] * id) + 8.5f);
        const uint8_t q0 = (uint8_t)(t0 < 15 ? t0 : 15);
        const uint8_t q1 = (uint8_t)(t1 < 15 ? t1 : 15);
        blk[2 + j] = (uint8_t)(q0 | (q1 << 4));
    }
}

template <int T>
__global__ __launch_bounds__(256) void quant_kernel(const float* __restrict__ src, uint8_t* __restrict__ dst,
                                                    int64_t nblocks) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblocks) return;
    const float* x = src + i * QK;
    float xv[QK];
#pragma unroll
    for (int j = 0; j < QK; j += 4) {
        const f32x4 v = *(const f32x4*)(x + j);
        xv[j] = v.x; xv[j + 1] = v.y; xv[j + 2] = v.z; xv[j + 3] = v.w;
    }
    if constexpr (T == FATTN_TYPE_Q8_0)
        quant_block_q8_0(xv, dst + i * kQ8Bytes);
    else
        quant_block_q4_0(xv, dst + i * kQ4Bytes);
}

// Strided f32 -> F16 / Q8_0 / Q4_0 copy: ggml's GGML_OP_CPY into a KV-cache view
// (upstream ggml cpy f32 -> f16/q8_0/q4_0).  src and dst
// have the same ne (ne0 = row length, a multiple of 32 for the block types)
// and any byte strides nb1..nb3; rows are contiguous (src nb0 = 4, dst nb0 =
// element / block size).  One thread per 32-element block (per element for
// F16): the writes of one token's K rows land straight in the cache, whether
// it is laid out [Hkv][N][row] (head stride > row) or [N][Hkv][row].
struct CpyArgs {
    const uint8_t* src;
    uint8_t* dst;
    int64_t ne0, ne1, ne2, ne3;
    int64_t snb1, snb2, snb3;
    int64_t dnb1, dnb2, dnb3;
};

template <int T>
__global__ __launch_bounds__(256) void cpy_f32_kernel(const CpyArgs a, int64_t units) {
    constexpr int UE = T == FATTN_TYPE_F16 ? 1 : QK;  // elements per unit
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= units) return;
    const int64_t upr = a.ne0 / UE;
    const int64_t b = i % upr, r = i / upr;
    const int64_t i1 = r % a.ne1, i2 = (r / a.ne1) % a.ne2, i3 = r / (a.ne1 * a.ne2);
    const float* x = (const float*)(a.src + i1 * a.snb1 + i2 * a.snb2 + i3 * a.snb3) + b * UE;
    uint8_t* y = a.dst + i1 * a.dnb1 + i2 * a.dnb2 + i3 * a.dnb3;
    if constexpr (T == FATTN_TYPE_F16) {
        *(uint16_t*)(y + b * 2) = __builtin_bit_cast(uint16_t, (f16)x[0]);
    } else {
        float xv[QK];
#pragma unroll
        for (int j = 0; j < QK; j++) xv[j] = x[j];
        if constexpr (T == FATTN_TYPE_Q8_0)
            quant_block_q8_0(xv, y + b * kQ8Bytes);
        else
            quant_block_q4_0(xv, y + b * kQ4Bytes);
    }
}

// Prefill K/V staging (the prefill planner's default for Q8_0 / Q4_0 caches):
// the quantised rows of every (sequence, kv head) -- contiguous blocks, head
// base at ik3 * nb3 + ik2 * nb2 -- become f16 rows [Skv][Hkv][N][D] in the
// caller's workspace, h(q * d) with one f16 rounding: the value the in-kernel
// dequantisation of every other kernel produces (src/utils.h:10-11), so the
// f16 prefill kernel over the staged rows computes the same attention.  The
// prefill re-reads each K/V tile once per 256-row query tile (16 times at
// n_q = 4096); staging converts it once (35.7 MB read, 67 MB written at the
// prefill shape) instead of 16 times in the MFMA loop.  Thread = 8 values of
// one block (16 B of f16 written); grid (blocks * 4 / 256, Hkv, Skv).
template <int KT>
__device__ __forceinline__ void kv_stage_f16_block(const uint8_t* __restrict__ src, int64_t nb2, int64_t nb3,
                                                   uint16_t* __restrict__ dst, int64_t nblk, int64_t bx, int head,
                                                   int seq, int gy) {
    const int64_t t = bx * 256 + threadIdx.x;
    if (t >= 4 * nblk) return;
    const int64_t b = t >> 2;
    const int j = (int)(t & 3);
    constexpr int BB = KT == FATTN_TYPE_Q8_0 ? kQ8Bytes : kQ4Bytes;
    const uint8_t* blk = src + (int64_t)seq * nb3 + (int64_t)head * nb2 + b * BB;
    const float d = (float)__builtin_bit_cast(f16, *(const uint16_t*)blk);  // (blocks are 2-byte aligned)
    const uint16_t* qw = (const uint16_t*)(blk + 2 + (KT == FATTN_TYPE_Q8_0 ? 8 * j : 8 * (j & 1)));
    uint32_t by[8];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const uint32_t w = qw[e];
        by[2 * e] = w & 0xFF;
        by[2 * e + 1] = w >> 8;
    }
    f16x8 h;
#pragma unroll
    for (int e = 0; e < 8; e++) {
        float q;
        if constexpr (KT == FATTN_TYPE_Q8_0) q = (float)(int8_t)by[e];
        else q = (float)((int)(j < 2 ? by[e] & 0x0F : by[e] >> 4) - 8);  // elements 0-15 low nibbles, 16-31 high
        h[e] = (f16)(q * d);  // exact product (<= 19 significant bits), one rounding to f16
    }
    uint16_t* y = dst + (((int64_t)seq * gy + head) * nblk + b) * QK + 8 * j;
    *(f16x8*)y = h;
}
template <int KT>
__global__ __launch_bounds__(256) void kv_stage_f16_kernel(const uint8_t* __restrict__ src, int64_t nb2, int64_t nb3,
                                                           uint16_t* __restrict__ dst, int64_t nblk) {
    kv_stage_f16_block<KT>(src, nb2, nb3, dst, nblk, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.y);
}

}  // namespace fattn
