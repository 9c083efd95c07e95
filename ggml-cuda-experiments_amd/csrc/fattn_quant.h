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

__global__ __launch_bounds__(256) void dequant_q8_0_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst,
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

__global__ __launch_bounds__(256) void dequant_q4_0_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst,
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

__global__ __launch_bounds__(256) void dequant_f16_kernel(const uint16_t* __restrict__ src, float* __restrict__ dst,
                                                          int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dst[i] = (float)__builtin_bit_cast(f16, src[i]);
}

__global__ __launch_bounds__(256) void quant_q8_0_kernel(const float* __restrict__ src, uint8_t* __restrict__ dst,
                                                         int64_t nblocks) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblocks) return;
    const float* x = src + i * QK;
    float xv[QK];
#pragma unroll
    for (int j = 0; j < QK; j += 4) {
        const f32x4 v = *(const f32x4*)(x + j);
        xv[j] = v.x; xv[j + 1] = v.y; xv[j + 2] = v.z; xv[j + 3] = v.w;
    }
    float amax = 0.0f;
#pragma unroll
    for (int j = 0; j < QK; j++) amax = fmaxf(amax, fabsf(xv[j]));
    const float d = amax / 127.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    uint8_t* blk = dst + i * kQ8Bytes;
    const uint16_t dh = __builtin_bit_cast(uint16_t, (f16)opaque(d));
    blk[0] = dh & 0xff;
    blk[1] = dh >> 8;
#pragma unroll
    for (int j = 0; j < QK; j++) blk[2 + j] = (uint8_t)(int8_t)roundf(xv[j] * id);
}

__global__ __launch_bounds__(256) void quant_q4_0_kernel(const float* __restrict__ src, uint8_t* __restrict__ dst,
                                                         int64_t nblocks) {
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblocks) return;
    const float* x = src + i * QK;
    float xv[QK];
#pragma unroll
    for (int j = 0; j < QK; j += 4) {
        const f32x4 v = *(const f32x4*)(x + j);
        xv[j] = v.x; xv[j + 1] = v.y; xv[j + 2] = v.z; xv[j + 3] = v.w;
    }
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
    uint8_t* blk = dst + i * kQ4Bytes;
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

}  // namespace fattn
