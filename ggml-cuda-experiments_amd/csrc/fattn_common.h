// fattn_common.h -- shared device helpers for the gfx950 attention kernels.
//
// Replaces src/tensor-mma.h (WMMA 16x16x16 fragments, WARP_SIZE 32) and the
// warp_reduce_* butterflies of src/cuda_info.h:46-85 with CDNA4 primitives:
// wave64 shuffles and __builtin_amdgcn_mfma_f32_16x16x32_f16.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fattn_debug.h"

namespace fattn {

constexpr int kWave = 64;

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) uint8_t lds_u8;

// ggml block geometry
constexpr int QK = 32;
constexpr int kQ8Bytes = 34;  // {f16 d; int8 qs[32]}
constexpr int kQ4Bytes = 18;  // {f16 d; uint8 qs[16]}

template <int T>
struct TypeInfo;
template <>
struct TypeInfo<FATTN_TYPE_F16> {
    static constexpr int block_elems = 1;
    static constexpr int block_bytes = 2;
};
template <>
struct TypeInfo<FATTN_TYPE_Q8_0> {
    static constexpr int block_elems = QK;
    static constexpr int block_bytes = kQ8Bytes;
};
template <>
struct TypeInfo<FATTN_TYPE_Q4_0> {
    static constexpr int block_elems = QK;
    static constexpr int block_bytes = kQ4Bytes;
};

template <int T, int D>
constexpr int row_bytes() {
    return D / TypeInfo<T>::block_elems * TypeInfo<T>::block_bytes;
}

// ---------------------------------------------------------------- bit helpers

__device__ __forceinline__ uint32_t perm_b32(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t shift) {
    return __builtin_amdgcn_alignbyte(hi, lo, shift);
}
__device__ __forceinline__ f16x2 as_h2(uint32_t x) { return __builtin_bit_cast(f16x2, x); }
__device__ __forceinline__ uint32_t as_u32(f16x2 x) { return __builtin_bit_cast(uint32_t, x); }

// f16 pair with both halves = the f16 whose bits are the low 16 bits of x
__device__ __forceinline__ f16x2 bcast_h(uint32_t bits16) {
    const uint32_t b = bits16 & 0xffffu;
    return as_h2(b | (b << 16));
}

// Four int8 (two's complement, packed in a dword) -> two f16 pairs holding the
// exact integer values.  Magic-number trick: f16 bits 0x64uu = 1024 + uu, so
// with uu = q ^ 0x80 = q + 128 the value is 1152 + q; subtracting 1152 is exact.
__device__ __forceinline__ void i8x4_to_h2x2(uint32_t w, f16x2& lo, f16x2& hi) {
    const uint32_t t = w ^ 0x80808080u;
    const uint32_t p0 = perm_b32(0x64646464u, t, 0x04010400u);  // bytes: t0,0x64,t1,0x64
    const uint32_t p1 = perm_b32(0x64646464u, t, 0x04030402u);  // bytes: t2,0x64,t3,0x64
    const f16x2 off = {(f16)-1152.0f, (f16)-1152.0f};
    lo = as_h2(p0) + off;
    hi = as_h2(p1) + off;
}

// Four nibbles already isolated in the low 4 bits of each byte of w ->
// two f16 pairs holding (nib - 8) exactly (Q4_0 offset).
__device__ __forceinline__ void u4x4_to_h2x2(uint32_t w, f16x2& lo, f16x2& hi) {
    const uint32_t p0 = perm_b32(0x64646464u, w, 0x04010400u);
    const uint32_t p1 = perm_b32(0x64646464u, w, 0x04030402u);
    const f16x2 off = {(f16)-1032.0f, (f16)-1032.0f};
    lo = as_h2(p0) + off;
    hi = as_h2(p1) + off;
}

// ---------------------------------------------------------------- LDS reads
// The ggml block rows sit in LDS exactly as in HBM, so a block's qs bytes are
// only 2-byte aligned.  read8_at<MOD8>() returns the 8 bytes at `off` where
// off % 8 == MOD8 is known at compile time.

template <int MOD8>
__device__ __forceinline__ u32x2 read8_at(const uint8_t* smem, uint32_t off) {
    u32x2 r;
    if constexpr (MOD8 == 0) {
        r = *(const u32x2*)(smem + off);
    } else if constexpr (MOD8 == 4) {
        r.x = *(const uint32_t*)(smem + off);
        r.y = *(const uint32_t*)(smem + off + 4);
    } else if constexpr (MOD8 == 2) {
        const u32x2 w01 = *(const u32x2*)(smem + off - 2);
        const uint32_t w2 = *(const uint32_t*)(smem + off + 6);
        r.x = alignbyte(w01.y, w01.x, 2);
        r.y = alignbyte(w2, w01.y, 2);
    } else {  // 6
        const uint32_t w0 = *(const uint32_t*)(smem + off - 2);
        const u32x2 w12 = *(const u32x2*)(smem + off + 2);
        r.x = alignbyte(w12.x, w0, 2);
        r.y = alignbyte(w12.y, w12.x, 2);
    }
    return r;
}

// ---------------------------------------------------------------- wave reductions
// wave64 replacements for warp_reduce_max / warp_reduce_sum (cuda_info.h:46-85).
// Attention only needs the 4 lanes {l, l^16, l^32, l^48} that share one MFMA
// column.  gfx950's v_permlane16_swap / v_permlane32_swap exchange rows of 16 /
// halves of 32 lanes on the VALU (no LDS round trip like ds_bpermute):
// swap(a=x, b=x) leaves a = x with odd rows <- even rows and b = x with even
// rows <- odd rows, so op(a, b) is the xor-16 (resp. xor-32) reduction in every
// lane.  Written as inline asm with both registers in/out: through the
// __builtin_amdgcn_permlane*_swap intrinsics hipcc (ROCm 7.2) stores the first
// result for both when the operands are copies of one value (caught by
// tests/test_gpu_prims.py).  The s_nop covers the VALU-write -> permlane hazard,
// which the compiler does not see inside the asm.
__device__ __forceinline__ float xor16_pair(float x, bool is_max) {
    float a = x, b = x;
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return is_max ? fmaxf(a, b) : a + b;
}
__device__ __forceinline__ float xor32_pair(float x, bool is_max) {
    float a = x, b = x;
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    return is_max ? fmaxf(a, b) : a + b;
}
__device__ __forceinline__ float grp4_max(float x) { return xor32_pair(xor16_pair(x, true), true); }
__device__ __forceinline__ float grp4_sum(float x) { return xor32_pair(xor16_pair(x, false), false); }

// Segmented reductions over contiguous power-of-two lane groups of `seg`
// lanes (seg <= 64, wave-uniform), entirely on the VALU: DPP quad_perm (xor 1,
// xor 2), row_half_mirror / row_mirror (pair the 4- / 8-lane halves once
// those are uniform), then the permlane swaps for rows / halves.  Every lane
// ends with its group's result.  EXEC must be full.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
template <bool IS_MAX>
__device__ __forceinline__ float seg_reduce(float x, int seg) {
    auto op = [](float a, float b) { return IS_MAX ? fmaxf(a, b) : a + b; };
    if (seg > 1) x = op(x, dpp_mov<0xB1>(x));   // quad_perm [1,0,3,2]
    if (seg > 2) x = op(x, dpp_mov<0x4E>(x));   // quad_perm [2,3,0,1]
    if (seg > 4) x = op(x, dpp_mov<0x141>(x));  // row_half_mirror
    if (seg > 8) x = op(x, dpp_mov<0x140>(x));  // row_mirror
    if (seg > 16) x = xor16_pair(x, IS_MAX);
    if (seg > 32) x = xor32_pair(x, IS_MAX);
    return x;
}

__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) x = fmaxf(x, __shfl_xor(x, m, kWave));
    return x;
}
__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) x += __shfl_xor(x, m, kWave);
    return x;
}

// ---------------------------------------------------------------- sc1 memory ops
// Write-through stores / L1-bypassing loads for data handed between workgroups
// of one launch (MI355X_MICROARCH.md, inter-workgroup visibility).
// Stores: inline asm with no destination register (nothing for the compiler
// to misplace); callers drain them with an explicit s_waitcnt vmcnt(0).  The
// trailing s_nop covers the VMEM-store-data hazard (a store of more than 8
// bytes must not have its data VGPRs overwritten by the next VALU instruction):
// hipcc's hazard recognizer does not see inside inline asm, and with the
// multi-query kernel's register pressure it reused the data registers of one
// store as the address of the next at once (elements .x/.y corrupted).
__device__ __forceinline__ void st_sc1(void* p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1_x2(void* p, u32x2 v) {
    asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
// Loads of handed-off words: compiler-tracked (relaxed agent-scope atomic
// loads lower to global_load_dword(x2) ... sc1), so hipcc places every wait
// itself -- no register is live before its data has landed.
__device__ __forceinline__ u32x2 ld_sc1_x2(const void* p) {
    const uint64_t x = __hip_atomic_load((const uint64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return u32x2{(uint32_t)x, (uint32_t)(x >> 32)};
}
__device__ __forceinline__ uint32_t ld_sc1_u32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Keeps uses of a value loaded by an UNTRACKED inline-asm load below the
// explicit wait that retires it (the split kernel's Q and mask-word prefetch,
// the only such loads left; tools/isa_hazard_check.py audits the ISA).
// Integer scalars / vectors only: with a float-vector "+v"/"=v" operand hipcc
// (ROCm 7.2) mis-assigned the elements (a bit_cast of .y read .x's register).
// The comment "RETIRED(tag) <registers>" marks, for tools/isa_hazard_check.py,
// the point from which the loads of `tag` have landed (the caller's wait sits
// just before it; volatile asm statements keep their source order).
template <int TAG, typename T>
__device__ __forceinline__ void reg_fence(T& v) {
    static_assert(!__is_same(T, f32x4) && !__is_same(T, f32x2), "float vector asm operands are miscompiled");
    asm volatile("; RETIRED(%1) %0" : "+v"(v) : "n"(TAG));
}

__device__ __forceinline__ f32x4 mfma16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

}  // namespace fattn
