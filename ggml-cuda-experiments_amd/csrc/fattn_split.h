// fattn_split.h -- split-KV ("flash decoding") attention kernel for gfx950.
//
// Replaces flash_attn_row / flash_attn_row_fast (src/flash_row_float.h:4-413)
// and, for small query counts, flash_attn_ext_f16 (src/flash-llama.h:5-438).
// Same math: s = scale*q.k + mask, online softmax (max, sum) per KV chunk,
// unnormalised P.V, merged with the log-sum-exp rule of fa_reduce
// (src/flash_row_float.h:429-471) -- but built MI355X-first:
//
//  * Work unit: one workgroup = 4 waves = (KV chunk, 16 packed query rows).
//    The 16 MFMA rows pack (query row x q-head) pairs that share one KV head
//    (GQA broadcast ik2 = iq2 / (ne02/ne12), flash-llama.h:128-140), so a
//    32q/8kv decode packs 4 heads into one tile instead of re-reading K/V 4x.
//  * Each wave owns a contiguous slice of the chunk and streams it in steps of
//    32 positions.  The raw ggml rows (f16 / Q8_0 / Q4_0 blocks, exactly as in
//    HBM) plus the step's mask rows are copied HBM -> LDS with
//    global_load_lds_dwordx4 (fully coalesced 1 KiB per wave instruction; a
//    dword-granular variant serves arbitrary ggml row strides), NBUF steps in
//    flight per wave, retired with counted s_waitcnt vmcnt -- no workgroup
//    barrier inside the loop.
//  * Dequantisation happens on the LDS -> VGPR hop straight into MFMA operand
//    layout: K as the A operand of S^T = K.Q^T (v_mfma_f32_16x16x32_f16),
//    V (transposed by byte gathers for Q8_0/Q4_0, by ds_read_b64_tr_b16 for f16)
//    as the A operand of O^T = V^T.P^T.  The "swapped" products keep each
//    query column on one lane group, so P feeds PV with no lane movement and
//    the row max/sum need only two xor-shuffles (wave64: lanes l, l^16, l^32,
//    l^48).  Dequant is h(q*d) with one f16 rounding -- exactly the oracle's
//    fp16 rounding of the dequantised value (src/utils.h:10-11).
//  * fp32 MFMA accumulators, fp32 softmax state (the reference keeps fp16).
//  * The 4 waves' states merge through LDS; with several chunks the partials
//    (O, m, l) go to the caller's workspace and fattn_combine merges them.
#pragma once

#include "fattn_common.h"

namespace fattn {

constexpr int kSplitWaves = 4;
constexpr int kStep = 32;   // KV positions per wave step (= one PV k-step)
constexpr int kRows = 16;   // packed query rows per workgroup (MFMA N)
constexpr int VT_F16T = 100;  // V f16 stored transposed ([D][N], flash_row_float.h:177)

struct SplitArgs {
    const uint8_t* q;
    const uint8_t* k;
    const uint8_t* v;
    const uint8_t* mask;
    float* dst;
    float* ws_o;   // [S][Y][C][16][D]
    float* ws_ml;  // [S][Y][C][16][2]
    int64_t q_nb1, q_nb2, q_nb3;
    int64_t k_nb1, k_nb2, k_nb3;
    int64_t v_nb0, v_nb1, v_nb2, v_nb3;
    int64_t m_nb1;
    int NQ, H, S;       // q ne1, ne2, ne3
    int N;              // kv length
    int rk2, rk3;       // H/Hkv, S/Skv
    int R;              // q-heads packed per tile
    int QPT;            // query rows per tile
    int n_hsub, n_qt;   // head subgroups, query-row tiles
    float R_inv;        // 1/R: m / R == int((m + 0.5) * R_inv) exactly for m, R <= 16
    int chunk_len;      // positions per workgroup (multiple of kStep*kSplitWaves)
    int n_chunks;
    int ncp;            // next power of two >= n_chunks (combine kernel)
    float scale_log2;   // scale * log2(e)
    int has_mask;
    int nbuf;           // steps in flight per wave (1..4); LDS per wave = wave_bytes
    int wave_bytes;
};

template <int KT, int VT, int D>
struct SplitCfg {
    static constexpr int KTT = KT;
    static constexpr int VTT = (VT == VT_F16T) ? FATTN_TYPE_F16 : VT;
    static constexpr int rowK = row_bytes<KT, D>();
    static constexpr int rowV = row_bytes<VTT, D>();
    static constexpr int kBytes = kStep * rowK;
    static constexpr int vBytes = kStep * rowV;
    static constexpr int mBytes = kRows * kStep * 2;  // up to 16 distinct mask rows
    static constexpr int stepBytes = (kBytes + vBytes + mBytes + 15) / 16 * 16;
    static constexpr int vscBytes = 0;
    static constexpr int kMergeStride = D + 4;  // floats; +16 B per row spreads rows over banks
    static constexpr int mergeBytes = kRows * kMergeStride * 4 + kRows * 2 * 4;
    // bytes of LDS one wave needs with nbuf steps in flight
    static constexpr int wave_bytes(int nbuf) {
        const int w = (nbuf * stepBytes + vscBytes + 15) / 16 * 16;
        return w > mergeBytes ? w : mergeBytes;
    }
    static constexpr int lds_bytes(int nbuf) { return kSplitWaves * wave_bytes(nbuf); }
};

template <int N>
__device__ __forceinline__ void wait_vmcnt_c() {
    static_assert(N >= 0, "");
    constexpr int n = N > 63 ? 63 : N;  // vmcnt is 6 bits; waiting for fewer is still correct
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory");
}

// wait until at most `outstanding` whole steps (NI instructions each) remain
template <int NI>
__device__ __forceinline__ void wait_steps(int outstanding) {
    switch (__builtin_amdgcn_readfirstlane(outstanding)) {
        case 0: wait_vmcnt_c<0>(); break;
        case 1: wait_vmcnt_c<NI>(); break;
        case 2: wait_vmcnt_c<2 * NI>(); break;
        default: wait_vmcnt_c<3 * NI>(); break;
    }
}

// ---------------------------------------------------------------- HBM -> LDS
// One step = [K rows | V rows | mask rows] for positions [n0, n0+32), copied
// as raw bytes.  GRAN = 16: 16-B pieces (quantised rows contiguous, f16 rows
// 16-B aligned); GRAN = 4: dword pieces for any ggml row stride.  Rows past N
// are clamped to N-1 (masked out later), so the LDS image never holds garbage.
// Mask rows use 16-B pieces on the fast path and 2-B pieces otherwise.
template <int KT, int VT, int D, int GRAN>
struct StepPlan {
    using C = SplitCfg<KT, VT, D>;
    static constexpr int PK = C::kBytes / GRAN;
    static constexpr int PV = C::vBytes / GRAN;
    static constexpr int NIKV = (PK + PV + kWave - 1) / kWave;
    // mask granule: LDS-DMA writes lane*4 bytes for sub-dword sizes, so the
    // generic path moves dwords (2 positions) and needs even-padded mask rows
    static constexpr int MG = GRAN == 16 ? 16 : 4;
    static constexpr int MPR = kStep * 2 / MG;           // mask pieces per row
    // all 16 mask rows are always copied (rows past the tile clamp to a valid
    // query row) so every step issues the same, compile-time instruction count
    static constexpr int PM = kRows * MPR;
    static constexpr int NIM = PM / kWave;
    static_assert(PM % kWave == 0, "");
};

template <int KT, int VT, int D, int GRAN, bool HM>
__device__ __forceinline__ void issue_step(const SplitArgs& a, const uint8_t* kbase, const uint8_t* vbase,
                                           int n0, int mrow0, uint8_t* buf, int lane) {
    using C = SplitCfg<KT, VT, D>;
    using P = StepPlan<KT, VT, D, GRAN>;
#pragma unroll
    for (int i = 0; i < P::NIKV; i++) {
        const int p = i * kWave + lane;
        const uint8_t* src;
        if (p < P::PK) {
            const int byte = p * GRAN;
            if constexpr (KT == FATTN_TYPE_F16) {
                // f16 rows: 16-B chunks XOR-swizzled by row (conflict-free ds_read_b128)
                constexpr int CPR = C::rowK / 16;
                const int row = byte / C::rowK;
                const int chunk = ((byte % C::rowK) / 16) ^ (row & (CPR - 1));
                const int rr = min(n0 + row, a.N - 1);
                src = kbase + (int64_t)rr * a.k_nb1 + chunk * 16 + (byte & 15);
            } else if constexpr (GRAN == 16) {
                src = kbase + (int64_t)n0 * C::rowK + byte;
            } else {
                const int row = byte / C::rowK;
                const int rr = min(n0 + row, a.N - 1);
                src = kbase + (int64_t)rr * a.k_nb1 + (byte % C::rowK);
            }
        } else {
            const int byte = (p - P::PK) * GRAN;
            if constexpr (VT == VT_F16T) {
                // V^T tile: D rows (one per head dim) of kStep f16; needs N % 32 == 0
                const int d = byte / (kStep * 2);
                src = vbase + (int64_t)d * a.v_nb0 + (int64_t)n0 * 2 + (byte % (kStep * 2));
            } else if constexpr (VT == FATTN_TYPE_F16) {
                constexpr int CPR = C::rowV / 16;
                const int row = byte / C::rowV;
                const int chunk = ((byte % C::rowV) / 16) ^ (((row & 7) << 1) & (CPR - 1));
                const int rr = min(n0 + row, a.N - 1);
                src = vbase + (int64_t)rr * a.v_nb1 + chunk * 16 + (byte & 15);
            } else if constexpr (GRAN == 16) {
                src = vbase + (int64_t)n0 * C::rowV + byte;
            } else {
                const int row = byte / C::rowV;
                const int rr = min(n0 + row, a.N - 1);
                src = vbase + (int64_t)rr * a.v_nb1 + (byte % C::rowV);
            }
        }
        if (p < P::PK + P::PV) {
            // the size operand must be a literal
            if constexpr (GRAN == 16) {
                __builtin_amdgcn_global_load_lds((const void*)src, (void*)(buf + i * kWave * 16), 16, 0, 0);
            } else {
                __builtin_amdgcn_global_load_lds((const void*)src, (void*)(buf + i * kWave * 4), 4, 0, 0);
            }
        }
    }
    if constexpr (HM) {
        uint8_t* mbuf = buf + C::kBytes + C::vBytes;
#pragma unroll
        for (int i = 0; i < P::NIM; i++) {
            const int q = i * kWave + lane;
            const int mr = q / P::MPR;
            const int off = (q % P::MPR) * P::MG;
            const int qrow = min(mrow0 + mr, a.NQ - 1);
            int pos = n0 + off / 2;
            if constexpr (P::MG == 4) pos = min(pos, (a.N - 1) & ~1);  // rows padded to even length
            const uint8_t* src = a.mask + (int64_t)qrow * a.m_nb1 + (int64_t)pos * 2;
            if constexpr (P::MG == 16) {
                __builtin_amdgcn_global_load_lds((const void*)src, (void*)(mbuf + i * kWave * 16), 16, 0, 0);
            } else {
                __builtin_amdgcn_global_load_lds((const void*)src, (void*)(mbuf + i * kWave * 4), 4, 0, 0);
            }
        }
    }
}

// ---------------------------------------------------------------- block scales
// The f16 scale of block b of a raw ggml row sits at byte BB*b.  row_scales()
// fetches the dwords holding all of a row's scales (2 x ds_read2_b32 for 4
// blocks); scale_bits() extracts block b's 16 bits.
template <int T, int D>
struct RowScales {
    uint32_t w[D / QK];
};
template <int T, int D>
__device__ __forceinline__ RowScales<T, D> row_scales(const uint8_t* row) {
    constexpr int BB = TypeInfo<T>::block_bytes;
    RowScales<T, D> s;
#pragma unroll
    for (int b = 0; b < D / QK; b++) s.w[b] = *(const uint32_t*)(row + ((BB * b) & ~3));
    return s;
}
template <int T, int D>
__device__ __forceinline__ uint32_t scale_bits(const RowScales<T, D>& s, int b) {
    constexpr int BB = TypeInfo<T>::block_bytes;
    return ((BB * b) & 2) ? (s.w[b] >> 16) : (s.w[b] & 0xffffu);
}
// f16 pair {scale of row r0, scale of row r1} for block b
template <int T, int D>
__device__ __forceinline__ f16x2 scale_pair(const RowScales<T, D>& s0, const RowScales<T, D>& s1, int b) {
    constexpr int BB = TypeInfo<T>::block_bytes;
    // v_perm: low half from s0.w[b], high half from s1.w[b]
    return as_h2(((BB * b) & 2) ? perm_b32(s1.w[b], s0.w[b], 0x07060302u) : perm_b32(s1.w[b], s0.w[b], 0x05040100u));
}

// ---------------------------------------------------------------- operands
// K operand (A of S^T = K.Q^T) for tile t (16 rows), block/k-step b:
// lane l -> row 16t + (l&15), elements d = 32b + 8(l>>4) + j.
template <int KT, int D>
__device__ __forceinline__ f16x8 k_operand(const uint8_t* kb, int row, int g, int b, uint32_t dbits) {
    if constexpr (KT == FATTN_TYPE_F16) {
        constexpr int CPR = D * 2 / 16;
        const int chunk = (4 * b + g) ^ (row & (CPR - 1));
        return *(const f16x8*)(kb + row * (D * 2) + chunk * 16);
    } else if constexpr (KT == FATTN_TYPE_Q8_0) {
        constexpr int RB = row_bytes<KT, D>();
        const uint32_t base = row * RB + kQ8Bytes * b;
        u32x2 raw;
        switch ((kQ8Bytes * b + 2) & 7) {  // b is a compile-time constant after unrolling
            case 0: raw = read8_at<0>(kb, base + 2 + 8 * g); break;
            case 2: raw = read8_at<2>(kb, base + 2 + 8 * g); break;
            case 4: raw = read8_at<4>(kb, base + 2 + 8 * g); break;
            default: raw = read8_at<6>(kb, base + 2 + 8 * g); break;
        }
        const f16x2 d = bcast_h(dbits);
        f16x2 h0, h1, h2, h3;
        i8x4_to_h2x2(raw.x, h0, h1);
        i8x4_to_h2x2(raw.y, h2, h3);
        h0 *= d; h1 *= d; h2 *= d; h3 *= d;
        f16x8 r;
        r.s01 = h0; r.s23 = h1; r.s45 = h2; r.s67 = h3;
        return r;
    } else {  // Q4_0
        constexpr int RB = row_bytes<KT, D>();
        const uint32_t base = row * RB + kQ4Bytes * b;
        u32x2 raw;
        switch ((kQ4Bytes * b + 2) & 7) {
            case 0: raw = read8_at<0>(kb, base + 2 + 8 * (g & 1)); break;
            case 2: raw = read8_at<2>(kb, base + 2 + 8 * (g & 1)); break;
            case 4: raw = read8_at<4>(kb, base + 2 + 8 * (g & 1)); break;
            default: raw = read8_at<6>(kb, base + 2 + 8 * (g & 1)); break;
        }
        const uint32_t sh = (g >> 1) * 4;
        const f16x2 d = bcast_h(dbits);
        f16x2 h0, h1, h2, h3;
        u4x4_to_h2x2((raw.x >> sh) & 0x0F0F0F0Fu, h0, h1);
        u4x4_to_h2x2((raw.y >> sh) & 0x0F0F0F0Fu, h2, h3);
        h0 *= d; h1 *= d; h2 *= d; h3 *= d;
        f16x8 r;
        r.s01 = h0; r.s23 = h1; r.s45 = h2; r.s67 = h3;
        return r;
    }
}

// V operand (A of O^T = V^T.P^T) for column group c (16 columns):
// lane l -> column dc = 16c + (l&15); element j = 4t + r <-> row 16t + 4g + r.
// For quantised V the per-(row, block) scales come from the compact array
// vsc[b][row] (f16) built once per step.
__device__ __forceinline__ uint32_t lds_u8_pair(const uint8_t* p0, const uint8_t* p1) {
    return (uint32_t)(*p0) | ((uint32_t)(*p1) << 16);
}

template <int VT, int D>
__device__ __forceinline__ f16x8 v_operand_f16(const uint8_t* vb, int c, int g, int i) {
    if constexpr (VT == VT_F16T) {
        const uint8_t* p = vb + (16 * c + i) * (kStep * 2) + 8 * g;
        const u32x2 lo = *(const u32x2*)p;
        const u32x2 hi = *(const u32x2*)(p + 32);
        u32x4 r = {lo.x, lo.y, hi.x, hi.y};
        return __builtin_bit_cast(f16x8, r);
    } else {
        constexpr int RB = D * 2;
        constexpr int CPR = RB / 16;
        const int q = i >> 2, p = i & 3;
        const int chunk = 2 * c + (p >> 1);
        const int r0 = 4 * g + q, r1 = 16 + 4 * g + q;
        const int a0 = r0 * RB + ((chunk ^ (((r0 & 7) << 1) & (CPR - 1))) * 16) + (p & 1) * 8;
        const int a1 = r1 * RB + ((chunk ^ (((r1 & 7) << 1) & (CPR - 1))) * 16) + (p & 1) * 8;
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + a0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + a1));
        u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
        u32x4 r = {l2.x, l2.y, h2.x, h2.y};
        return __builtin_bit_cast(f16x8, r);
    }
}

// ---------------------------------------------------------------- tile geometry
// A tile packs rows m = (query row m / R, head m % R).  No runtime integer
// division (hipcc expands those into long scalar loops).
__device__ __forceinline__ int div_R(const SplitArgs& a, int m) { return (int)(((float)m + 0.5f) * a.R_inv); }

// number of valid rows of tile (qt, hs); they form a prefix [0, rv)
__device__ __forceinline__ int tile_rows(const SplitArgs& a, int qt, int hs) {
    const int rows_q = min(a.QPT, a.NQ - qt * a.QPT);
    const int heads = min(a.R, a.rk2 - hs * a.R);
    return rows_q * heads;  // heads < R only when R == 16 (then QPT == 1)
}

// ---------------------------------------------------------------- diagnostics
// Diagnostic build only (-DFATTN_STAMPS, libfattn_stamps.so): lane 0 of every
// wave records s_memrealtime (100 MHz) at phase boundaries into g_stamps
// [block][wave][8].  No stamp executes in the product library.
#ifdef FATTN_STAMPS
__device__ unsigned long long* g_stamps;
#define FATTN_STAMP(k)                                                                          \
    do {                                                                                        \
        if (lane == 0 && g_stamps) {                                                            \
            const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                     \
            const int64_t blk_ = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x; \
            g_stamps[(blk_ * kSplitWaves + wave) * 8 + (k)] = t_;                                \
        }                                                                                       \
    } while (0)
#else
#define FATTN_STAMP(k) do { } while (0)
#endif

// ---------------------------------------------------------------- kernel

template <int KT, int VT, int D, int GRAN, bool HM>
__global__ __launch_bounds__(kSplitWaves * kWave, (KT == FATTN_TYPE_F16 || GRAN == 4) ? 2 : 4) void fattn_split_kernel(
    const SplitArgs a) {
    using C = SplitCfg<KT, VT, D>;
    using P = StepPlan<KT, VT, D, GRAN>;
    constexpr int NI = P::NIKV + (HM ? P::NIM : 0);  // VMEM instructions per step
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NB = D / QK;   // 32-wide k-steps of QK^T (= ggml blocks per row)
    constexpr int NC = D / 16;   // 16-wide output column groups (MFMA tiles of O^T)
    constexpr float kNegInf = -__builtin_inff();
    constexpr bool kVQ8 = C::VTT == FATTN_TYPE_Q8_0;

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g = lane >> 4;
    const int i16 = lane & 15;
    FATTN_STAMP(0);

    // ---- tile decode: y -> (kv head, head subgroup, query-row tile)
    const int chunk = blockIdx.x;
    const int y = blockIdx.y;
    const int iq3 = blockIdx.z;
    int qt = 0, hs = 0, ik2 = y, ik3 = iq3;  // common case without runtime division
    if (a.n_qt != 1 || a.n_hsub != 1) {
        qt = y % a.n_qt;
        hs = (y / a.n_qt) % a.n_hsub;
        ik2 = y / (a.n_qt * a.n_hsub);
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;

    // this lane's MFMA column m = i16 -> (query row, q head)
    const int m = i16;
    const int mq = div_R(a, m);
    const int mh = hs * a.R + (m - mq * a.R);
    const int iq1 = qt * a.QPT + mq;
    const int iq2 = ik2 * a.rk2 + mh;
    const bool row_ok = (m < a.QPT * a.R) && (iq1 < a.NQ) && (mh < a.rk2);

    // ---- this wave's KV slice
    const int wl = a.chunk_len / kSplitWaves;
    const int c_hi = min(a.N, (chunk + 1) * a.chunk_len);
    const int w_lo = chunk * a.chunk_len + wave * wl;
    const int w_hi = min(c_hi, w_lo + wl);
    const int nsteps = w_hi > w_lo ? (w_hi - w_lo + kStep - 1) / kStep : 0;
    const int nbuf = a.nbuf;

    const uint8_t* kbase = a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3;
    const uint8_t* vbase = a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3;
    uint8_t* wbuf = smem + wave * a.wave_bytes;
    const int mrow0 = qt * a.QPT;

    for (int s = 0; s < nbuf && s < nsteps; s++) {
        issue_step<KT, VT, D, GRAN, HM>(a, kbase, vbase, w_lo + s * kStep, mrow0, wbuf + s * C::stepBytes, lane);
    }

    FATTN_STAMP(1);
    // ---- Q^T operand (B of S^T = K.Q^T), rounded to f16 like src/utils.h:10
    f16x8 qop[NB];
    {
        const float* qrow = (const float*)(a.q + (int64_t)(row_ok ? iq1 : 0) * a.q_nb1 +
                                           (int64_t)(row_ok ? iq2 : 0) * a.q_nb2 + (int64_t)iq3 * a.q_nb3);
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const f32x4 x0 = *(const f32x4*)(qrow + 32 * b + 8 * g);
            const f32x4 x1 = *(const f32x4*)(qrow + 32 * b + 8 * g + 4);
            f16x8 h;
            h.s0 = (f16)x0.x; h.s1 = (f16)x0.y; h.s2 = (f16)x0.z; h.s3 = (f16)x0.w;
            h.s4 = (f16)x1.x; h.s5 = (f16)x1.y; h.s6 = (f16)x1.z; h.s7 = (f16)x1.w;
            const f16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
            qop[b] = row_ok ? h : z;
        }
    }
    // Q is loaded after the first steps' LDS-DMA is in flight, so the HBM stream
    // starts at once; waiting for Q (the youngest loads) retires those steps too
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    float m_run = kNegInf;  // running max (log2 domain) of column m
    float l_run = 0.0f;     // this lane's partial row sum
    f32x4 o[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) o[c] = f32x4{0, 0, 0, 0};

    const float log2e = 1.4426950408889634f;
    int cur = 0;  // buffer of step s
    for (int s = 0; s < nsteps; s++) {
        wait_steps<NI>(min(nbuf - 1, nsteps - 1 - s));
        if (s == 0) FATTN_STAMP(2);
#ifdef FATTN_DIAG_NOCOMPUTE
        // diagnostic build only: memory-side ceiling of this access pattern
        if (s + nbuf < nsteps) {
            issue_step<KT, VT, D, GRAN, HM>(a, kbase, vbase, w_lo + (s + nbuf) * kStep, mrow0,
                                            wbuf + cur * C::stepBytes, lane);
        }
        cur = (cur + 1 == nbuf) ? 0 : cur + 1;
        continue;
#endif
        const uint8_t* buf = wbuf + cur * C::stepBytes;
        const uint8_t* kb = buf;
        const uint8_t* vb = buf + C::kBytes;
        const uint8_t* mb = buf + C::kBytes + C::vBytes;
        const int n0 = w_lo + s * kStep;
        const int nvalid = min(kStep, w_hi - n0);

        // -- S^T = K.Q^T for the two 16-row tiles
        f32x4 st[2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
            st[t] = f32x4{0, 0, 0, 0};
            if constexpr (KT == FATTN_TYPE_F16) {
#pragma unroll
                for (int b = 0; b < NB; b++) st[t] = mfma16(k_operand<KT, D>(kb, 16 * t + i16, g, b, 0), qop[b], st[t]);
            } else {
                const RowScales<KT, D> ks = row_scales<KT, D>(kb + (16 * t + i16) * C::rowK);
#pragma unroll
                for (int b = 0; b < NB; b++)
                    st[t] = mfma16(k_operand<KT, D>(kb, 16 * t + i16, g, b, scale_bits(ks, b)), qop[b], st[t]);
            }
        }

        // -- scale + mask (log2 domain); positions past this wave's slice -> -inf
        float sv[8];
#pragma unroll
        for (int t = 0; t < 2; t++) {
            float mk[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (HM) {
                const uint8_t* mp = mb + (mq < a.QPT ? mq : 0) * (kStep * 2) + (16 * t + 4 * g) * 2;
                const u32x2 mw = *(const u32x2*)mp;
                const f16x2 m01 = as_h2(mw.x), m23 = as_h2(mw.y);
                mk[0] = (float)m01.x; mk[1] = (float)m01.y; mk[2] = (float)m23.x; mk[3] = (float)m23.y;
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float x = st[t][r] * a.scale_log2 + mk[r] * log2e;
                sv[4 * t + r] = (16 * t + 4 * g + r) < nvalid ? x : kNegInf;
            }
        }

        // -- online softmax for column m (the 4 lanes l, l^16, l^32, l^48 share it)
        float tmax = fmaxf(fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3])),
                           fmaxf(fmaxf(sv[4], sv[5]), fmaxf(sv[6], sv[7])));
        tmax = grp4_max(tmax);
        const float m_new = fmaxf(m_run, tmax);
        const float m_use = (m_new == kNegInf) ? 0.0f : m_new;
        if (__builtin_amdgcn_ballot_w64(m_new != m_run)) {  // rescale only when a max moved
            const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
            l_run *= alpha;
#pragma unroll
            for (int c = 0; c < NC; c++) o[c] *= alpha;
        }
        m_run = m_new;
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; j++) pv[j] = __builtin_amdgcn_exp2f(sv[j] - m_use);
        l_run += ((pv[0] + pv[1]) + (pv[2] + pv[3])) + ((pv[4] + pv[5]) + (pv[6] + pv[7]));

        f16x8 pb;
        pb.s0 = (f16)pv[0]; pb.s1 = (f16)pv[1]; pb.s2 = (f16)pv[2]; pb.s3 = (f16)pv[3];
        pb.s4 = (f16)pv[4]; pb.s5 = (f16)pv[5]; pb.s6 = (f16)pv[6]; pb.s7 = (f16)pv[7];

        // -- O^T += V^T.P^T
        if constexpr (C::VTT == FATTN_TYPE_F16) {
#pragma unroll
            for (int c = 0; c < NC; c++) o[c] = mfma16(v_operand_f16<VT, D>(vb, c, g, i16), pb, o[c]);
        } else {
            const int rA = 4 * g, rB = 16 + 4 * g;
            // scales of this lane's 8 rows (4g..4g+3, 16+4g..16+4g+3), all blocks
            RowScales<C::VTT, D> vs[8];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                vs[r] = row_scales<C::VTT, D>(vb + (rA + r) * C::rowV);
                vs[4 + r] = row_scales<C::VTT, D>(vb + (rB + r) * C::rowV);
            }
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const f16x2 d01 = scale_pair(vs[0], vs[1], b), d23 = scale_pair(vs[2], vs[3], b);
                const f16x2 d45 = scale_pair(vs[4], vs[5], b), d67 = scale_pair(vs[6], vs[7], b);
                constexpr int BB = TypeInfo<C::VTT>::block_bytes;
                if constexpr (kVQ8) {
                    // one u16 per row carries columns 2i (-> tile E_b) and 2i+1 (-> tile O_b)
                    const uint8_t* cp = vb + b * BB + 2 + 2 * i16;
                    uint32_t w[8];
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        w[r] = *(const uint16_t*)(cp + (rA + r) * C::rowV);
                        w[4 + r] = *(const uint16_t*)(cp + (rB + r) * C::rowV);
                    }
                    f16x8 ae, ao;
                    const f16x2 off = {(f16)-1152.0f, (f16)-1152.0f};
                    const f16x2 dd[4] = {d01, d23, d45, d67};
#pragma unroll
                    for (int pr = 0; pr < 4; pr++) {
                        // bytes [e_r, o_r, e_r+1, o_r+1] -> xor 0x80 -> f16 magic 0x64xx
                        const uint32_t t2 = (w[2 * pr] | (w[2 * pr + 1] << 16)) ^ 0x80808080u;
                        const f16x2 ve = (as_h2(perm_b32(0x64646464u, t2, 0x04020400u)) + off) * dd[pr];
                        const f16x2 vo = (as_h2(perm_b32(0x64646464u, t2, 0x04030401u)) + off) * dd[pr];
                        ae[2 * pr] = ve.x; ae[2 * pr + 1] = ve.y;
                        ao[2 * pr] = vo.x; ao[2 * pr + 1] = vo.y;
                    }
                    o[2 * b] = mfma16(ae, pb, o[2 * b]);
                    o[2 * b + 1] = mfma16(ao, pb, o[2 * b + 1]);
                } else {  // Q4_0: byte i carries column i (low nibble) and 16+i (high nibble)
                    const uint8_t* cp = vb + b * BB + 2 + i16;
                    uint32_t w[8];
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        w[r] = cp[(rA + r) * C::rowV];
                        w[4 + r] = cp[(rB + r) * C::rowV];
                    }
                    f16x8 al, ah;
                    const f16x2 off = {(f16)-1032.0f, (f16)-1032.0f};
                    const f16x2 dd[4] = {d01, d23, d45, d67};
#pragma unroll
                    for (int pr = 0; pr < 4; pr++) {
                        const uint32_t x = w[2 * pr] | (w[2 * pr + 1] << 16);
                        const f16x2 vl = (as_h2((x & 0x000F000Fu) | 0x64006400u) + off) * dd[pr];
                        const f16x2 vh = (as_h2(((x >> 4) & 0x000F000Fu) | 0x64006400u) + off) * dd[pr];
                        al[2 * pr] = vl.x; al[2 * pr + 1] = vl.y;
                        ah[2 * pr] = vh.x; ah[2 * pr + 1] = vh.y;
                    }
                    o[2 * b] = mfma16(al, pb, o[2 * b]);
                    o[2 * b + 1] = mfma16(ah, pb, o[2 * b + 1]);
                }
            }
        }

        // -- refill this buffer with step s + nbuf
        if (s + nbuf < nsteps) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            issue_step<KT, VT, D, GRAN, HM>(a, kbase, vbase, w_lo + (s + nbuf) * kStep, mrow0,
                                            wbuf + cur * C::stepBytes, lane);
        }
        cur = (cur + 1 == nbuf) ? 0 : cur + 1;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    FATTN_STAMP(3);

    // ---- per-wave state -> LDS (this wave's own region), then merge the 4 waves
    const float l_tot = grp4_sum(l_run);
    constexpr int MS = C::kMergeStride;
    float* mo = (float*)wbuf;                      // [16][MS]
    float* mml = (float*)(wbuf + kRows * MS * 4);  // [16][2]
    if constexpr (kVQ8) {
        // tile E_b holds columns 32b + 2(4g+reg), O_b the odd neighbours
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const f32x4 e = o[2 * b], od = o[2 * b + 1];
            *(f32x4*)(mo + m * MS + 32 * b + 8 * g) = f32x4{e.x, od.x, e.y, od.y};
            *(f32x4*)(mo + m * MS + 32 * b + 8 * g + 4) = f32x4{e.z, od.z, e.w, od.w};
        }
    } else {
#pragma unroll
        for (int c = 0; c < NC; c++) *(f32x4*)(mo + m * MS + 16 * c + 4 * g) = o[c];
    }
    if (g == 0) {
        mml[2 * m] = m_run;
        mml[2 * m + 1] = l_tot;
    }
    __syncthreads();
    FATTN_STAMP(4);

    constexpr int EPT = D / 16;  // outputs per thread: 16 rows x D over 256 threads
    const int tm = threadIdx.x / 16;
    const int tj = threadIdx.x % 16;
    const int d0 = tj * EPT;
    float M = kNegInf;
    float mw[kSplitWaves], lw[kSplitWaves];
#pragma unroll
    for (int w = 0; w < kSplitWaves; w++) {
        const float* ml = (const float*)(smem + w * a.wave_bytes + kRows * MS * 4);
        mw[w] = ml[2 * tm];
        lw[w] = ml[2 * tm + 1];
        M = fmaxf(M, mw[w]);
    }
    float L = 0.0f;
    float acc[EPT];
#pragma unroll
    for (int e = 0; e < EPT; e++) acc[e] = 0.0f;
#pragma unroll
    for (int w = 0; w < kSplitWaves; w++) {
        const float wt = (mw[w] == kNegInf) ? 0.0f : __builtin_amdgcn_exp2f(mw[w] - M);
        L += wt * lw[w];
        const float* ow = (const float*)(smem + w * a.wave_bytes) + tm * MS + d0;
#pragma unroll
        for (int e = 0; e < EPT; e++) acc[e] += wt * ow[e];
    }

    // valid rows of this tile form a prefix [0, rv)
    const int rv = tile_rows(a, qt, hs);
    auto dst_row = [&](int r) -> float* {
        const int rq = div_R(a, r);
        const int riq1 = qt * a.QPT + rq;
        const int riq2 = ik2 * a.rk2 + hs * a.R + (r - rq * a.R);
        return a.dst + (((int64_t)iq3 * a.NQ + riq1) * a.H + riq2) * D;
    };
    if (a.n_chunks == 1) {
        if (tm < rv) {
            float* out = dst_row(tm) + d0;
            const float inv = 1.0f / L;  // L == 0 (row fully masked) -> NaN like the reference
#pragma unroll
            for (int e = 0; e < EPT; e += 4) {
                f32x4 v;
                v.x = L == 0.0f ? __builtin_nanf("") : acc[e] * inv;
                v.y = L == 0.0f ? __builtin_nanf("") : acc[e + 1] * inv;
                v.z = L == 0.0f ? __builtin_nanf("") : acc[e + 2] * inv;
                v.w = L == 0.0f ? __builtin_nanf("") : acc[e + 3] * inv;
                *(f32x4*)(out + e) = v;
            }
        }
        return;
    }

    // ---- several chunks: plain stores of this chunk's partial; fattn_combine_kernel
    // (next launch on the stream) merges them -- the kernel boundary publishes.
    if (tm < rv) {
        const int64_t slot = (((int64_t)iq3 * gridDim.y + y) * a.n_chunks + chunk) * kRows + tm;
#pragma unroll
        for (int e = 0; e < EPT; e += 4) *(f32x4*)(a.ws_o + slot * D + d0 + e) = f32x4{acc[e], acc[e + 1], acc[e + 2], acc[e + 3]};
        if (tj == 0) *(float2*)(a.ws_ml + 2 * slot) = float2{M, L};
    }
    FATTN_STAMP(5);
}

// ---------------------------------------------------------------- combine
// Log-sum-exp merge of the chunk partials (fa_reduce, flash_row_float.h:415-472,
// in fp32 and parallel).  One workgroup per (y, z) tile; only its rv valid rows.
// 16 thread groups = rv rows x G chunk subsets; every thread issues all of its
// loads (O partials + (m, l) pairs) before consuming any: one memory round trip.
template <int D>
__global__ __launch_bounds__(256) void fattn_combine_kernel(const SplitArgs a) {
    constexpr float kNegInf = -__builtin_inff();
    constexpr int EPT = D / 16;
    constexpr int MAXC = 64 / EPT * 2;  // max chunks one thread folds (register budget)
    __shared__ float red[kRows][D];
    __shared__ float wts[kRows][64];
    __shared__ float rowML[kRows][2];
    const int y = blockIdx.x, iq3 = blockIdx.y;
    int qt = 0, hs = 0, ik2 = y;
    if (a.n_qt != 1 || a.n_hsub != 1) {
        qt = y % a.n_qt;
        hs = (y / a.n_qt) % a.n_hsub;
        ik2 = y / (a.n_qt * a.n_hsub);
    }
    const int rv = tile_rows(a, qt, hs);
    const int NCH = a.n_chunks;
    const int G = max(1, kRows / max(rv, 1));
    const int grp = threadIdx.x / 16, tj = threadIdx.x % 16, d0 = tj * EPT;
    const int64_t sb = ((int64_t)iq3 * gridDim.x + y) * NCH;
    // (1) issue every load first
    float v[MAXC][EPT];
    const int r = grp / G, cg = grp % G;
    const bool active = grp < rv * G;
    // loads are unconditional (chunk index clamped, weight zeroed below): a
    // guarded load would make hipcc branch + wait vmcnt(0) per load
    const int kmax = active ? (NCH - cg + G - 1) / G : 0;
    {
        const int rr = active ? r : 0;
#pragma unroll
        for (int k = 0; k < MAXC; k++) {
            const int c = min(cg + k * G, NCH - 1);
            const float* wo = a.ws_o + ((sb + c) * kRows + rr) * D + d0;
#pragma unroll
            for (int e = 0; e < EPT; e += 4) {
                const f32x4 x = *(const f32x4*)(wo + e);
                v[k][e] = x.x; v[k][e + 1] = x.y; v[k][e + 2] = x.z; v[k][e + 3] = x.w;
            }
        }
    }
    // (2) (m, l) of chunk c of row r lives in thread r * NCP + c (NCP = next
    // power of two >= NCH, <= 64): segmented xor-reductions inside one wave give
    // each row's max and normaliser in a fixed order (deterministic).
    const int NCP = a.ncp;
    const int mr = threadIdx.x / NCP, mc = threadIdx.x % NCP;
    float mv = kNegInf, lv = 0.0f;
    if (mr < rv && mc < NCH) {
        const float2 x = *(const float2*)(a.ws_ml + 2 * ((sb + mc) * kRows + mr));
        mv = x.x;
        lv = x.y;
    }
    float Mr = mv;
    for (int o = 1; o < NCP; o <<= 1) Mr = fmaxf(Mr, __shfl_xor(Mr, o, kWave));
    const float wt = (mv == kNegInf) ? 0.0f : __builtin_amdgcn_exp2f(mv - Mr);
    float Lr = wt * lv;
    for (int o = 1; o < NCP; o <<= 1) Lr += __shfl_xor(Lr, o, kWave);
    if (mr < rv) {
        wts[mr][mc] = wt;
        if (mc == 0) rowML[mr][1] = Lr;
    }
    __syncthreads();
    // (3) fold this thread's chunks
    if (active) {
        float s8[EPT];
#pragma unroll
        for (int e = 0; e < EPT; e++) s8[e] = 0.0f;
#pragma unroll
        for (int k = 0; k < MAXC; k++) {
            const float wt = k < kmax ? wts[r][min(cg + k * G, NCH - 1)] : 0.0f;
#pragma unroll
            for (int e = 0; e < EPT; e++) s8[e] += wt * v[k][e];
        }
#pragma unroll
        for (int e = 0; e < EPT; e++) red[grp][d0 + e] = s8[e];
    }
    __syncthreads();
    // (4) sum the G subsets of each row, normalise, store
    if (grp < rv) {
        const float Lr = rowML[grp][1];
        const float inv = 1.0f / Lr;
        const int rq = div_R(a, grp);
        const int riq1 = qt * a.QPT + rq;
        const int riq2 = ik2 * a.rk2 + hs * a.R + (grp - rq * a.R);
        float* out = a.dst + (((int64_t)iq3 * a.NQ + riq1) * a.H + riq2) * D + d0;
#pragma unroll
        for (int e = 0; e < EPT; e++) {
            float x = 0.0f;
            for (int k = 0; k < G; k++) x += red[grp * G + k][d0 + e];
            out[e] = (Lr == 0.0f) ? __builtin_nanf("") : x * inv;
        }
    }
}

}  // namespace fattn
