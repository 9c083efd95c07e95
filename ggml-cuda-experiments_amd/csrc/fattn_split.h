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
    int chunk_len;      // positions per workgroup (multiple of kStep*kSplitWaves)
    int n_chunks;
    float scale_log2;   // scale * log2(e)
    int has_mask;
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
    static constexpr int nbufRaw = 20480 / stepBytes;
    static constexpr int NBUF = nbufRaw < 2 ? 2 : (nbufRaw > 4 ? 4 : nbufRaw);
    static constexpr int vscBytes = (VTT == FATTN_TYPE_F16) ? 0 : kStep * (D / QK) * 2;
    static constexpr int waveBytes = (NBUF * stepBytes + vscBytes + 15) / 16 * 16;
    static constexpr int mergeBytes = kRows * (D + 2) * 4;
    static_assert(waveBytes >= mergeBytes, "merge scratch must fit in a wave's buffers");
    static constexpr int ldsBytes = kSplitWaves * waveBytes;
};

template <int N>
__device__ __forceinline__ void wait_vmcnt_c() {
    static_assert(N >= 0, "");
    constexpr int n = N > 63 ? 63 : N;  // vmcnt is 6 bits; waiting for fewer is still correct
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory");
}

// wait until at most `outstanding` whole steps (NI instructions each) remain
template <int NI, int NBUF>
__device__ __forceinline__ void wait_steps(int outstanding) {
    switch (__builtin_amdgcn_readfirstlane(outstanding)) {
        case 0: wait_vmcnt_c<0>(); break;
        case 1: wait_vmcnt_c<NI>(); break;
        case 2: if constexpr (NBUF > 2) wait_vmcnt_c<2 * NI>(); break;
        default: if constexpr (NBUF > 3) wait_vmcnt_c<3 * NI>(); break;
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

// ---------------------------------------------------------------- operands
// K operand (A of S^T = K.Q^T) for tile t (16 rows), block/k-step b:
// lane l -> row 16t + (l&15), elements d = 32b + 8(l>>4) + j.
template <int KT, int D>
__device__ __forceinline__ f16x8 k_operand(const uint8_t* kb, int row, int g, int b) {
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
        const f16x2 d = bcast_h(*(const uint16_t*)(kb + base));
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
        const f16x2 d = bcast_h(*(const uint16_t*)(kb + base));
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

// ---------------------------------------------------------------- kernel

template <int KT, int VT, int D, int GRAN, bool HM>
__global__ __launch_bounds__(kSplitWaves * kWave, 2) void fattn_split_kernel(const SplitArgs a) {
    using C = SplitCfg<KT, VT, D>;
    using P = StepPlan<KT, VT, D, GRAN>;
    constexpr int NI = P::NIKV + (HM ? P::NIM : 0);  // VMEM instructions per step
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NB = D / QK;   // 32-wide k-steps of QK^T (= ggml blocks per row)
    constexpr int NC = D / 16;   // 16-wide output column groups
    constexpr float kNegInf = -__builtin_inff();

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g = lane >> 4;
    const int i16 = lane & 15;

    // ---- tile decode: y -> (kv head, head subgroup, query-row tile)
    const int chunk = blockIdx.x;
    const int y = blockIdx.y;
    const int iq3 = blockIdx.z;
    const int qt = y % a.n_qt;
    const int hs = (y / a.n_qt) % a.n_hsub;
    const int ik2 = y / (a.n_qt * a.n_hsub);
    const int ik3 = iq3 / a.rk3;

    // this lane's MFMA column m = i16 -> (query row, q head)
    const int m = i16;
    const int mq = m / a.R;
    const int mh = hs * a.R + (m % a.R);
    const int iq1 = qt * a.QPT + mq;
    const int iq2 = ik2 * a.rk2 + mh;
    const bool row_ok = (m < a.QPT * a.R) && (iq1 < a.NQ) && (mh < a.rk2);

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
    // all ordinary global loads retire before the first LDS-DMA is issued
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- this wave's KV slice
    const int wl = a.chunk_len / kSplitWaves;
    const int c_hi = min(a.N, (chunk + 1) * a.chunk_len);
    const int w_lo = chunk * a.chunk_len + wave * wl;
    const int w_hi = min(c_hi, w_lo + wl);
    const int nsteps = w_hi > w_lo ? (w_hi - w_lo + kStep - 1) / kStep : 0;

    const uint8_t* kbase = a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3;
    const uint8_t* vbase = a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3;
    uint8_t* wbuf = smem + wave * C::waveBytes;
    uint8_t* vsc = wbuf + C::NBUF * C::stepBytes;
    const int mrow0 = qt * a.QPT;

    for (int s = 0; s < C::NBUF && s < nsteps; s++) {
        issue_step<KT, VT, D, GRAN, HM>(a, kbase, vbase, w_lo + s * kStep, mrow0, wbuf + s * C::stepBytes, lane);
    }

    float m_run = kNegInf;  // running max (log2 domain) of column m
    float l_run = 0.0f;     // this lane's partial row sum
    f32x4 o[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) o[c] = f32x4{0, 0, 0, 0};

    const float log2e = 1.4426950408889634f;
    for (int s = 0; s < nsteps; s++) {
        wait_steps<NI, C::NBUF>(min(C::NBUF - 1, nsteps - 1 - s));
        const uint8_t* buf = wbuf + (s % C::NBUF) * C::stepBytes;
        const uint8_t* kb = buf;
        const uint8_t* vb = buf + C::kBytes;
        const uint8_t* mb = buf + C::kBytes + C::vBytes;
        const int n0 = w_lo + s * kStep;
        const int nvalid = min(kStep, w_hi - n0);

        // -- V scales -> compact [b][row] f16 array (quantised V only)
        if constexpr (C::vscBytes > 0) {
            constexpr int E = kStep * NB;
#pragma unroll
            for (int e0 = 0; e0 < E; e0 += kWave) {
                const int e = e0 + lane;
                if (e < E) {
                    const int row = e % kStep, b = e / kStep;
                    const uint16_t sc = *(const uint16_t*)(vb + row * C::rowV + b * TypeInfo<C::VTT>::block_bytes);
                    *(uint16_t*)(vsc + (b * kStep + row) * 2) = sc;
                }
            }
        }

        // -- S^T = K.Q^T for the two 16-row tiles
        f32x4 st[2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
            st[t] = f32x4{0, 0, 0, 0};
#pragma unroll
            for (int b = 0; b < NB; b++) st[t] = mfma16(k_operand<KT, D>(kb, 16 * t + i16, g, b), qop[b], st[t]);
        }

        // -- scale + mask (log2 domain), tail positions -> -inf
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
                const int pos = 16 * t + 4 * g + r;
                const float x = st[t][r] * a.scale_log2 + mk[r] * log2e;
                sv[4 * t + r] = pos < nvalid ? x : kNegInf;
            }
        }

        // -- online softmax for column m (4 lanes share it)
        float tmax = sv[0];
#pragma unroll
        for (int j = 1; j < 8; j++) tmax = fmaxf(tmax, sv[j]);
        tmax = grp4_max(tmax);
        const float m_new = fmaxf(m_run, tmax);
        const float m_use = (m_new == kNegInf) ? 0.0f : m_new;
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
        m_run = m_new;
        float psum = 0.0f;
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            pv[j] = __builtin_amdgcn_exp2f(sv[j] - m_use);
            psum += pv[j];
        }
        l_run = l_run * alpha + psum;
#pragma unroll
        for (int c = 0; c < NC; c++) o[c] *= alpha;

        f16x8 pb;
        pb.s0 = (f16)pv[0]; pb.s1 = (f16)pv[1]; pb.s2 = (f16)pv[2]; pb.s3 = (f16)pv[3];
        pb.s4 = (f16)pv[4]; pb.s5 = (f16)pv[5]; pb.s6 = (f16)pv[6]; pb.s7 = (f16)pv[7];

        // -- O^T += V^T.P^T
        if constexpr (C::VTT == FATTN_TYPE_F16) {
#pragma unroll
            for (int c = 0; c < NC; c++) o[c] = mfma16(v_operand_f16<VT, D>(vb, c, g, i16), pb, o[c]);
        } else {
            const bool tail = nvalid < kStep;
#pragma unroll
            for (int b = 0; b < NB; b++) {
                // scales of rows 4g..4g+3 and 16+4g..16+4g+3 for block b
                const u32x2 s0 = *(const u32x2*)(vsc + (b * kStep + 4 * g) * 2);
                const u32x2 s1 = *(const u32x2*)(vsc + (b * kStep + 16 + 4 * g) * 2);
                const f16x2 d01 = as_h2(s0.x), d23 = as_h2(s0.y), d45 = as_h2(s1.x), d67 = as_h2(s1.y);
                constexpr int BB = TypeInfo<C::VTT>::block_bytes;
                const uint8_t* col = vb + b * BB + 2;
                const int rA = 4 * g, rB = 16 + 4 * g;
                if constexpr (C::VTT == FATTN_TYPE_Q8_0) {
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint8_t* cp = col + 16 * h + i16;
                        uint32_t x0 = lds_u8_pair(cp + (rA + 0) * C::rowV, cp + (rA + 1) * C::rowV);
                        uint32_t x1 = lds_u8_pair(cp + (rA + 2) * C::rowV, cp + (rA + 3) * C::rowV);
                        uint32_t x2 = lds_u8_pair(cp + (rB + 0) * C::rowV, cp + (rB + 1) * C::rowV);
                        uint32_t x3 = lds_u8_pair(cp + (rB + 2) * C::rowV, cp + (rB + 3) * C::rowV);
                        const f16x2 off = {(f16)-1152.0f, (f16)-1152.0f};
                        f16x2 v0 = (as_h2(x0 ^ 0x64806480u) + off) * d01;
                        f16x2 v1 = (as_h2(x1 ^ 0x64806480u) + off) * d23;
                        f16x2 v2 = (as_h2(x2 ^ 0x64806480u) + off) * d45;
                        f16x2 v3 = (as_h2(x3 ^ 0x64806480u) + off) * d67;
                        if (tail) {
                            const f16x2 z = {0, 0};
                            v0 = (rA + 1 < nvalid) ? v0 : ((rA < nvalid) ? f16x2{v0.x, 0} : z);
                            v1 = (rA + 3 < nvalid) ? v1 : ((rA + 2 < nvalid) ? f16x2{v1.x, 0} : z);
                            v2 = (rB + 1 < nvalid) ? v2 : ((rB < nvalid) ? f16x2{v2.x, 0} : z);
                            v3 = (rB + 3 < nvalid) ? v3 : ((rB + 2 < nvalid) ? f16x2{v3.x, 0} : z);
                        }
                        f16x8 av;
                        av.s01 = v0; av.s23 = v1; av.s45 = v2; av.s67 = v3;
                        o[2 * b + h] = mfma16(av, pb, o[2 * b + h]);
                    }
                } else {  // Q4_0: both nibbles of one byte feed column groups 2b and 2b+1
                    const uint8_t* cp = col + i16;
                    const uint32_t x0 = lds_u8_pair(cp + (rA + 0) * C::rowV, cp + (rA + 1) * C::rowV);
                    const uint32_t x1 = lds_u8_pair(cp + (rA + 2) * C::rowV, cp + (rA + 3) * C::rowV);
                    const uint32_t x2 = lds_u8_pair(cp + (rB + 0) * C::rowV, cp + (rB + 1) * C::rowV);
                    const uint32_t x3 = lds_u8_pair(cp + (rB + 2) * C::rowV, cp + (rB + 3) * C::rowV);
                    const f16x2 off = {(f16)-1032.0f, (f16)-1032.0f};
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const int sh = 4 * h;
                        f16x2 v0 = (as_h2(((x0 >> sh) & 0x000F000Fu) | 0x64006400u) + off) * d01;
                        f16x2 v1 = (as_h2(((x1 >> sh) & 0x000F000Fu) | 0x64006400u) + off) * d23;
                        f16x2 v2 = (as_h2(((x2 >> sh) & 0x000F000Fu) | 0x64006400u) + off) * d45;
                        f16x2 v3 = (as_h2(((x3 >> sh) & 0x000F000Fu) | 0x64006400u) + off) * d67;
                        if (tail) {
                            const f16x2 z = {0, 0};
                            v0 = (rA + 1 < nvalid) ? v0 : ((rA < nvalid) ? f16x2{v0.x, 0} : z);
                            v1 = (rA + 3 < nvalid) ? v1 : ((rA + 2 < nvalid) ? f16x2{v1.x, 0} : z);
                            v2 = (rB + 1 < nvalid) ? v2 : ((rB < nvalid) ? f16x2{v2.x, 0} : z);
                            v3 = (rB + 3 < nvalid) ? v3 : ((rB + 2 < nvalid) ? f16x2{v3.x, 0} : z);
                        }
                        f16x8 av;
                        av.s01 = v0; av.s23 = v1; av.s45 = v2; av.s67 = v3;
                        o[2 * b + h] = mfma16(av, pb, o[2 * b + h]);
                    }
                }
            }
        }

        // -- refill this buffer with step s + NBUF
        if (s + C::NBUF < nsteps) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            issue_step<KT, VT, D, GRAN, HM>(a, kbase, vbase, w_lo + (s + C::NBUF) * kStep, mrow0,
                                        wbuf + (s % C::NBUF) * C::stepBytes, lane);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    // ---- per-wave state -> LDS (this wave's own buffers), then merge 4 waves
    const float l_tot = grp4_sum(l_run);
    float* mo = (float*)wbuf;                 // [16][D]
    float* mml = (float*)(wbuf + kRows * D * 4);  // [16][2]
#pragma unroll
    for (int c = 0; c < NC; c++) *(f32x4*)(mo + m * D + 16 * c + 4 * g) = o[c];
    if (g == 0) {
        mml[2 * m] = m_run;
        mml[2 * m + 1] = l_tot;
    }
    __syncthreads();

    constexpr int EPT = D / 16;  // outputs per thread: 16 rows x D over 256 threads
    const int tm = threadIdx.x / 16;
    const int d0 = (threadIdx.x % 16) * EPT;
    float M = kNegInf;
    float mw[kSplitWaves], lw[kSplitWaves];
#pragma unroll
    for (int w = 0; w < kSplitWaves; w++) {
        const float* ml = (const float*)(smem + w * C::waveBytes + kRows * D * 4);
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
        const float* ow = (const float*)(smem + w * C::waveBytes) + tm * D + d0;
#pragma unroll
        for (int e = 0; e < EPT; e++) acc[e] += wt * ow[e];
    }

    // row validity for the merged row tm
    const int tq = tm / a.R;
    const int th = hs * a.R + (tm % a.R);
    const int tiq1 = qt * a.QPT + tq;
    const int tiq2 = ik2 * a.rk2 + th;
    const bool t_ok = (tm < a.QPT * a.R) && (tiq1 < a.NQ) && (th < a.rk2);
    if (!t_ok) return;
    if (a.n_chunks == 1) {
        float* out = a.dst + (((int64_t)iq3 * a.NQ + tiq1) * a.H + tiq2) * D + d0;
        const float inv = 1.0f / L;  // L == 0 (row fully masked) -> NaN like the reference
#pragma unroll
        for (int e = 0; e < EPT; e++) out[e] = (L == 0.0f) ? __builtin_nanf("") : acc[e] * inv;
    } else {
        const int64_t slot = (((int64_t)iq3 * gridDim.y + y) * a.n_chunks + chunk) * kRows + tm;
        float* wo = a.ws_o + slot * D + d0;
#pragma unroll
        for (int e = 0; e < EPT; e++) wo[e] = acc[e];
        if (d0 == 0) {
            a.ws_ml[2 * slot] = M;
            a.ws_ml[2 * slot + 1] = L;
        }
    }
}

// ---------------------------------------------------------------- combine
// Log-sum-exp merge of the chunk partials (fa_reduce, flash_row_float.h:415-472,
// in fp32 and parallel over the head dimension instead of one serial lane).
template <int D>
__global__ __launch_bounds__(256) void fattn_combine_kernel(const SplitArgs a) {
    constexpr float kNegInf = -__builtin_inff();
    constexpr int EPT = D / 16;
    const int y = blockIdx.x;
    const int iq3 = blockIdx.y;
    const int tm = threadIdx.x / 16;
    const int d0 = (threadIdx.x % 16) * EPT;
    const int qt = y % a.n_qt;
    const int hs = (y / a.n_qt) % a.n_hsub;
    const int ik2 = y / (a.n_qt * a.n_hsub);
    const int tq = tm / a.R;
    const int th = hs * a.R + (tm % a.R);
    const int tiq1 = qt * a.QPT + tq;
    const int tiq2 = ik2 * a.rk2 + th;
    const bool t_ok = (tm < a.QPT * a.R) && (tiq1 < a.NQ) && (th < a.rk2);
    if (!t_ok) return;
    const int64_t base = ((int64_t)iq3 * gridDim.x + y) * a.n_chunks;
    float M = kNegInf;
    for (int c = 0; c < a.n_chunks; c++) M = fmaxf(M, a.ws_ml[2 * ((base + c) * kRows + tm)]);
    float L = 0.0f;
    float acc[EPT];
#pragma unroll
    for (int e = 0; e < EPT; e++) acc[e] = 0.0f;
    for (int c = 0; c < a.n_chunks; c++) {
        const int64_t slot = (base + c) * kRows + tm;
        const float mc = a.ws_ml[2 * slot];
        const float wt = (mc == kNegInf) ? 0.0f : __builtin_amdgcn_exp2f(mc - M);
        L += wt * a.ws_ml[2 * slot + 1];
        const float* wo = a.ws_o + slot * D + d0;
#pragma unroll
        for (int e = 0; e < EPT; e++) acc[e] += wt * wo[e];
    }
    float* out = a.dst + (((int64_t)iq3 * a.NQ + tiq1) * a.H + tiq2) * D + d0;
    const float inv = 1.0f / L;
#pragma unroll
    for (int e = 0; e < EPT; e++) out[e] = (L == 0.0f) ? __builtin_nanf("") : acc[e] * inv;
}

}  // namespace fattn
