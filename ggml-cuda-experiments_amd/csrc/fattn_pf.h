// fattn_pf.h -- prefill-shaped attention over ggml-quantised KV for gfx950:
// >= 256 packed query rows per kv head and enough (kv head x query tile)
// workgroups to fill the chip (n_q = N = 4096 prompt processing, the MFMA-bound
// shape of SURVEY.md §8d).
//
// Replaces flash_attn_ext_f16<D,Q,C> (src/flash-llama.h:5-438) for long query
// blocks.  Same math as the split / multi-query kernels (scale * q.k + mask,
// online softmax, P.V; f16 operands, f32 accumulation), laid out for the
// 32x32 matrix cores:
//
//  * one workgroup = 8 waves = 256 packed (query row x q-head) rows of one kv
//    head, 32 per wave; the KV sequence is walked in 64-key tiles;
//  * HBM -> LDS: the tile's raw ggml K and V rows by buffer_load ... lds (1-KiB
//    wave instructions dealt round-robin over the waves), three raw tiles in
//    flight; the workgroup dequantises each tile ONCE -- wave w takes half
//    block w of every row, K and V -- into f16 K and V images, h(q*d) with one
//    f16 rounding (src/utils.h:10-11);
//  * "swapped" products on v_mfma_f32_32x32x16_f16: S^T = K.Q^T (K rows from
//    the image by ds_read_b128, Q^T kept in registers), so a lane holds 16
//    keys of ONE query row -- the row max / sum are in-lane ops and one
//    v_permlane32_swap; then O^T = V^T.P^T where P^T is the S^T accumulator
//    itself converted to f16 (no lane movement): the 16 keys of each PV k-step
//    are taken in the accumulator's own order and V^T is gathered in the same
//    order with ds_read_b64_tr_b16 (4 keys x 16 dims per 16-lane group);
//  * each wave's 32 mask rows of a tile (4 KiB) arrive by four coalesced 1-KiB
//    LDS-DMA instructions into the wave's own LDS slot, a tile ahead;
//  * one workgroup barrier per tile: while the waves run tile s from one image
//    pair, the workgroup dequantises tile s+1 into the other and tiles s+2,
//    s+3 are in flight; the two waves of each SIMD run their phases staggered
//    (one's VALU beside the other's MFMA).
//
// LDS (D = 128), every image read address = one per-lane base + an immediate:
//   [0, 64 KiB)   two image pairs.  K image [8 dim-slices][64 keys][32 B]
//                 (16-B halves swapped on rows with bit 3 set); V image
//                 [4 dim-blocks][64 keys][64 B] (16-B chunk c of row r at
//                 c ^ ((r >> 2) & 3)).  Both read and written conflict-free.
//   then          3 raw tiles [K rows | V rows], 8 mask slots [32 rows][8 x 16 B]
//                 (16-B piece pc of row r at pc ^ ((r >> 1) & 7)).
#pragma once

#include "fattn_mq.h"
#include "fattn_quant.h"

namespace fattn {

constexpr int kPfWaves = 8;
constexpr int kPfRowsW = 32;                    // packed rows per wave
constexpr int kPfRows = kPfWaves * kPfRowsW;    // per workgroup
constexpr int kPfKeys = 64;                     // keys per tile

typedef float f32x16 __attribute__((ext_vector_type(16)));

// image dims: D = 80 (f16 K/V only) is laid out as 96 -- whole 32-dim blocks of
// O^T -- with dims 80..95 zero in Q, K and V (DMA'd from past the descriptor)
constexpr int pf_image_dims(int D) { return D == 80 ? 96 : D; }

template <int KT, int D>
struct PfCfg {
    static_assert(D == 64 || D == 80 || D == 96 || D == 128, "at most one half ggml block per wave and row");
    static_assert(D != 80 || KT == FATTN_TYPE_F16, "D = 80: f16 K/V (80 is not a whole number of ggml blocks)");
    static constexpr int DI = pf_image_dims(D);
    static constexpr int NT = kPfWaves * kWave;
    // f16 K/V: LDS-DMA straight into the images (no raw tiles, no dequantisation);
    // three image pairs: tile s in use, s+1 and s+2 in flight
    static constexpr bool kDirect = KT == FATTN_TYPE_F16;
    static constexpr int rowB = row_bytes<KT, D>();
    static constexpr int kvRaw = kPfKeys * rowB;                    // raw K (or V) bytes per tile
    static constexpr int rawBytes = (2 * kvRaw + 15) / 16 * 16;
    static constexpr int nRaw = kDirect ? 0 : 3;
    static constexpr int img = kPfKeys * DI * 2;                    // one f16 image
    static constexpr int pairBytes = 2 * img;                       // K image + V image
    static constexpr int nPairs = kDirect ? 3 : 2;
    static constexpr int ahead = kDirect ? 2 : 3;                   // tiles in flight beyond the current one
    static constexpr int rawOff = nPairs * pairBytes;
    static constexpr int maskOff = rawOff + nRaw * rawBytes;
    static constexpr int maskSlot = kPfRowsW * 128;                 // 32 rows x 64 keys x f16
    // epilogue: every wave parks its 32 normalised rows, [8 waves][32 rows][DI + 4] f32
    static constexpr int parkBytes = kPfWaves * kPfRowsW * (DI + 4) * 4;
    static constexpr int loopBytes = maskOff + kPfWaves * maskSlot;
    static constexpr int ldsBytes = loopBytes > parkBytes ? loopBytes : parkBytes;
    static constexpr int NI = (kvRaw + 1023) / 1024;                // 1-KiB DMA instructions per K (or V) tile
    // instructions j = 0 .. 2*NI-1 (K then V) go to wave j % 8
    static constexpr int ni_wave(int w) { return (2 * NI - w + kPfWaves - 1) / kPfWaves; }
    static constexpr int NIM = maskSlot / 1024;                     // mask DMA instructions per wave and tile
    static_assert(ldsBytes <= 163840, "");
};

template <int KT, int D>
__device__ __forceinline__ void pf_issue(const StepSrc& rs, int n0, uint32_t lds, int wave, int lane) {
#ifdef FATTN_MQ_NOMEM
    return;  // diagnostic build only
#endif
    using C = PfCfg<KT, D>;
    for (int j = wave; j < 2 * C::NI; j += kPfWaves) {  // wave-uniform
        const bool is_v = j >= C::NI;
        const int i = is_v ? j - C::NI : j;
        const int byte = i * 1024 + lane * 16;
        if (C::kvRaw % 1024 == 0 || byte < C::kvRaw)
            dma<16>(is_v ? rs.v : rs.k, lds + (is_v ? C::kvRaw : 0) + i * 1024, (uint32_t)n0 * C::rowB + byte);
    }
}

// f16 K/V: this lane's source offsets (tile-relative; + n0 * nb1 per tile) of
// its wave's DMA instructions j = wave + 8i, i < NIW (j < NJ: K image bytes
// [1024j, +1024); else V image bytes [1024(j-NJ), +1024); NJ = the image's
// 1-KiB pieces), laid out as the image swizzles above.  Rows are addressed by nb1
// (any 16-B aligned stride).
template <int D>
struct PfDirect {
    static constexpr int NJ = kPfKeys * pf_image_dims(D) * 2 / 1024;  // 1-KiB pieces per image (D = 80, 96: 12)
    static constexpr int NIW = 2 * NJ / kPfWaves;      // DMA instructions per wave and tile
    static_assert(kPfWaves == 8 && NIW * kPfWaves == 2 * NJ && NIW <= 4, "every wave the same count");
};
template <int D>
__device__ __forceinline__ void pf_direct_offsets(const SplitArgs& a, int wave, int lane, uint32_t (&off)[4]) {
    constexpr int NJ = PfDirect<D>::NJ;
#pragma unroll
    for (int i = 0; i < PfDirect<D>::NIW; i++) {
        const int j = wave + 8 * i;      // (wave-uniform; K pieces first)
        // (image dims past D -- D = 80 -- come from past the descriptor: zeros;
        // kPadOff stays past it after the per-tile row offset is added)
        constexpr uint32_t kPadOff = 0x80000000u;
        if (j < NJ) {  // K: slice kk = j / 2, rows 32 (j & 1) + lane / 2, stored half lane & 1
            const int kk = j >> 1, r = 32 * (j & 1) + (lane >> 1), hh = lane & 1;
            const int sh = hh ^ ((r >> 3) & 1);
            off[i] = 16 * kk + 8 * sh < D ? (uint32_t)r * (uint32_t)a.k_nb1 + kk * 32 + sh * 16 : kPadOff;
        } else {  // V: dim block db = jj / 4, rows 16 (jj & 3) + lane / 4, stored chunk lane & 3
            const int jj = j - NJ, db = jj >> 2, r = 16 * (jj & 3) + (lane >> 2), pc = lane & 3;
            const int lc = pc ^ ((r >> 2) & 3);
            off[i] = 32 * db + 8 * lc < D ? (uint32_t)r * (uint32_t)a.v_nb1 + db * 64 + lc * 16 : kPadOff;
        }
    }
}

template <int D>
__device__ __forceinline__ void pf_direct_issue(const SplitArgs& a, const StepSrc& rs, int n0, uint32_t pair_lds,
                                                int wave, const uint32_t (&off)[4]) {
#ifdef FATTN_MQ_NOMEM
    return;  // diagnostic build only
#endif
    const uint32_t nk = (uint32_t)n0 * (uint32_t)a.k_nb1, nv = (uint32_t)n0 * (uint32_t)a.v_nb1;
    constexpr int NJ = PfDirect<D>::NJ;
#pragma unroll
    for (int i = 0; i < PfDirect<D>::NIW; i++) {
        const int j = wave + 8 * i;
        if (j < NJ)
            dma<16>(rs.k, pair_lds + j * 1024, nk + off[i]);
        else
            dma<16>(rs.v, pair_lds + PfCfg<FATTN_TYPE_F16, D>::img + (j - NJ) * 1024, nv + off[i]);
    }
}

// counted wait: at most nraw (0..2) raw-tile DMA groups and nmask (0/1) mask
// groups of this wave still in flight (vmcnt counts in issue order).  Counted
// with the SMALLEST per-wave group (ni_wave of the last wave): a wave that
// issues one more instruction per tile waits for that one too -- it belongs to
// the youngest group, issued a tile earlier -- and no wave needs a switch over
// its id (the branch trees cost ~300 SALU per wave and tile)
template <int KT, int D>
__device__ __forceinline__ void pf_vm_wait(int nraw, int nmask) {
    constexpr int NI = PfCfg<KT, D>::ni_wave(kPfWaves - 1);
    constexpr int NM = PfCfg<KT, D>::NIM;
    if (nmask) {
        if (nraw >= 2) wait_vmcnt_c<2 * NI + NM>();
        else if (nraw == 1) wait_vmcnt_c<NI + NM>();
        else wait_vmcnt_c<NM>();
    } else {
        if (nraw >= 2) wait_vmcnt_c<2 * NI>();
        else if (nraw == 1) wait_vmcnt_c<NI>();
        else wait_vmcnt_c<0>();
    }
}

// raw tile -> f16 images: wave w dequantises half h = w & 1 of block b = w >> 1
// of row `lane`, for K (into dim slice 2b + h) and V (dim block b, chunks 2h, 2h+1)
// (D = 64: two blocks, waves 0-3; waves 4-7 -- the prioritised half -- skip it).
// In two steps (pf_dequant_load: the LDS reads of the raw words;
// pf_dequant_store: conversion and image writes), so an A/B build can split
// them around the S^T chains (FATTN_PF_DEQ_EARLY).
struct PfRaw {
    HalfRaw k, v;
};
template <int KT, int D>
__device__ __forceinline__ PfRaw pf_dequant_load(const uint8_t* rb, int wave, int lane) {
    using C = PfCfg<KT, D>;
    const int b = wave >> 1, h = wave & 1;
    PfRaw r;
    if (b >= D / QK) return r;  // wave-uniform (D = 64: waves 4-7 idle; r unused)
    r.k = dequant_half_load<KT, D>(rb, lane, b, h);
    r.v = dequant_half_load<KT, D>(rb + C::kvRaw, lane, b, h);
    return r;
}
template <int KT, int D>
__device__ __forceinline__ void pf_dequant_store(const PfRaw& r, uint8_t* k16, uint8_t* v16, int wave, int lane) {
#ifdef FATTN_MQ_NODEQ
    return;  // diagnostic build only
#endif
    const int b = wave >> 1, h = wave & 1;
    if (b >= D / QK) return;  // wave-uniform
    u32x4 ck[2], cv[2];
    dequant_half_cvt<KT>(r.k, h, ck);
    dequant_half_cvt<KT>(r.v, h, cv);
    uint8_t* kd = k16 + wave * (kPfKeys * 32) + lane * 32;
    const int sk = (lane >> 3) & 1;
    *(u32x4*)(kd + sk * 16) = ck[0];
    *(u32x4*)(kd + (sk ^ 1) * 16) = ck[1];
    uint8_t* vd = v16 + b * (kPfKeys * 64) + lane * 64;
    const int sv = (lane >> 2) & 3;
    *(u32x4*)(vd + ((2 * h) ^ sv) * 16) = cv[0];
    *(u32x4*)(vd + ((2 * h + 1) ^ sv) * 16) = cv[1];
}

template <int KT, int D>
__device__ __forceinline__ void pf_dequant(const uint8_t* rb, uint8_t* k16, uint8_t* v16, int wave, int lane) {
    pf_dequant_store<KT, D>(pf_dequant_load<KT, D>(rb, wave, lane), k16, v16, wave, lane);
}

__device__ __forceinline__ f32x16 mfma32(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int KT, int D, bool HM>
__global__ __launch_bounds__(kPfWaves* kWave, 1) void fattn_pf_kernel(const SplitArgs a) {
    using C = PfCfg<KT, D>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NK = C::DI / 16;   // 16-dim k-steps of S^T = K.Q^T
    constexpr int NDB = C::DI / 32;  // 32-dim blocks of O^T
    constexpr int NM = HM ? 1 : 0;
    constexpr float kNegInf = -__builtin_inff();
    constexpr float kDeferLog2 = 8.0f;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the second-dispatched half loses VALU arbitration to its SIMD partner
    // every phase; static priority evens that out (MI355X_MICROARCH.md, two
    // waves per SIMD, item 4)
    if (a.pf_stagger & 2) {
        if (wave >= kPfWaves / 2) __builtin_amdgcn_s_setprio(1);
    }
    const int h = lane >> 5;      // k-group of the MFMA operands
    const int c32 = lane & 31;    // MFMA column: this lane's packed row within the wave

    // ---- tile decode: y -> (kv head, query tile); whole head groups (R = rk2)
    int y = blockIdx.y;
    // XCD-aware order (pf_stagger bit 2): workgroups are dealt round-robin to the
    // 8 XCDs, so consecutive y -- the query tiles of one kv head -- would land
    // on 8 different L2s; remap so that each XCD takes a contiguous range of y
    // (the query tiles of a few heads share their K/V stream in one L2)
    if ((a.pf_stagger & 4) && gridDim.y % 8 == 0) y = (y & 7) * (gridDim.y >> 3) + (y >> 3);
    const int iq3 = blockIdx.z;
    int qt = 0, ik2 = y, ik3 = iq3;
    if (a.pf_flags) {
        // masked: query tiles may see different KV ranges (causal: tile qt sees
        // 4 qt + 4 of them), so the longest go first -- the last query tile of
        // every head, then the one before, ... (longest-first dispatch)
        const int nh = gridDim.y / a.n_qt;
        qt = a.n_qt - 1 - y / nh;
        ik2 = y % nh;
    } else if (a.n_qt != 1) {
        qt = y % a.n_qt;
        ik2 = y / a.n_qt;
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;
    auto row_of = [&](int p, int& iq1, int& iq2) {  // packed row -> (query row, q head)
        const int mq = div_R(a, p);
        iq1 = qt * a.QPT + mq;
        iq2 = ik2 * a.rk2 + (p - mq * a.R);
        return mq < a.QPT && iq1 < a.NQ;  // (R not a power of two: rows past QPT * R are none)
    };
    int iq1, iq2;
    const bool row_ok = row_of(kPfRowsW * wave + c32, iq1, iq2);
    // live KV tile range of this query tile: [t0, t0 + ntiles).  With a mask,
    // pf_mask_flags_kernel marked each (query tile, KV tile) block that has any
    // key above -inf; tiles outside the first..last marked one are never
    // fetched (causal prefill: about half of them).  Blocks inside the range
    // that are -inf for a whole wave are skipped below.
    int t0 = 0, ntiles = a.N / kPfKeys;
    if (a.pf_flags) {
        const uint8_t* fl = a.pf_flags + (int64_t)qt * ntiles;
        int lo = ntiles, hi = -1;
        for (int b = 0; b < ntiles; b += kWave) {  // wave-uniform; every wave computes the same range
            const bool f = b + lane < ntiles && fl[b + lane] != 0;
            const uint64_t m = __builtin_amdgcn_ballot_w64(f);
            if (m) {
                lo = min(lo, b + (int)__builtin_ctzll(m));
                hi = b + 63 - (int)__builtin_clzll(m);
            }
        }
        t0 = lo;
        ntiles = hi >= lo ? hi - lo + 1 : 0;
    }
    // live tiles whose mask block is +-0 everywhere (flag 2: the prefill of a
    // zero or causal mask, away from the diagonal): their mask DMA goes through
    // an offset past the descriptor -- no traffic, zeros land in the slot, the
    // instruction count (vmcnt budget) is unchanged -- and the tile neither
    // waits for nor reads the slot (zeros in registers instead).
    // Bit s of zb[s / 64]: tile t0 + s (the first 256 live tiles).
    uint64_t zb[4] = {0, 0, 0, 0};
    if (a.pf_flags) {
        const uint8_t* fl = a.pf_flags + (int64_t)qt * (a.N / kPfKeys) + t0;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const int b = 64 * w + lane;
            zb[w] = __builtin_amdgcn_ballot_w64(b < ntiles && fl[b] == 2);
        }
    }

    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    rs.m = make_srd(a.mask, HM ? a.m_span : 0);
    const uint32_t lds0 = lds_addr(smem);
    constexpr int kNRaw = C::nRaw ? C::nRaw : 1;
    auto raw_lds = [&](int s) { return lds0 + C::rawOff + (s % kNRaw) * C::rawBytes; };
    auto raw_ptr = [&](int s) { return smem + C::rawOff + (s % kNRaw) * C::rawBytes; };
    const uint32_t mslot = lds0 + C::maskOff + wave * C::maskSlot;

    // ---- Q^T operands (B of S^T = K.Q^T): dims 16kk + 8h .. +8 of this lane's
    // row, rounded to f16 like src/utils.h:10; rows past n_q read zeros
    f16x8 qop[NK];
    {
        const auto qs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.q + (int64_t)iq3 * a.q_nb3), 0,
                                                          a.q_span, 0x00020000);
        const uint32_t qoff =
            row_ok ? (uint32_t)iq1 * (uint32_t)a.q_nb1 + (uint32_t)iq2 * (uint32_t)a.q_nb2 + 32 * h : a.q_span;
#pragma unroll
        for (int kk = 0; kk < NK; kk++) {
            // (image dims past D, D = 80: from past the descriptor, zeros)
            const uint32_t qk = 16 * kk + 8 * h < D ? qoff + 64 * kk : a.q_span;
            const f32x4 x0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(qs, qk, 0, 0));
            const f32x4 x1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(qs, qk + 16, 0, 0));
            f16x8 hq;
            hq.s0 = (f16)x0.x; hq.s1 = (f16)x0.y; hq.s2 = (f16)x0.z; hq.s3 = (f16)x0.w;
            hq.s4 = (f16)x1.x; hq.s5 = (f16)x1.y; hq.s6 = (f16)x1.z; hq.s7 = (f16)x1.w;
            qop[kk] = hq;
        }
    }

    // ---- mask DMA: instruction k of a tile fills slot units 64k .. 64k+63;
    // lane i -> unit 64k + i = row 8k + i/8, stored piece i%8 = piece
    // (i%8) ^ ((row >> 1) & 7) of the row's 128 B (64 keys)
    uint32_t moff[C::NIM];
    if constexpr (HM) {
#pragma unroll
        for (int k = 0; k < C::NIM; k++) {
            const int rr = 8 * k + (lane >> 3);
            int q1, q2;
            const bool ok = row_of(kPfRowsW * wave + rr, q1, q2);
            const int pc = (lane & 7) ^ ((rr >> 1) & 7);
            moff[k] = ok ? (uint32_t)q1 * (uint32_t)a.m_nb1 + 16 * pc : a.m_span;
        }
    }
    // tile s's mask block is +-0 everywhere (flag 2; wave-uniform)
    auto zero_of = [&](int s) { return s < 256 && ((zb[s >> 6] >> (s & 63)) & 1); };
    // such a tile's mask DMA goes through an offset past the descriptor (no
    // traffic, the instruction count unchanged).  (FATTN_PF_ZERO_SKIP, A/B
    // builds, quantised K/V: not issued at all, the counted waits leaving its
    // group out -- Q8_0 zero mask 446-455 vs 430-453 us, causal 251 vs 245:
    // slower, profiles/r04_j)
#ifdef FATTN_PF_ZERO_SKIP
    constexpr bool kSkipZero = !C::kDirect;  // diagnostic build only
#else
    constexpr bool kSkipZero = false;
#endif
    auto mask_groups = [&](int s) { return (HM && !(kSkipZero && zero_of(s))) ? 1 : 0; };
    auto mask_issue = [&](int s) {
        if constexpr (HM) {
#ifndef FATTN_MQ_NOMEM
            const uint32_t n2 = (uint32_t)(t0 + s) * kPfKeys * 2;
            const bool zero = zero_of(s);
            if (kSkipZero && zero) return;
#pragma unroll
            for (int k = 0; k < C::NIM; k++) {
                const uint32_t off = (moff[k] == a.m_span || zero) ? a.m_span : moff[k] + n2;
                dma<16>(rs.m, mslot + k * 1024, off);
            }
#endif
        }
    };
    // this lane's mask reads: row c32, piece pc = 4t + u (keys 32t + 8u + 0..7), half h
    uint32_t maddr[2][4];
#pragma unroll
    for (int t = 0; t < 2; t++) {
#pragma unroll
        for (int u = 0; u < 4; u++)
            maddr[t][u] = C::maskOff + wave * C::maskSlot + (c32 * 8 + ((4 * t + u) ^ ((c32 >> 1) & 7))) * 16 + 8 * h;
    }

    // per-lane LDS read bases (image pair 0; pair 1 is + pairBytes)
    // K: slice kk, row 32t + c32, half h -> kk*2048 + t*1024 + kbase
    const uint32_t kbase = c32 * 32 + ((h ^ ((c32 >> 3) & 1)) * 16);
    // V^T gather, 16-lane group (h, dh), lane gi of it: row 32t + 16q + 8e + 4h + gi/4,
    // chunk (2dh + (gi&3)/2) ^ ((h + 2e) & 3), half gi&1 -> db*4096 + t*2048 + q*1024 + vbase[e]
    const int gi = lane & 15, dh = (lane >> 4) & 1;
    uint32_t vbase[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int row = 8 * e + 4 * h + (gi >> 2);
        const int ch = (2 * dh + ((gi & 3) >> 1)) ^ ((h + 2 * e) & 3);
        vbase[e] = C::img + row * 64 + ch * 16 + (gi & 1) * 8;
    }

    // ---- prologue.  Quantised: raw tiles 0..2, mask 0; dequantise tile 0.
    // f16: image pairs 0 and 1, mask 0 (the first body waits for pair 0).
    uint32_t doff[4];
    if constexpr (C::kDirect) {
        pf_direct_offsets<D>(a, wave, lane, doff);
        for (int s = 0; s < 2 && s < ntiles; s++)
            pf_direct_issue<D>(a, rs, (t0 + s) * kPfKeys, lds0 + s * C::pairBytes, wave, doff);
        if (ntiles > 0) mask_issue(0);
    } else {
        for (int s = 0; s < 3 && s < ntiles; s++) pf_issue<KT, D>(rs, (t0 + s) * kPfKeys, raw_lds(s), wave, lane);
        if (ntiles > 0) mask_issue(0);
        // raw 0 landed (raw 1, 2 and mask 0 may fly on)
        pf_vm_wait<KT, D>(min(2, ntiles - 1), ntiles > 0 ? mask_groups(0) : 0);
        __syncthreads();
        if (ntiles > 0) pf_dequant<KT, D>(raw_ptr(0), smem, smem + C::img, wave, lane);
    }

    float m_run = kNegInf;    // reference max (log2 domain) of this lane's row
    f32x2 l2 = {0.0f, 0.0f};  // this lane's partial row sums (its 32 of every 64 keys)
    f32x16 o[NDB];
#pragma unroll
    for (int db = 0; db < NDB; db++) {
#pragma unroll
        for (int j = 0; j < 16; j++) o[db][j] = 0.0f;
    }
    const float log2e = 1.4426950408889634f;
    const float scale = a.scale_log2 / log2e;

#ifdef FATTN_STAMPS
    // diagnostic build only: shader-clock cycles per phase, summed over tiles
    // (0 wait+barrier, 1 DMA issue, 2 dequant, 3 S^T, 4 softmax, 5 O^T)
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t t_prev = __builtin_amdgcn_s_memtime();
#define PF_T(k)                                              \
    do {                                                     \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();    \
        ph[k] += t_ - t_prev;                                \
        t_prev = t_;                                         \
    } while (0)
#else
#define PF_T(k) do { } while (0)
#endif
    auto body = [&](int s, auto par) {
        constexpr int P = decltype(par)::value;  // image pair of tile s
        // quantised: raw s+1 landed (raw s+2 and mask s may fly on);
        // f16: image pair of tile s landed (tile s+1 and mask s may fly on)
        PF_T(7);
        pf_vm_wait<KT, D>(s + C::ahead - 1 < ntiles ? 1 : 0, C::kDirect ? NM : mask_groups(s));
        __syncthreads();
        PF_T(0);
        if constexpr (C::kDirect) {
            // into the pair every wave finished reading before the barrier
            if (s + 2 < ntiles)
                pf_direct_issue<D>(a, rs, (t0 + s + 2) * kPfKeys, lds0 + ((P + 2) % 3) * C::pairBytes, wave, doff);
        }
        PF_T(1);
        // (the round-1 phase stagger -- waves 4-7 dequantising after their
        // compute, FATTN_OPT_PF_STAGGER bit 0 -- measured neutral and was
        // removed: it kept the dequantisation's state live across the compute)
#ifndef FATTN_PF_DEQ_EARLY
        // reads, conversion and image writes of tile s + 1 in one piece before
        // tile s's compute.  (FATTN_PF_DEQ_EARLY, A/B builds: the raw words read
        // before the S^T operand reads and converted after the S^T chains --
        // Q8_0 zero mask 439-452 vs 439-449 us, random mask 458-480 vs 483-486,
        // Q4_0 432-441 vs 419-434: no net gain for 14 more VGPRs, profiles/r04_i)
        if constexpr (!C::kDirect) {
            if (s + 1 < ntiles)
                pf_dequant<KT, D>(raw_ptr(s + 1), smem + (P ^ 1) * C::pairBytes,
                                  smem + (P ^ 1) * C::pairBytes + C::img, wave, lane);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        PfRaw deq;
        const bool deq_next = false;
#else
        // diagnostic build only: the raw words of tile s + 1 (this wave's half
        // block) read now, converted and written after the S^T chains
        PfRaw deq;
        const bool deq_next = !C::kDirect && s + 1 < ntiles;  // workgroup-uniform
        if constexpr (!C::kDirect) {
            if (deq_next) deq = pf_dequant_load<KT, D>(raw_ptr(s + 1), wave, lane);
        }
#endif
        PF_T(2);
        // quantised: raw tile s + 3 is issued during this tile's first S^T chain
        // (an issue that stalls on a full memory queue then waits beside the
        // MFMAs, not in front of them), so it comes after mask s + 1; at the
        // mask wait only raw s + 2 is younger than mask s (tile 0: nothing)
        const int mask_younger = C::kDirect ? (s + C::ahead < ntiles ? 1 : 0) : s == 0 ? 0 : (s + 2 < ntiles ? 1 : 0);
        auto issue_raw = [&] {
            if constexpr (!C::kDirect) {
                if (s + 3 < ntiles) pf_issue<KT, D>(rs, (t0 + s + 3) * kPfKeys, raw_lds(s + 3), wave, lane);
            }
        };
#ifdef FATTN_MQ_NOCOMPUTE
        if constexpr (HM) {
            pf_vm_wait<KT, D>(mask_younger, 0);
            if (s + 1 < ntiles) mask_issue(s + 1);
        }
        issue_raw();
        return;  // diagnostic build only: copies, dequant and barriers
#endif
        const uint8_t* img = smem + P * C::pairBytes;  // K image; vbase includes + img

        // -- this wave's mask block of tile s (landed; raw s+3 / image s+2 may fly
        // on): read it, refill the slot, and skip the tile when the whole 32 x 64
        // block is -inf (causal prefill: a fully masked block adds nothing to m,
        // l or O, so skipping it is exact -- the rows' state is left untouched)
        // (a tile whose whole 256 x 64 mask block is +-0, flag 2, neither waits
        // for nor reads its empty slot: its mask values are zeros in registers;
        // the next DMA into the slot lands after the empty one, in issue order)
        u32x2 mk[2][4];
        bool live = true;
        if constexpr (HM) {
            const bool zero = zero_of(s);  // workgroup-uniform
            if (!zero) {
                pf_vm_wait<KT, D>(mask_younger, 0);
#pragma unroll
                for (int t = 0; t < 2; t++) {
#pragma unroll
                    for (int uu = 0; uu < 4; uu++) mk[t][uu] = *(const u32x2*)(smem + maddr[t][uu]);
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            } else {
#pragma unroll
                for (int t = 0; t < 2; t++) {
#pragma unroll
                    for (int uu = 0; uu < 4; uu++) mk[t][uu] = u32x2{0u, 0u};
                }
            }
            if (s + 1 < ntiles) mask_issue(s + 1);
            uint32_t open = 0;  // any key not at -inf (f16 0xFC00)
#pragma unroll
            for (int t = 0; t < 2; t++) {
#pragma unroll
                for (int uu = 0; uu < 4; uu++) open |= (mk[t][uu].x ^ 0xFC00FC00u) | (mk[t][uu].y ^ 0xFC00FC00u);
            }
            live = __builtin_amdgcn_ballot_w64(open != 0) != 0;
        }
        // (state of the tile's first half, shared by the two live blocks below)
        f16x8 ka[2][NK];
        f32x16 st0, st1;
        float u0[16], u1[16];
        float tmax0 = kNegInf;
        // scores (natural units) u = scale * s + mask; element j of subtile t is
        // key 32t + 8(j/4) + 4h + (j%4) of this lane's row
        auto scores = [&](const f32x16& stt, int t, float (&ut)[16]) {
            if constexpr (HM) {
#pragma unroll
                for (int uu = 0; uu < 4; uu++) {
                    const f16x2 m01 = as_h2(mk[t][uu].x), m23 = as_h2(mk[t][uu].y);
                    ut[4 * uu + 0] = fmaf(stt[4 * uu + 0], scale, (float)m01.x);
                    ut[4 * uu + 1] = fmaf(stt[4 * uu + 1], scale, (float)m01.y);
                    ut[4 * uu + 2] = fmaf(stt[4 * uu + 2], scale, (float)m23.x);
                    ut[4 * uu + 3] = fmaf(stt[4 * uu + 3], scale, (float)m23.y);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 16; j++) ut[j] = stt[j];
            }
        };
        if (live) {
        // -- one tile, phases overlapped within the wave (cdna_hip_programming.md
        // T19): the two subtiles' S^T chains back to back, the scores of subtile 0
        // (u = fma(s, scale, mask)) computed under subtile 1's MFMAs, subtile 0's
        // exponentials under nothing but their own latency, then subtile 1's
        // exponentials under subtile 0's P.V MFMAs.  Same arithmetic as before
        // (one max over the tile's 64 keys, one deferred-rescale decision).
        // K operands of subtile 0 (8 ds_read_b128, one LDS wait); subtile 1's
        // are read behind st0's chain (their latency under its MFMAs)
#pragma unroll
        for (int kk = 0; kk < NK; kk++) ka[0][kk] = *(const f16x8*)(img + kbase + kk * (kPfKeys * 32));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < 16; j++) st0[j] = 0.0f;
#pragma unroll
        for (int kk = 0; kk < NK; kk++) st0 = mfma32(ka[0][kk], qop[kk], st0);
#pragma unroll
        for (int kk = 0; kk < NK; kk++) ka[1][kk] = *(const f16x8*)(img + kbase + kk * (kPfKeys * 32) + 1024);
#pragma unroll
        for (int j = 0; j < 16; j++) st1[j] = 0.0f;
#pragma unroll
        for (int kk = 0; kk < NK; kk++) st1 = mfma32(ka[1][kk], qop[kk], st1);
        // scores (natural units) u = scale * s + mask; element j of subtile t is
        // key 32t + 8(j/4) + 4h + (j%4) of this lane's row.  Subtile 0's depend
        // only on st0: the scheduler places them between st1's MFMAs.
        scores(st0, 0, u0);
#pragma unroll
        for (int j = 0; j < 16; j++) tmax0 = fmaxf(tmax0, u0[j]);
        // one MFMA of st1's chain, then up to 4 of subtile 0's VALU
#pragma unroll
        for (int i = 0; i < NK; i++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        }  // live, first half
        // quantised: tile s + 1's images from the raw words read above (the
        // conversion VALU runs under the tail of the S^T chains)
        if constexpr (!C::kDirect) {
            if (deq_next)
                pf_dequant_store<KT, D>(deq, smem + (P ^ 1) * C::pairBytes, smem + (P ^ 1) * C::pairBytes + C::img, wave,
                                        lane);
        }
        // quantised: raw tile s + 3, issued while the S^T chains execute (a
        // skipped tile issues it here too)
        issue_raw();
        if (live) {
        scores(st1, 1, u1);
        float tmax = tmax0;
#pragma unroll
        for (int j = 0; j < 16; j++) tmax = fmaxf(tmax, u1[j]);
        // exponent argument: x * c - m (log2 domain); c = log2e with a mask,
        // scale * log2e without (scale > 0: the planner's condition)
        const float c = HM ? log2e : a.scale_log2;
        tmax = xor32_pair(tmax, true) * c;
        // deferred max (cdna_hip_programming.md T13), as in the multi-query kernel
        if (__builtin_amdgcn_ballot_w64(tmax > m_run + kDeferLog2)) {
            const float m_new = fmaxf(m_run, tmax);
            const float alpha = (m_new == kNegInf) ? 1.0f : __builtin_amdgcn_exp2f(m_run - m_new);
            l2 *= alpha;
#pragma unroll
            for (int db = 0; db < NDB; db++) o[db] *= alpha;
            m_run = m_new;
        }
        const float nm = (m_run == kNegInf) ? 0.0f : -m_run;
        auto probs = [&](const float (&ut)[16], f16x8 (&pbt)[2]) {
            float pv[16];
#pragma unroll
            for (int j = 0; j < 16; j++) pv[j] = __builtin_amdgcn_exp2f(fmaf(ut[j], c, nm));
#pragma unroll
            for (int j = 0; j < 16; j += 2) l2 += f32x2{pv[j], pv[j + 1]};
#pragma unroll
            for (int q = 0; q < 2; q++) {
                f16x8 x;
                x.s0 = (f16)pv[8 * q]; x.s1 = (f16)pv[8 * q + 1]; x.s2 = (f16)pv[8 * q + 2]; x.s3 = (f16)pv[8 * q + 3];
                x.s4 = (f16)pv[8 * q + 4]; x.s5 = (f16)pv[8 * q + 5]; x.s6 = (f16)pv[8 * q + 6]; x.s7 = (f16)pv[8 * q + 7];
                pbt[q] = x;
            }
        };
        // V^T operands of subtile t, k-step q: keys 32t + 16q + 8(i/4) + 4h + (i%4)
        // of k-group h (i = 0..7), gathered by ds_read_b64_tr_b16
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        auto v_reads = [&](int t, u32x4 (&va)[2][NDB]) {
#pragma unroll
            for (int q = 0; q < 2; q++) {
#pragma unroll
                for (int db = 0; db < NDB; db++) {
                    const uint32_t off = db * (kPfKeys * 64) + t * 2048 + q * 1024;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + vbase[0] + off));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + vbase[1] + off));
                    const u32x2 a2 = __builtin_bit_cast(u32x2, lo), b2 = __builtin_bit_cast(u32x2, hi);
                    va[q][db] = u32x4{a2.x, a2.y, b2.x, b2.y};
                }
            }
        };
        f16x8 pb0[2], pb1[2];
        u32x4 va0[2][NDB];
        v_reads(0, va0);          // their LDS latency runs under subtile 0's exponentials
        probs(u0, pb0);
        __builtin_amdgcn_sched_group_barrier(0x100, 4 * NDB, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 64, 0);
        __builtin_amdgcn_sched_barrier(0);
        // subtile 0's P.V (8 MFMAs) with subtile 1's exponentials between them
#pragma unroll
        for (int q = 0; q < 2; q++) {
#pragma unroll
            for (int db = 0; db < NDB; db++) o[db] = mfma32(__builtin_bit_cast(f16x8, va0[q][db]), pb0[q], o[db]);
        }
        probs(u1, pb1);
#pragma unroll
        for (int i = 0; i < 2 * NDB; i++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        u32x4 va1[2][NDB];
        v_reads(1, va1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 2; q++) {
#pragma unroll
            for (int db = 0; db < NDB; db++) o[db] = mfma32(__builtin_bit_cast(f16x8, va1[q][db]), pb1[q], o[db]);
        }
        }  // live
        PF_T(5);
    };
    if constexpr (C::kDirect) {
        for (int s = 0; s < ntiles; s += 3) {
            body(s, std::integral_constant<int, 0>());
            if (s + 1 < ntiles) body(s + 1, std::integral_constant<int, 1>());
            if (s + 2 < ntiles) body(s + 2, std::integral_constant<int, 2>());
        }
    } else {
        for (int s = 0; s < ntiles; s += 2) {
            body(s, std::integral_constant<int, 0>());
            if (s + 1 < ntiles) body(s + 1, std::integral_constant<int, 1>());
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#ifdef FATTN_STAMPS
    if (lane == 0 && g_stamps) {
        const int64_t blk = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        for (int k = 0; k < 8; k++) g_stamps[(blk * kPfWaves + wave) * 16 + k] = ph[k];
        g_stamps[(blk * kPfWaves + wave) * 16 + 8] = (unsigned long long)ntiles;
    }
#endif
#undef PF_T

    // ---- normalise and store.  O^T element j of block db is dim 32db + 8(j/4)
    // + 4h + (j%4) of this lane's row: stored straight from that layout, one
    // instruction would write 32 B into each of 32 rows -- partial lines, which
    // the memory writes as whole granules (WRITE_SIZE 2.1x the output on the
    // prefill shape, profiles/r04_prof1).  So each wave parks its 32 normalised
    // rows in LDS ([32 rows][DI + 4] f32, its own region; every wave is past
    // the loop's last LDS read: one barrier) and stores them back as whole
    // rows, 64 lanes x 16 B = 1 KiB of contiguous row bytes per instruction
    // (cdna_hip_programming.md T21).
    const float l_tot = xor32_pair(l2.x + l2.y, false);
#ifdef FATTN_PF_DIRECT_STORE
    // diagnostic build only (A/B): the row-per-lane stores from the accumulator layout
    if (row_ok) {
        float* out = a.dst + (((int64_t)iq3 * a.NQ + iq1) * a.H + iq2) * D + 4 * h;
        const float inv = 1.0f / l_tot;
#pragma unroll
        for (int db = 0; db < NDB; db++) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; r++) v[r] = l_tot == 0.0f ? __builtin_nanf("") : o[db][4 * u + r] * inv;
                if (32 * db + 8 * u + 4 * h < D) *(f32x4*)(out + 32 * db + 8 * u) = v;
            }
        }
    }
    return;
#endif
    constexpr int kStride = C::DI + 4;  // floats (+16 B a row: the parking writes are conflict-free)
    static_assert(kPfWaves * kPfRowsW * kStride * 4 <= C::ldsBytes, "");
    __syncthreads();  // every wave is done with the images, raw tiles and mask slots
    float* park = (float*)smem + wave * (kPfRowsW * kStride);
    {
        const float inv = 1.0f / l_tot;  // fully masked row -> NaN like the reference
        float* pk = park + c32 * kStride + 4 * h;
#pragma unroll
        for (int db = 0; db < NDB; db++) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; r++) v[r] = l_tot == 0.0f ? __builtin_nanf("") : o[db][4 * u + r] * inv;
                *(f32x4*)(pk + 32 * db + 8 * u) = v;
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the wave reads back only its own rows)
    constexpr int CPR = D / 4;                     // 16-B chunks of a dst row (D = 80: 20)
    static_assert(kPfRowsW * CPR % kWave == 0, "");
#pragma unroll
    for (int i = 0; i < kPfRowsW * CPR / kWave; i++) {
        const int g = kWave * i + lane;
        const int r = g / CPR, c = g % CPR;        // row of the wave, chunk of the row
        int q1, q2;
        if (row_of(kPfRowsW * wave + r, q1, q2)) {
            const f32x4 v = *(const f32x4*)(park + r * kStride + 4 * c);
            *(f32x4*)(a.dst + (((int64_t)iq3 * a.NQ + q1) * a.H + q2) * D + 4 * c) = v;
        }
    }
}

// ---- prefill mask pre-pass: flags[qt][s] for the (query tile, KV tile) block
// of the QPT mask rows x 64 keys: 0 when every value is -inf (f16 0xFC00; the
// block adds nothing), 2 when every value is +-0 (the mask adds nothing: its
// DMA is skipped), else 1.  One workgroup per block; every flag is written on
// every launch, so the array needs no initialisation.  Reads the mask once
// (f16 [NQ][N]).
__device__ __forceinline__ void pf_mask_flags_block(const uint8_t* __restrict__ mask, int64_t m_nb1, int NQ, int QPT,
                                                    int ntiles, uint8_t* __restrict__ flags, int s, int qt) {
    // thread -> (row qt*QPT + r, 16-B piece pc of the tile's 128 B): 8 pieces
    // per row; batches of 8 loads issued before one wait (a load per loop trip
    // made the block 8 serial memory round trips); rows past the mask re-read
    // its last row and count for nothing
    constexpr int kB = 8;
    uint32_t open = 0, nonzero = 0;
    for (int i0 = threadIdx.x; i0 < QPT * 8; i0 += 256 * kB) {
        u32x4 w[kB];
        bool ok[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int i = i0 + 256 * u;
            const int r = i >> 3, pc = i & 7;
            const int q = qt * QPT + r;
            ok[u] = i < QPT * 8 && q < NQ;
            const int qc = min(q, NQ - 1);
            w[u] = *(const u32x4*)(mask + (int64_t)qc * m_nb1 + (int64_t)s * kPfKeys * 2 + pc * 16);
        }
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const u32x4 x = w[u];
            const uint32_t op = (x.x ^ 0xFC00FC00u) | (x.y ^ 0xFC00FC00u) | (x.z ^ 0xFC00FC00u) | (x.w ^ 0xFC00FC00u);
            const uint32_t nz = (x.x | x.y | x.z | x.w) & 0x7FFF7FFFu;
            open |= ok[u] ? op : 0u;
            nonzero |= ok[u] ? nz : 0u;
        }
    }
    const int any_open = __syncthreads_or(open != 0);
    const int any_nonzero = __syncthreads_or(nonzero != 0);
    if (threadIdx.x == 0) flags[(int64_t)qt * ntiles + s] = !any_open ? 0 : any_nonzero ? 1 : 2;
}
static __global__ __launch_bounds__(256) void pf_mask_flags_kernel(const uint8_t* __restrict__ mask, int64_t m_nb1, int NQ,
                                                            int QPT, int ntiles, uint8_t* __restrict__ flags) {
    pf_mask_flags_block(mask, m_nb1, NQ, QPT, ntiles, flags, blockIdx.x, blockIdx.y);
}

// The prefill's pre-pass in ONE launch (round 6): the K rows staged to f16,
// the V rows staged, and the mask-flags blocks are independent jobs that ran
// as three serial launches (two kernel boundaries and two ramp-down tails on
// the plan's critical path).  Workgroups [0, nsk) stage K, [nsk, 2 nsk) stage
// V (each the kv_stage_f16 work of one (256-thread x 8-value) slice of one
// (kv head, seq)), the rest flag one (query tile, KV tile) block each; every
// workgroup has one role, so the flags' workgroup reductions stay uniform.
// STK: the cache's type, or 0 (f16 cache: flags only).
struct PfPrepassArgs {
    const uint8_t* k;
    const uint8_t* v;
    int64_t k_nb2, k_nb3, v_nb2, v_nb3;
    uint16_t* k16;
    uint16_t* v16;
    int64_t nblk;      // 32-value blocks per (kv head, seq)
    int per_head;      // staging workgroups per (kv head, seq)
    int hkv, skv;
    const uint8_t* mask;
    int64_t m_nb1;
    int NQ, QPT, ntiles, flags_on;
    uint8_t* flags;
};
template <int STK>
__global__ __launch_bounds__(256) void pf_prepass_kernel(const PfPrepassArgs p) {
    int64_t b = blockIdx.x;
    if constexpr (STK != 0) {
        const int64_t nsk = (int64_t)p.per_head * p.hkv * p.skv;
        if (b < 2 * nsk) {
            const bool isv = b >= nsk;
            if (isv) b -= nsk;
            const int64_t x = b % p.per_head;
            const int head = (int)((b / p.per_head) % p.hkv);
            const int seq = (int)(b / ((int64_t)p.per_head * p.hkv));
            kv_stage_f16_block<STK>(isv ? p.v : p.k, isv ? p.v_nb2 : p.k_nb2, isv ? p.v_nb3 : p.k_nb3,
                                    isv ? p.v16 : p.k16, p.nblk, x, head, seq, p.hkv);
            return;
        }
        b -= 2 * nsk;
    }
    pf_mask_flags_block(p.mask, p.m_nb1, p.NQ, p.QPT, p.ntiles, p.flags, (int)(b % p.ntiles), (int)(b / p.ntiles));
}

}  // namespace fattn
