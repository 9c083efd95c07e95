// fattn_mq.h -- multi-query attention over ggml-quantised KV for gfx950:
// the shapes with >= 32 query rows per kv head (config 5 batch decode, prefill).
//
// Replaces flash_attn_ext_f16<D,Q,C> (src/flash-llama.h:5-438) for many query
// rows.  The split-KV decode kernel (fattn_split.h) gives every wave its own
// KV slice and dequantises K/V on the LDS -> VGPR hop for its 16 query
// columns; with many query rows per kv head that would dequantise every K/V
// element once per 16 rows.  Here one workgroup owns 4*RPW packed
// (query row x q-head) rows -- RPW per wave, in 16-column MFMA groups -- and
// walks the KV sequence in 32-position tiles:
//
//  * all 256 threads copy a tile's raw ggml K/V rows and its mask rows
//    HBM -> LDS with buffer_load ... lds (three raw buffers, three tiles in
//    flight);
//  * the workgroup dequantises each tile ONCE, one ggml block per thread,
//    into f16 K and V images in LDS (XOR-swizzled like the decode kernel's f16
//    images: ds_read_b128 rows for K, ds_read_b64_tr_b16 transposed reads for
//    V), h(q*d) with one f16 rounding as the oracle's dequantise-then-round
//    (src/utils.h:10-11);
//  * every wave runs S^T = K.Q^T and O^T = V^T.P^T on v_mfma_f32_16x16x32_f16
//    for its RPW/16 column groups, each K / V operand read from LDS once and
//    used by all of them (LDS read bytes per MFMA / (RPW/16): at RPW = 16 the
//    image reads alone exceed the MFMA time, at RPW = 64 they take ~1/4 of
//    it), online softmax in the log2 domain.
//
// Software pipeline with ONE workgroup barrier per tile: while the waves run
// tile s from one image pair, the workgroup dequantises tile s+1 into the
// other, and the copies of tiles s+2, s+3 are in flight.
//
// RPW = 64 (256 rows, one workgroup per CU, accumulators partly in AGPRs) for
// prefill-sized problems; RPW = 16 (64 rows, two workgroups per CU) when that
// would leave the chip short of workgroups.  Split-KV only when the tiles
// alone cannot fill the chip; chunk partials then go through the decode
// kernel's last-arriver merge, one 16-row subtile per column group.
#pragma once

#include "fattn_split.h"

namespace fattn {

template <int KT, int D, int NW, int RPW>
struct MQCfg {
    static constexpr int NT = NW * kWave;                            // threads per workgroup
    static constexpr int rows = NW * RPW;                            // packed rows per workgroup
    static constexpr int rowB = row_bytes<KT, D>();
    static constexpr int kvRaw = kStep * rowB;                       // K (or V) raw bytes per tile
    static constexpr int mRaw = rows * kStep * 2;                    // mask rows x 32 f16
    static constexpr int rawBytes = (2 * kvRaw + mRaw + 15) / 16 * 16;
    static constexpr int img = kStep * D * 2;                        // one f16 image
    static constexpr int nRaw = 3;                                   // raw buffers
    static constexpr int imgOff = nRaw * rawBytes;
    static constexpr int ldsBytes = imgOff + 2 * 2 * img;            // + (K16, V16) x 2
    static constexpr int PKV = kvRaw / 16;                           // 16-B pieces of K (or V)
    static constexpr int NIKV = (PKV + NT - 1) / NT;
    static constexpr int PM = mRaw / 16;
    static constexpr int NIM = PM / NT;
    static_assert(PM % NT == 0, "");
    static_assert(ldsBytes <= 163840, "");
    // DMA instructions wave w issues per tile (mask pieces only with a mask):
    // the last K/V instruction is partial (e.g. 272 pieces of a Q8_0 D=128
    // tile) and skipped by the waves with no piece in it, so the per-wave
    // vmcnt budget differs
    static constexpr int ni_wave(int w, bool hm) {
        int n = hm ? NIM : 0;
        for (int i = 0; i < NIKV; i++) n += (i * NT + w * kWave < PKV) ? 2 : 0;
        return n;
    }
};

// Copy tile [n0, n0 + 32) (raw K rows | raw V rows | mask rows) into `buf`;
// all 256 threads, 16-B pieces, lane-linear.  Rows past N / query rows past
// the tile's fall outside the descriptors: zeros, no traffic.
template <int KT, int D, int NW, int RPW, bool HM>
__device__ __forceinline__ void mq_issue(const SplitArgs& a, const StepSrc& rs, int n0, int mrow0, uint8_t* buf,
                                         int wave, int lane) {
#ifdef FATTN_MQ_NOMEM
    return;  // diagnostic build only: no HBM traffic (compute on whatever LDS holds)
#endif
    using C = MQCfg<KT, D, NW, RPW>;
    constexpr int NT = C::NT;
    const int tid = wave * kWave + lane;
    // LDS base of this wave's 1-KiB slot in each 4-KiB instruction group (M0: scalar)
    const uint32_t lb = __builtin_amdgcn_readfirstlane(lds_addr(buf) + wave * kWave * 16);
#pragma unroll
    for (int i = 0; i < C::NIKV; i++) {
        const int p = i * NT + tid;
        if (i * NT + wave * kWave >= C::PKV) continue;  // wave-uniform (ni_wave)
        if (C::PKV % NT == 0 || p < C::PKV) {
            const uint32_t off = (uint32_t)n0 * C::rowB + p * 16;
            dma<16>(rs.k, lb + i * NT * 16, off);
            dma<16>(rs.v, lb + C::kvRaw + i * NT * 16, off);
        }
    }
    if constexpr (HM) {
#pragma unroll
        for (int i = 0; i < C::NIM; i++) {
            const int q = i * NT + tid;
            const int mr = q / 4, off = (q % 4) * 16;  // 64-B mask row = 4 pieces
            // rows past the tile's QPT query rows: outside the descriptor (no traffic)
            const uint32_t moff =
                mr < a.QPT ? (uint32_t)(mrow0 + mr) * (uint32_t)a.m_nb1 + (uint32_t)n0 * 2 + off : a.m_span;
            dma<16>(rs.m, lb + 2 * C::kvRaw + i * NT * 16, moff);
        }
    }
}

// wait until this wave's pieces of all but the `pending` youngest in-flight
// tiles have landed (pending = 0, 1, 2)
template <int NI>
__device__ __forceinline__ void wait_tiles_n(int pending) {
    if (pending <= 0) {
        wait_vmcnt_c<0>();
    } else if (pending == 1) {
        wait_vmcnt_c<NI>();
    } else {
        wait_vmcnt_c<2 * NI>();
    }
}
template <int KT, int D, int NW, int RPW, bool HM>
__device__ __forceinline__ void mq_wait_tiles(int wave, int pending) {
    using C = MQCfg<KT, D, NW, RPW>;
    switch (wave) {
        case 0: wait_tiles_n<C::ni_wave(0, HM)>(pending); break;
        case 1: wait_tiles_n<C::ni_wave(1, HM)>(pending); break;
        case 2: wait_tiles_n<C::ni_wave(2, HM)>(pending); break;
        case 3: wait_tiles_n<C::ni_wave(3, HM)>(pending); break;
        case 4: wait_tiles_n<C::ni_wave(4, HM)>(pending); break;
        case 5: wait_tiles_n<C::ni_wave(5, HM)>(pending); break;
        case 6: wait_tiles_n<C::ni_wave(6, HM)>(pending); break;
        default: wait_tiles_n<C::ni_wave(7, HM)>(pending); break;
    }
}

// Dequantise half h (elements 16h..16h+15) of ggml block b of raw row `row`
// into the two 16-B f16 chunks 4b+2h, 4b+2h+1: h(q * d), one f16 rounding
// (src/utils.h:10-11 dequantise-then-round).  The qs bytes are only 2-byte
// aligned: dword reads + v_alignbyte with a runtime shift.
// (in two steps, so a caller can issue the LDS reads early and convert later:
// dequant_half_load -> HalfRaw -> dequant_half_cvt)
struct HalfRaw {
    uint32_t u[5];  // the dwords holding the 16 qs bytes
    uint32_t dw;    // the dword holding the f16 scale
    uint32_t blk;   // byte offset of the block in the tile
};
template <int KT, int D>
__device__ __forceinline__ HalfRaw dequant_half_load(const uint8_t* raw, int row, int b, int h) {
    constexpr int RB = row_bytes<KT, D>();
    constexpr int BB = TypeInfo<KT>::block_bytes;
    HalfRaw r;
    r.blk = row * RB + BB * b;
    // Q8_0: qs bytes 16h..16h+15; Q4_0: all 16 qs bytes (low / high nibbles)
    const uint32_t q0 = r.blk + 2 + (KT == FATTN_TYPE_Q8_0 ? 16 * h : 0);
    const uint32_t qb = q0 & ~3u;
#pragma unroll
    for (int j = 0; j < 5; j++) r.u[j] = *(const uint32_t*)(raw + qb + 4 * j);
    r.dw = *(const uint32_t*)(raw + (r.blk & ~3u));
    return r;
}
template <int KT>
__device__ __forceinline__ void dequant_half_cvt(const HalfRaw& r, int h, u32x4 (&out)[2]) {
    const uint32_t sh = (r.blk + 2 + (KT == FATTN_TYPE_Q8_0 ? 16 * h : 0)) & 3u;
    uint32_t q[4];
#pragma unroll
    for (int j = 0; j < 4; j++) q[j] = alignbyte(r.u[j + 1], r.u[j], sh);
    const f16x2 d = bcast_h((r.blk & 2) ? (r.dw >> 16) : r.dw);
#pragma unroll
    for (int k = 0; k < 2; k++) {
        f16x2 h0, h1, h2, h3;
        if constexpr (KT == FATTN_TYPE_Q8_0) {
            i8x4_to_h2x2(q[2 * k], h0, h1);
            i8x4_to_h2x2(q[2 * k + 1], h2, h3);
        } else {  // elements 0-15: low nibbles of bytes 0-15; 16-31: high nibbles
            const uint32_t sft = 4 * h;
            u4x4_to_h2x2((q[2 * k] >> sft) & 0x0F0F0F0Fu, h0, h1);
            u4x4_to_h2x2((q[2 * k + 1] >> sft) & 0x0F0F0F0Fu, h2, h3);
        }
        h0 *= d; h1 *= d; h2 *= d; h3 *= d;
        out[k] = u32x4{as_u32(h0), as_u32(h1), as_u32(h2), as_u32(h3)};
    }
}
template <int KT, int D>
__device__ __forceinline__ void dequant_half(const uint8_t* raw, int row, int b, int h, u32x4 (&out)[2]) {
    dequant_half_cvt<KT>(dequant_half_load<KT, D>(raw, row, b, h), h, out);
}

// Tile `rb` (raw) -> f16 images k16 / v16 (decode kernel's swizzles).  Units
// of half a ggml block: [0, 64*NB) are K's, [64*NB, 128*NB) V's, dealt
// round-robin over the NT threads.
template <int KT, int D, int NT>
__device__ __forceinline__ void mq_dequant(const uint8_t* rb, int kv_raw, uint8_t* k16, uint8_t* v16, int tid) {
#ifdef FATTN_MQ_NODEQ
    return;  // diagnostic build only
#endif
    constexpr int NB = D / QK;
    constexpr int CPR = D * 2 / 16;
    constexpr int NU = 2 * kStep * NB;  // half blocks per image
#pragma unroll
    for (int i = 0; i < (2 * NU + NT - 1) / NT; i++) {
        const int unit = i * NT + tid;
        if ((2 * NU) % NT != 0 && unit >= 2 * NU) break;
        const bool is_v = unit >= NU;
        const int t = is_v ? unit - NU : unit;
        const int row = t / (2 * NB), b = (t / 2) % NB, h = t & 1;
        u32x4 ch[2];
        dequant_half<KT, D>(rb + (is_v ? kv_raw : 0), row, b, h, ch);
        uint8_t* dst = (is_v ? v16 : k16) + row * (D * 2);
        const int sw = is_v ? (((row & 7) << 1) & (CPR - 1)) : (row & (CPR - 1));
#pragma unroll
        for (int k = 0; k < 2; k++) *(u32x4*)(dst + (((4 * b + 2 * h + k) ^ sw) * 16)) = ch[k];
    }
}

template <int KT, int D, int NW, bool HM>
__global__ __launch_bounds__(NW * kWave, NW == 8 ? 1 : 2) void fattn_mq_kernel(const SplitArgs a) {
    constexpr int RPW = NW == 8 ? 32 : 16;  // packed rows per wave
    using C = MQCfg<KT, D, NW, RPW>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NB = D / QK;
    constexpr int NC = D / 16;
    constexpr int NG = RPW / kRows;  // 16-column MFMA groups per wave
    constexpr float kNegInf = -__builtin_inff();
    constexpr float kDeferLog2 = 8.0f;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4;
    const int i16 = lane & 15;

    // ---- tile decode: y -> (kv head, query tile); R = rk2 (whole head groups)
    const int chunk = blockIdx.x;
    const int y = blockIdx.y;
    const int iq3 = blockIdx.z;
    int qt = 0, ik2 = y, ik3 = iq3;
    if (a.n_qt != 1) {
        qt = y % a.n_qt;
        ik2 = y / a.n_qt;
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;

    // this lane's columns: packed row p = RPW * wave + 16 * gi + i16 -> (query row, q head)
    int mq[NG], iq1[NG], iq2[NG];
    bool row_ok[NG];
#pragma unroll
    for (int gi = 0; gi < NG; gi++) {
        const int p = RPW * wave + kRows * gi + i16;
        mq[gi] = div_R(a, p);
        iq1[gi] = qt * a.QPT + mq[gi];
        iq2[gi] = ik2 * a.rk2 + (p - mq[gi] * a.R);
        row_ok[gi] = mq[gi] < a.QPT && iq1[gi] < a.NQ;  // (R not a power of two: rows past QPT * R are none)
    }

    // ---- this workgroup's KV chunk: whole 32-position tiles (N % 32 == 0)
    const int c_lo = chunk * a.chunk_len;
    const int c_hi = min(a.N, c_lo + a.chunk_len);
    const int ntiles = c_hi > c_lo ? (c_hi - c_lo) / kStep : 0;

    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    rs.m = make_srd(a.mask, HM ? a.m_span : 0);
    const int mrow0 = qt * a.QPT;
    auto raw = [&](int s) { return smem + (s % C::nRaw) * C::rawBytes; };
    auto k16_of = [&](int s) { return smem + C::imgOff + (s & 1) * 2 * C::img; };

    // ---- Q^T operands (B of S^T = K.Q^T), rounded to f16 like src/utils.h:10
    f16x8 qop[NG][NB];
    {
        const auto qs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.q + (int64_t)iq3 * a.q_nb3), 0,
                                                          a.q_span, 0x00020000);
#pragma unroll
        for (int gi = 0; gi < NG; gi++) {
            const uint32_t qoff = row_ok[gi] ? (uint32_t)iq1[gi] * (uint32_t)a.q_nb1 +
                                                   (uint32_t)iq2[gi] * (uint32_t)a.q_nb2 + 32 * g
                                             : a.q_span;
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const f32x4 x0 =
                    __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(qs, qoff + 128 * b, 0, 0));
                const f32x4 x1 =
                    __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(qs, qoff + 128 * b + 16, 0, 0));
                f16x8 h;
                h.s0 = (f16)x0.x; h.s1 = (f16)x0.y; h.s2 = (f16)x0.z; h.s3 = (f16)x0.w;
                h.s4 = (f16)x1.x; h.s5 = (f16)x1.y; h.s6 = (f16)x1.z; h.s7 = (f16)x1.w;
                qop[gi][b] = h;
            }
        }
    }
    // three tiles in flight behind Q (loads retire in order: the first tile
    // wait covers Q too)
    for (int s = 0; s < 3 && s < ntiles; s++)
        mq_issue<KT, D, NW, RPW, HM>(a, rs, c_lo + s * kStep, mrow0, raw(s), wave, lane);

    // this lane's mask values of a tile: rows mq[gi], positions 16t + 4g + r
    auto mask_regs = [&](const uint8_t* rb, u32x2 (&mk)[NG][2]) {
        if constexpr (HM) {
#pragma unroll
            for (int gi = 0; gi < NG; gi++) {
                const uint8_t* mb = rb + 2 * C::kvRaw + (mq[gi] < a.QPT ? mq[gi] : 0) * (kStep * 2) + 8 * g;
                mk[gi][0] = *(const u32x2*)mb;
                mk[gi][1] = *(const u32x2*)(mb + 32);
            }
        }
    };

    u32x2 mk_cur[NG][2];
#pragma unroll
    for (int gi = 0; gi < NG; gi++) mk_cur[gi][0] = mk_cur[gi][1] = u32x2{0, 0};
    if (ntiles > 0) {
        mq_wait_tiles<KT, D, NW, RPW, HM>(wave, min(2, ntiles - 1));
        __syncthreads();
        mq_dequant<KT, D, C::NT>(raw(0), C::kvRaw, k16_of(0), k16_of(0) + C::img, tid);
        mask_regs(raw(0), mk_cur);
    }

    float m_run[NG], l_run[NG];
    f32x4 o[NG][NC];
#pragma unroll
    for (int gi = 0; gi < NG; gi++) {
        m_run[gi] = kNegInf;
        l_run[gi] = 0.0f;
#pragma unroll
        for (int c = 0; c < NC; c++) o[gi][c] = f32x4{0, 0, 0, 0};
    }
    const float log2e = 1.4426950408889634f;

    // One barrier per tile: after the barrier of iteration s, image s is
    // complete, raw tile s + 1 has landed, and raw buffer s % 3 (tile s,
    // consumed in iteration s - 1) takes tile s + 3; the workgroup then
    // dequantises tile s + 1 into the other image while each wave runs tile s.
    for (int s = 0; s < ntiles; s++) {
        if (s + 1 < ntiles) mq_wait_tiles<KT, D, NW, RPW, HM>(wave, min(1, ntiles - 2 - s));
        __syncthreads();
        if (s + 3 < ntiles) mq_issue<KT, D, NW, RPW, HM>(a, rs, c_lo + (s + 3) * kStep, mrow0, raw(s + 3), wave, lane);
        u32x2 mk_next[NG][2];
#pragma unroll
        for (int gi = 0; gi < NG; gi++) mk_next[gi][0] = mk_next[gi][1] = u32x2{0, 0};
        if (s + 1 < ntiles) {
            mq_dequant<KT, D, C::NT>(raw(s + 1), C::kvRaw, k16_of(s + 1), k16_of(s + 1) + C::img, tid);
            mask_regs(raw(s + 1), mk_next);
        }
#ifdef FATTN_MQ_NOCOMPUTE
        continue;  // diagnostic build only: copies, dequant and barriers
#endif
        const uint8_t* k16 = k16_of(s);
        const uint8_t* v16 = k16 + C::img;
        // -- S^T = K.Q^T for the two 16-position subtiles; each K operand feeds NG MFMAs
        f32x4 st[NG][2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
#pragma unroll
            for (int gi = 0; gi < NG; gi++) st[gi][t] = f32x4{0, 0, 0, 0};
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const f16x8 ka = k_operand<FATTN_TYPE_F16, D>(k16, 16 * t + i16, g, b, 0);
#pragma unroll
                for (int gi = 0; gi < NG; gi++) st[gi][t] = mfma16(ka, qop[gi][b], st[gi][t]);
            }
        }
        // -- online softmax per column group
        f16x8 pb[NG];
#pragma unroll
        for (int gi = 0; gi < NG; gi++) {
            float sv[8];
#pragma unroll
            for (int t = 0; t < 2; t++) {
                const f16x2 m01 = as_h2(mk_cur[gi][t].x), m23 = as_h2(mk_cur[gi][t].y);
                const float mk[4] = {(float)m01.x, (float)m01.y, (float)m23.x, (float)m23.y};
#pragma unroll
                for (int r = 0; r < 4; r++) sv[4 * t + r] = st[gi][t][r] * a.scale_log2 + mk[r] * log2e;
            }
            float tmax = fmaxf(fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3])),
                               fmaxf(fmaxf(sv[4], sv[5]), fmaxf(sv[6], sv[7])));
            tmax = grp4_max(tmax);
            // deferred max (cdna_hip_programming.md T13): the reference max moves
            // only when a column's tile max passes it by more than kDeferLog2, so
            // the O-wide rescale is rare; meanwhile P <= 2^kDeferLog2 (exact in
            // f16's range, same relative precision).  The decision precedes this
            // tile's exponentials, and O, l are scaled together.
            if (__builtin_amdgcn_ballot_w64(tmax > m_run[gi] + kDeferLog2)) {
                const float m_new = fmaxf(m_run[gi], tmax);
                const float alpha = (m_new == kNegInf) ? 1.0f : __builtin_amdgcn_exp2f(m_run[gi] - m_new);
                l_run[gi] *= alpha;
#pragma unroll
                for (int c = 0; c < NC; c++) o[gi][c] *= alpha;
                m_run[gi] = m_new;
            }
            const float m_use = (m_run[gi] == kNegInf) ? 0.0f : m_run[gi];
            float pv[8];
#pragma unroll
            for (int j = 0; j < 8; j++) pv[j] = __builtin_amdgcn_exp2f(sv[j] - m_use);
            l_run[gi] += ((pv[0] + pv[1]) + (pv[2] + pv[3])) + ((pv[4] + pv[5]) + (pv[6] + pv[7]));
            pb[gi].s0 = (f16)pv[0]; pb[gi].s1 = (f16)pv[1]; pb[gi].s2 = (f16)pv[2]; pb[gi].s3 = (f16)pv[3];
            pb[gi].s4 = (f16)pv[4]; pb[gi].s5 = (f16)pv[5]; pb[gi].s6 = (f16)pv[6]; pb[gi].s7 = (f16)pv[7];
        }
        // -- O^T += V^T.P^T; each V operand feeds NG MFMAs
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const f16x8 va = v_operand_f16<FATTN_TYPE_F16, D>(v16, c, g, i16);
#pragma unroll
            for (int gi = 0; gi < NG; gi++) o[gi][c] = mfma16(va, pb[gi], o[gi][c]);
        }
#pragma unroll
        for (int gi = 0; gi < NG; gi++) {
            mk_cur[gi][0] = mk_next[gi][0];
            mk_cur[gi][1] = mk_next[gi][1];
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    float l_tot[NG];
#pragma unroll
    for (int gi = 0; gi < NG; gi++) l_tot[gi] = grp4_sum(l_run[gi]);

    if (a.n_chunks == 1) {
#pragma unroll
        for (int gi = 0; gi < NG; gi++) {
            if (!row_ok[gi]) continue;
            float* out = a.dst + (((int64_t)iq3 * a.NQ + iq1[gi]) * a.H + iq2[gi]) * D + 4 * g;
            const float inv = 1.0f / l_tot[gi];  // fully masked row -> NaN like the reference
#pragma unroll
            for (int c = 0; c < NC; c++) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; r++) v[r] = l_tot[gi] == 0.0f ? __builtin_nanf("") : o[gi][c][r] * inv;
                *(f32x4*)(out + 16 * c) = v;
            }
        }
        return;
    }

    // ---- several chunks: publish each column group's 16 rows as subtile
    // (tile, 4*NG) in the decode kernel's partial layout.  merge_launch: the
    // subtiles' chunk partials merge in fattn_mq_merge_kernel (the kernel
    // boundary orders the stores before its loads); otherwise the last
    // workgroup of the tile merges them (same hand-off as fattn_split_kernel)
    constexpr int SUBS = NW * NG;
    const int64_t tile = (int64_t)iq3 * gridDim.y + y;
    if (a.merge_launch) {
#pragma unroll
        for (int gi = 0; gi < NG; gi++) {
            const int64_t slot = ((tile * SUBS + wave * NG + gi) * a.n_chunks + chunk) * kRows + i16;
            if (a.part_f16) {  // (SplitArgs::part_f16: O / l in f16, 8 B per 4 dims)
                const float inv = l_tot[gi] > 0.0f ? 1.0f / l_tot[gi] : 0.0f;
#pragma unroll
                for (int c = 0; c < NC; c++) {
                    const f16x2 lo = {(_Float16)(o[gi][c][0] * inv), (_Float16)(o[gi][c][1] * inv)};
                    const f16x2 hi = {(_Float16)(o[gi][c][2] * inv), (_Float16)(o[gi][c][3] * inv)};
                    *(u32x2*)((uint16_t*)a.ws_o + slot * D + 16 * c + 4 * g) =
                        u32x2{__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi)};
                }
            } else {
#pragma unroll
                for (int c = 0; c < NC; c++) *(f32x4*)(a.ws_o + slot * D + 16 * c + 4 * g) = o[gi][c];
            }
            if (g == 0) *(f32x2*)(a.ws_ml + 2 * slot) = f32x2{m_run[gi], l_tot[gi]};
        }
        return;
    }
    // this launch's stamp on the tile's arrival word (arrival_begin,
    // fattn_split.h): ahead of the publish, so the drain below covers it
    if (tid == 0) arrival_begin(a, tile);
    {
        auto bits = [](float x) { return __builtin_bit_cast(uint32_t, x); };
#pragma unroll
        for (int gi = 0; gi < NG; gi++) {
            const int64_t sub = tile * SUBS + wave * NG + gi;
            const int64_t slot = (sub * a.n_chunks + chunk) * kRows + i16;
#pragma unroll
            for (int c = 0; c < NC; c++)
                st_sc1(a.ws_o + slot * D + 16 * c + 4 * g,
                       u32x4{bits(o[gi][c][0]), bits(o[gi][c][1]), bits(o[gi][c][2]), bits(o[gi][c][3])});
            if (g == 0) st_sc1_x2(a.ws_ml + 2 * slot, u32x2{bits(m_run[gi]), bits(l_tot[gi])});
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last_flag = (int*)smem;
    if (tid == 0) *last_flag = arrive_last(a, tile, a.n_chunks);
    __syncthreads();
    if (!*last_flag) return;
    __syncthreads();  // the flag word is reused by the merge's LDS
    // valid packed rows: the prefix [0, tq * R), query-major
    const int valid = min(a.QPT, a.NQ - qt * a.QPT) * a.R;
    for (int j = 0; j < SUBS; j++) {
        const int rv = min(kRows, valid - kRows * j);
        if (rv <= 0) break;
        combine_tile<D>(a, tile * SUBS + j, qt, 0, ik2, iq3, rv, kRows * j, smem);
        __syncthreads();
    }
}

// Second launch of a split multi-query plan (SplitArgs::merge_launch): one
// wave per packed row of a 16-row subtile merges the row's chunk partials
// (merge_row_parts: the fa_reduce LSE merge of src/flash_row_float.h:415-472
// in fp32, fixed order) and writes the normalised dst row.  grid.y runs over
// (tile, subtile) pairs, y' = tile_y * SUBS + sub, so the partial slots are
// the multi-query kernel's ((tile * SUBS + sub) * chunks + chunk) * 16 + row.
template <int D, int KIT, int SUBS, bool F16 = false>  // F16: the f16 partials of SplitArgs::part_f16
__global__ __launch_bounds__(256) void fattn_mq_merge_kernel(const SplitArgs a) {
    const int lane = threadIdx.x & 63;
    const int tm = blockIdx.x * 4 + (threadIdx.x >> 6);  // row of the subtile
    const int ys = blockIdx.y, iq3 = blockIdx.z;
    const int y = ys / SUBS, sub = ys % SUBS;
    int qt = 0, ik2 = y;  // the multi-query kernel's tile decode
    if (a.n_qt != 1) {
        qt = y % a.n_qt;
        ik2 = y / a.n_qt;
    }
    const int p = kRows * sub + tm;  // packed row of the tile
    if (p >= min(a.QPT, a.NQ - qt * a.QPT) * a.R) return;
    const int64_t slot0 = ((int64_t)iq3 * gridDim.y + ys) * a.n_chunks * kRows + tm;  // chunk 0's row
    const int rq = div_R(a, p);
    float* out = a.dst + (((int64_t)iq3 * a.NQ + qt * a.QPT + rq) * a.H + ik2 * a.rk2 + (p - rq * a.R)) * D;
    if constexpr (F16) {
        merge_row_parts_h<D, KIT>((const uint16_t*)a.ws_o + slot0 * D, a.ws_ml + 2 * slot0, a.n_chunks, out, lane,
                                  kRows * D, 2 * kRows);
    } else {
        merge_row_parts<D, KIT>(a.ws_o + slot0 * D, a.ws_ml + 2 * slot0, a.n_chunks, out, lane, kRows * D, 2 * kRows);
    }
}

}  // namespace fattn
