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
//    flight; the workgroup dequantises each tile ONCE (one half ggml block per
//    thread for K and one for V) into f16 K and V images, h(q*d) with one f16
//    rounding (src/utils.h:10-11);
//  * "swapped" products on v_mfma_f32_32x32x16_f16: S^T = K.Q^T (K rows from
//    the image by ds_read_b128, Q^T kept in registers), so a lane holds 16
//    keys of ONE query row -- the row max / sum are 31 in-lane ops and one
//    v_permlane32_swap; then O^T = V^T.P^T where P^T is the S^T accumulator
//    itself converted to f16 (no lane movement): the 16 keys of each PV k-step
//    are taken in the accumulator's own order and V^T is gathered in the same
//    order with ds_read_b64_tr_b16 (4 keys x 16 dims per 16-lane group);
//  * mask values straight from L2 into registers one tile ahead (the mask of
//    a query row is shared by every head of the row, so it stays L2-resident);
//  * one workgroup barrier per tile: while the waves run tile s from one image
//    pair, the workgroup dequantises tile s+1 into the other and tiles s+2,
//    s+3 are in flight.
//
// LDS images: K [64 keys][D] f16, 16-B chunk c of row r at c ^ (r & 15) (rows
// 0..15 of one ds_read_b128 phase hit 16 distinct chunks); V [64 keys][D] f16,
// chunk c of row r at c ^ 2(r & 3) (the 4 rows x 32 B of one transposed-read
// lane group hit 8 distinct chunks, chunk pairs stay adjacent).
#pragma once

#include "fattn_mq.h"

namespace fattn {

constexpr int kPfWaves = 8;
constexpr int kPfRowsW = 32;                    // packed rows per wave
constexpr int kPfRows = kPfWaves * kPfRowsW;    // per workgroup
constexpr int kPfKeys = 64;                     // keys per tile

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int KT, int D>
struct PfCfg {
    static constexpr int NT = kPfWaves * kWave;
    static constexpr int rowB = row_bytes<KT, D>();
    static constexpr int kvRaw = kPfKeys * rowB;                    // raw K (or V) bytes per tile
    static constexpr int rawBytes = (2 * kvRaw + 15) / 16 * 16;
    static constexpr int nRaw = 3;
    static constexpr int img = kPfKeys * D * 2;                     // one f16 image
    static constexpr int imgOff = nRaw * rawBytes;
    static constexpr int ldsBytes = imgOff + 2 * 2 * img;           // + (K16, V16) x 2
    static constexpr int NI = (kvRaw + 1023) / 1024;                // 1-KiB DMA instructions per K (or V) tile
    // instructions j = 0 .. 2*NI-1 (K then V) go to wave j % 8
    static constexpr int ni_wave(int w) { return (2 * NI - w + kPfWaves - 1) / kPfWaves; }
    static constexpr int NB = D / QK;                               // ggml blocks per row
    static constexpr int NU = kPfKeys * NB * 2;                     // half blocks per image
    static_assert(NU == NT, "one K and one V half block per thread");
    static_assert(ldsBytes <= 163840, "");
};

template <int KT, int D>
__device__ __forceinline__ void pf_issue(const StepSrc& rs, int n0, uint8_t* buf, int wave, int lane) {
#ifdef FATTN_MQ_NOMEM
    return;  // diagnostic build only
#endif
    using C = PfCfg<KT, D>;
    const uint32_t lb = lds_addr(buf);
    for (int j = wave; j < 2 * C::NI; j += kPfWaves) {  // wave-uniform
        const bool is_v = j >= C::NI;
        const int i = is_v ? j - C::NI : j;
        const int byte = i * 1024 + lane * 16;
        if (C::kvRaw % 1024 == 0 || byte < C::kvRaw)
            dma<16>(is_v ? rs.v : rs.k, lb + (is_v ? C::kvRaw : 0) + i * 1024, (uint32_t)n0 * C::rowB + byte);
    }
}

// counted wait: all but this wave's `pending` youngest DMA tiles (pending 0/1),
// with `extra` younger non-DMA loads allowed to stay in flight too
template <int NI>
__device__ __forceinline__ void pf_wait_n(int pending) {
    if (pending <= 0) {
        wait_vmcnt_c<0>();
    } else {
        wait_vmcnt_c<NI>();
    }
}
template <int KT, int D>
__device__ __forceinline__ void pf_wait(int wave, int pending) {
    using C = PfCfg<KT, D>;
    switch (wave) {
        case 0: pf_wait_n<C::ni_wave(0)>(pending); break;
        case 1: pf_wait_n<C::ni_wave(1)>(pending); break;
        case 2: pf_wait_n<C::ni_wave(2)>(pending); break;
        case 3: pf_wait_n<C::ni_wave(3)>(pending); break;
        case 4: pf_wait_n<C::ni_wave(4)>(pending); break;
        case 5: pf_wait_n<C::ni_wave(5)>(pending); break;
        case 6: pf_wait_n<C::ni_wave(6)>(pending); break;
        default: pf_wait_n<C::ni_wave(7)>(pending); break;
    }
}

// raw tile -> f16 images: thread t dequantises half block (t & 1) of block
// (t >> 1) % NB of row t / (2 NB), for K and for V
template <int KT, int D>
__device__ __forceinline__ void pf_dequant(const uint8_t* rb, uint8_t* k16, uint8_t* v16, int tid) {
#ifdef FATTN_MQ_NODEQ
    return;  // diagnostic build only
#endif
    using C = PfCfg<KT, D>;
    constexpr int NB = C::NB;
    const int row = tid / (2 * NB), b = (tid / 2) % NB, h = tid & 1;
    u32x4 ck[2], cv[2];
    dequant_half<KT, D>(rb, row, b, h, ck);
    dequant_half<KT, D>(rb + C::kvRaw, row, b, h, cv);
    const int c0 = 4 * b + 2 * h;
    uint8_t* kd = k16 + row * (D * 2);
    uint8_t* vd = v16 + row * (D * 2);
    *(u32x4*)(kd + ((c0 ^ (row & 15)) * 16)) = ck[0];
    *(u32x4*)(kd + (((c0 + 1) ^ (row & 15)) * 16)) = ck[1];
    *(u32x4*)(vd + ((c0 ^ (2 * (row & 3))) * 16)) = cv[0];
    *(u32x4*)(vd + (((c0 + 1) ^ (2 * (row & 3))) * 16)) = cv[1];
}

__device__ __forceinline__ f32x16 mfma32(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int KT, int D, bool HM>
__global__ __launch_bounds__(kPfWaves* kWave, 1) void fattn_pf_kernel(const SplitArgs a) {
    using C = PfCfg<KT, D>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NK = D / 16;   // 16-dim k-steps of S^T = K.Q^T
    constexpr int NDB = D / 32;  // 32-dim blocks of O^T
    constexpr float kNegInf = -__builtin_inff();
    constexpr float kDeferLog2 = 8.0f;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;      // k-group of the MFMA operands
    const int c32 = lane & 31;    // MFMA column: this lane's packed row within the wave

    // ---- tile decode: y -> (kv head, query tile); whole head groups (R = rk2)
    const int y = blockIdx.y;
    const int iq3 = blockIdx.z;
    int qt = 0, ik2 = y, ik3 = iq3;
    if (a.n_qt != 1) {
        qt = y % a.n_qt;
        ik2 = y / a.n_qt;
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;
    const int p = kPfRowsW * wave + c32;  // packed row
    const int mq = div_R(a, p);
    const int iq1 = qt * a.QPT + mq;
    const int iq2 = ik2 * a.rk2 + (p - mq * a.R);
    const bool row_ok = iq1 < a.NQ;
    const int ntiles = a.N / kPfKeys;

    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    auto raw = [&](int s) { return smem + (s % C::nRaw) * C::rawBytes; };
    auto k16_of = [&](int s) { return smem + C::imgOff + (s & 1) * 2 * C::img; };

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
            const f32x4 x0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(qs, qoff + 64 * kk, 0, 0));
            const f32x4 x1 =
                __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(qs, qoff + 64 * kk + 16, 0, 0));
            f16x8 hq;
            hq.s0 = (f16)x0.x; hq.s1 = (f16)x0.y; hq.s2 = (f16)x0.z; hq.s3 = (f16)x0.w;
            hq.s4 = (f16)x1.x; hq.s5 = (f16)x1.y; hq.s6 = (f16)x1.z; hq.s7 = (f16)x1.w;
            qop[kk] = hq;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- mask: this lane's keys of tile s are 32t + 8u + 4h + {0..3}
    // (u = 0..3): eight 8-B loads into registers, a tile ahead.  Issued as
    // inline asm (like the LDS-DMA): the compiler's own waits would otherwise
    // count them without the DMA behind them and drain the prefetch; the
    // explicit counted wait at the top of each tile covers them.
    const i32x4 msrd = make_srd(a.mask, HM ? a.m_span : 0);
    const uint32_t mrow = HM && row_ok ? (uint32_t)iq1 * (uint32_t)a.m_nb1 : (HM ? a.m_span : 0u);
    auto mask_issue = [&](int s, u32x2 (&mk)[2][4]) {
        if constexpr (HM) {
#pragma unroll
            for (int t = 0; t < 2; t++) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t off = row_ok ? mrow + (uint32_t)(s * kPfKeys + 32 * t + 8 * u + 4 * h) * 2 : mrow;
                    asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(mk[t][u]) : "v"(off), "s"(msrd) : "memory");
                }
            }
        }
    };
    // two register sets, alternating by tile parity (no copies of asm-loaded
    // registers before their wait)
    u32x2 mkA[2][4], mkB[2][4];
#pragma unroll
    for (int t = 0; t < 2; t++) {
#pragma unroll
        for (int u = 0; u < 4; u++) mkA[t][u] = mkB[t][u] = u32x2{0u, 0u};
    }

    // ---- prologue: mask 0, raw tiles 0..2; dequantise tile 0
    if (ntiles > 0) mask_issue(0, mkA);
    for (int s = 0; s < 3 && s < ntiles; s++) pf_issue<KT, D>(rs, s * kPfKeys, raw(s), wave, lane);
    // raw 0 and mask 0 landed; raw 1, 2 may still fly
    if (ntiles > 2) {
        switch (wave) {  // two DMA tiles younger than raw 0
            case 0: wait_vmcnt_c<2 * C::ni_wave(0)>(); break;
            case 1: wait_vmcnt_c<2 * C::ni_wave(1)>(); break;
            case 2: wait_vmcnt_c<2 * C::ni_wave(2)>(); break;
            case 3: wait_vmcnt_c<2 * C::ni_wave(3)>(); break;
            case 4: wait_vmcnt_c<2 * C::ni_wave(4)>(); break;
            case 5: wait_vmcnt_c<2 * C::ni_wave(5)>(); break;
            case 6: wait_vmcnt_c<2 * C::ni_wave(6)>(); break;
            default: wait_vmcnt_c<2 * C::ni_wave(7)>(); break;
        }
    } else {
        pf_wait<KT, D>(wave, ntiles - 1);
    }
    __syncthreads();
    if (ntiles > 0) pf_dequant<KT, D>(raw(0), k16_of(0), k16_of(0) + C::img, tid);

    float m_run = kNegInf;  // reference max (log2 domain) of this lane's row
    float l_run = 0.0f;     // this lane's partial row sum (its 32 of every 64 keys)
    f32x16 o[NDB];
#pragma unroll
    for (int db = 0; db < NDB; db++) {
#pragma unroll
        for (int j = 0; j < 16; j++) o[db][j] = 0.0f;
    }
    const float log2e = 1.4426950408889634f;

    auto body = [&](int s, u32x2 (&mk_cur)[2][4], u32x2 (&mk_next)[2][4]) {
        // raw s+1 and mask s landed (the youngest DMA tile, s+2, may fly on)
        pf_wait<KT, D>(wave, s + 2 < ntiles ? 1 : 0);
#pragma unroll
        for (int t = 0; t < 2; t++) {
#pragma unroll
            for (int u = 0; u < 4; u++) reg_fence(mk_cur[t][u]);
        }
        __syncthreads();
        if (s + 1 < ntiles) mask_issue(s + 1, mk_next);
        if (s + 3 < ntiles) pf_issue<KT, D>(rs, (s + 3) * kPfKeys, raw(s + 3), wave, lane);
        if (s + 1 < ntiles) pf_dequant<KT, D>(raw(s + 1), k16_of(s + 1), k16_of(s + 1) + C::img, tid);
#ifdef FATTN_MQ_NOCOMPUTE
        return;  // diagnostic build only: copies, dequant and barriers
#endif
        const uint8_t* k16 = k16_of(s);
        const uint8_t* v16 = k16 + C::img;

        // -- S^T = K.Q^T: two 32-key subtiles
        f32x16 st[2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
#pragma unroll
            for (int j = 0; j < 16; j++) st[t][j] = 0.0f;
            const int row = 32 * t + c32;
#pragma unroll
            for (int kk = 0; kk < NK; kk++) {
                const f16x8 ka = *(const f16x8*)(k16 + row * (D * 2) + (((2 * kk + h) ^ (row & 15)) * 16));
                st[t] = mfma32(ka, qop[kk], st[t]);
            }
        }

        // -- online softmax (log2 domain); element j of subtile t is key
        // 32t + 8(j/4) + 4h + (j%4) of this lane's row
        float sv[2][16];
#pragma unroll
        for (int t = 0; t < 2; t++) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                float mk[4] = {0.f, 0.f, 0.f, 0.f};
                if constexpr (HM) {
                    const f16x2 m01 = as_h2(mk_cur[t][u].x), m23 = as_h2(mk_cur[t][u].y);
                    mk[0] = (float)m01.x; mk[1] = (float)m01.y; mk[2] = (float)m23.x; mk[3] = (float)m23.y;
                }
#pragma unroll
                for (int r = 0; r < 4; r++) sv[t][4 * u + r] = st[t][4 * u + r] * a.scale_log2 + mk[r] * log2e;
            }
        }
#ifdef FATTN_PF_NOSOFTMAX
        // diagnostic build only: P = raw scores (MFMA + LDS reads, no softmax)
        f16x8 pb[2][2];
#pragma unroll
        for (int t = 0; t < 2; t++) {
#pragma unroll
            for (int q = 0; q < 2; q++) {
                f16x8 x;
#pragma unroll
                for (int i = 0; i < 8; i++) x[i] = (f16)sv[t][8 * q + i];
                pb[t][q] = x;
            }
        }
        l_run += 1.0f;
#else
        float tmax = kNegInf;
#pragma unroll
        for (int t = 0; t < 2; t++) {
#pragma unroll
            for (int j = 0; j < 16; j++) tmax = fmaxf(tmax, sv[t][j]);
        }
        tmax = xor32_pair(tmax, true);
        // deferred max (cdna_hip_programming.md T13), as in the multi-query kernel
        if (__builtin_amdgcn_ballot_w64(tmax > m_run + kDeferLog2)) {
            const float m_new = fmaxf(m_run, tmax);
            const float alpha = (m_new == kNegInf) ? 1.0f : __builtin_amdgcn_exp2f(m_run - m_new);
            l_run *= alpha;
#pragma unroll
            for (int db = 0; db < NDB; db++) o[db] *= alpha;
            m_run = m_new;
        }
        const float m_use = (m_run == kNegInf) ? 0.0f : m_run;
        f16x8 pb[2][2];
        float lsum = 0.0f;
#pragma unroll
        for (int t = 0; t < 2; t++) {
            float pv[16];
#pragma unroll
            for (int j = 0; j < 16; j++) {
                pv[j] = __builtin_amdgcn_exp2f(sv[t][j] - m_use);
                lsum += pv[j];
            }
#pragma unroll
            for (int q = 0; q < 2; q++) {
                f16x8 x;
                x.s0 = (f16)pv[8 * q]; x.s1 = (f16)pv[8 * q + 1]; x.s2 = (f16)pv[8 * q + 2]; x.s3 = (f16)pv[8 * q + 3];
                x.s4 = (f16)pv[8 * q + 4]; x.s5 = (f16)pv[8 * q + 5]; x.s6 = (f16)pv[8 * q + 6]; x.s7 = (f16)pv[8 * q + 7];
                pb[t][q] = x;
            }
        }
        l_run += lsum;
#endif

        // -- O^T += V^T.P^T: k-step (t, q) covers keys 32t + 16q + 8(i/4) + 4h + (i%4)
        // of k-group h (i = 0..7), V^T gathered in that order: 16-lane group
        // (h, dh) reads rows r0 + {0..3} (r0 = 32t + 16q + 4h, then + 8) x dims
        // 32db + 16dh + {0..15}; lane i of the group supplies row r0 + i/4, dims
        // + 4(i%4) .. + 3, and receives dim 32db + 16dh + i of the 4 rows
        const int gi = lane & 15, dh = (lane >> 4) & 1;
#pragma unroll
        for (int t = 0; t < 2; t++) {
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int r0 = 32 * t + 16 * q + 4 * h + (gi >> 2);
                const int r1 = r0 + 8;
#pragma unroll
                for (int db = 0; db < NDB; db++) {
                    const int ch = 4 * db + 2 * dh + ((gi & 3) >> 1);
                    const int a0 = r0 * (D * 2) + ((ch ^ (2 * (r0 & 3))) * 16) + (gi & 1) * 8;
                    const int a1 = r1 * (D * 2) + ((ch ^ (2 * (r1 & 3))) * 16) + (gi & 1) * 8;
                    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(v16 + a0));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(v16 + a1));
                    const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
                    const u32x4 r = {l2.x, l2.y, h2.x, h2.y};
                    o[db] = mfma32(__builtin_bit_cast(f16x8, r), pb[t][q], o[db]);
                }
            }
        }
    };
    for (int s = 0; s < ntiles; s += 2) {
        body(s, mkA, mkB);
        if (s + 1 < ntiles) body(s + 1, mkB, mkA);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    // ---- normalise and store: O^T element j of block db is dim
    // 32db + 8(j/4) + 4h + (j%4) of this lane's row
    const float l_tot = xor32_pair(l_run, false);
    if (row_ok) {
        float* out = a.dst + (((int64_t)iq3 * a.NQ + iq1) * a.H + iq2) * D + 4 * h;
        const float inv = 1.0f / l_tot;  // fully masked row -> NaN like the reference
#pragma unroll
        for (int db = 0; db < NDB; db++) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; r++) v[r] = l_tot == 0.0f ? __builtin_nanf("") : o[db][4 * u + r] * inv;
                *(f32x4*)(out + 32 * db + 8 * u) = v;
            }
        }
    }
}

}  // namespace fattn
