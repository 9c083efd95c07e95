// fattn_pf4.h -- prefill attention over ggml-quantised KV, one wave per SIMD.
//
// Same problem, planner conditions and LDS images as fattn_pf.h (replaces
// flash_attn_ext_f16, src/flash-llama.h:5-438, for long query blocks), but
// the 256 packed rows of a workgroup go to FOUR waves of 64 rows -- two
// 32-row blocks per wave -- so each SIMD runs one wave that owns every
// instruction stream on it.  With two independent row blocks a wave can put
// one block's VALU work beside the other block's MFMAs (cdna_hip_programming.md
// 'Fused attention prefill', the 4-wave one-wave-per-SIMD structure).  Per
// 64-key tile, between one workgroup barrier and the next:
//
//   R1  S^T(rb0)   16 MFMA   |  dequantise tile s+1 (block `wave` of 64 rows)
//       max(rb0), deferred rescale of rb0
//   R2  S^T(rb1)   16 MFMA   |  exponentials, row sums, P(rb0) -> f16
//       max(rb1), deferred rescale of rb1
//   R3  O^T(rb0)   16 MFMA   |  exponentials, row sums, P(rb1) -> f16
//   R4  O^T(rb1)   16 MFMA
//
// each region one basic block, its MFMAs and VALU interleaved by
// sched_group_barrier.  O^T (2 x 64 f32 per lane) lives in the accumulator
// registers next to everything else in the 512-register file.
#pragma once

#include "fattn_pf.h"

namespace fattn {

constexpr int kPf4Waves = 4;
constexpr int kPf4RowsW = 64;  // packed rows per wave (two 32-row blocks)

template <int KT, int D>
struct Pf4Cfg {
    using B = PfCfg<KT, D>;
    static constexpr int maskSlot = kPf4RowsW * 128;               // 64 rows x 64 keys x f16
    static constexpr int maskOff = B::rawOff + B::nRaw * B::rawBytes;
    static constexpr int ldsBytes = maskOff + kPf4Waves * maskSlot;
    static constexpr int NIM = maskSlot / 1024;
    // raw K/V DMA instructions j = 0 .. 2*NI-1 go to wave j % 4
    static constexpr int ni_wave(int w) { return (2 * B::NI - w + kPf4Waves - 1) / kPf4Waves; }
    static_assert(ldsBytes <= 163840, "");
};

template <int KT, int D>
__device__ __forceinline__ void pf4_issue(const StepSrc& rs, int n0, uint32_t lds, int wave, int lane) {
#ifdef FATTN_MQ_NOMEM
    return;  // diagnostic build only
#endif
    using C = PfCfg<KT, D>;
    for (int j = wave; j < 2 * C::NI; j += kPf4Waves) {  // wave-uniform
        const bool is_v = j >= C::NI;
        const int i = is_v ? j - C::NI : j;
        const int byte = i * 1024 + lane * 16;
        if (C::kvRaw % 1024 == 0 || byte < C::kvRaw)
            dma<16>(is_v ? rs.v : rs.k, lds + (is_v ? C::kvRaw : 0) + i * 1024, (uint32_t)n0 * C::rowB + byte);
    }
}

// at most `pending` (0..2) of this wave's raw-tile DMA groups still in flight
template <int KT, int D, int W>
__device__ __forceinline__ void pf4_wait_w(int pending) {
    constexpr int NI = Pf4Cfg<KT, D>::ni_wave(W);
    if (pending <= 0) {
        wait_vmcnt_c<0>();
    } else if (pending == 1) {
        wait_vmcnt_c<NI>();
    } else {
        wait_vmcnt_c<2 * NI>();
    }
}
template <int KT, int D>
__device__ __forceinline__ void pf4_wait(int wave, int pending) {
    switch (wave) {
        case 0: pf4_wait_w<KT, D, 0>(pending); break;
        case 1: pf4_wait_w<KT, D, 1>(pending); break;
        case 2: pf4_wait_w<KT, D, 2>(pending); break;
        default: pf4_wait_w<KT, D, 3>(pending); break;
    }
}

// raw tile -> f16 images: wave w dequantises ggml block w (both halves) of row
// `lane` for K (dim slices 2w, 2w+1) and V (dim block w)
template <int KT, int D>
__device__ __forceinline__ void pf4_dequant(const uint8_t* rb, uint8_t* k16, uint8_t* v16, int wave, int lane) {
#ifdef FATTN_MQ_NODEQ
    return;  // diagnostic build only
#endif
    using C = PfCfg<KT, D>;
    const int sk = (lane >> 3) & 1, sv = (lane >> 2) & 3;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        u32x4 ck[2], cv[2];
        dequant_half<KT, D>(rb, lane, wave, h, ck);
        dequant_half<KT, D>(rb + C::kvRaw, lane, wave, h, cv);
        uint8_t* kd = k16 + (2 * wave + h) * (kPfKeys * 32) + lane * 32;
        *(u32x4*)(kd + sk * 16) = ck[0];
        *(u32x4*)(kd + (sk ^ 1) * 16) = ck[1];
        uint8_t* vd = v16 + wave * (kPfKeys * 64) + lane * 64;
        *(u32x4*)(vd + ((2 * h) ^ sv) * 16) = cv[0];
        *(u32x4*)(vd + ((2 * h + 1) ^ sv) * 16) = cv[1];
    }
}

// ask the scheduler for N x {1 MFMA, V VALU, L DS} in this region
template <int N, int V, int L>
__device__ __forceinline__ void pf4_interleave() {
#ifdef FATTN_PF4_NO_SGB
    return;  // diagnostic build: compiler's own schedule
#endif
#pragma unroll
    for (int i = 0; i < N; i++) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, V, 0);  // VALU
        __builtin_amdgcn_sched_group_barrier(0x080, L, 0);  // DS
    }
}

template <int KT, int D, bool HM>
__global__ __launch_bounds__(kPf4Waves* kWave, 1) void fattn_pf4_kernel(const SplitArgs a) {
    using C = PfCfg<KT, D>;
    using C4 = Pf4Cfg<KT, D>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NK = D / 16;   // 16-dim k-steps of S^T = K.Q^T
    constexpr int NDB = D / 32;  // 32-dim blocks of O^T
    constexpr float kNegInf = -__builtin_inff();
    constexpr float kDeferLog2 = 8.0f;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = lane >> 5;      // k-group of the MFMA operands
    const int c32 = lane & 31;    // MFMA column: this lane's row within a 32-row block

    // ---- tile decode: y -> (kv head, query tile); whole head groups (R = rk2)
    const int y = blockIdx.y;
    const int iq3 = blockIdx.z;
    int qt = 0, ik2 = y, ik3 = iq3;
    if (a.n_qt != 1) {
        qt = y % a.n_qt;
        ik2 = y / a.n_qt;
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;
    auto row_of = [&](int p, int& iq1, int& iq2) {  // packed row -> (query row, q head)
        const int mq = div_R(a, p);
        iq1 = qt * a.QPT + mq;
        iq2 = ik2 * a.rk2 + (p - mq * a.R);
        return iq1 < a.NQ;
    };
    int iq1[2], iq2[2];
    bool row_ok[2];
#pragma unroll
    for (int rb = 0; rb < 2; rb++) row_ok[rb] = row_of(kPf4RowsW * wave + 32 * rb + c32, iq1[rb], iq2[rb]);
    const int ntiles = a.N / kPfKeys;

    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    rs.m = make_srd(a.mask, HM ? a.m_span : 0);
    const uint32_t lds0 = lds_addr(smem);
    auto raw_lds = [&](int s) { return lds0 + C::rawOff + (s % C::nRaw) * C::rawBytes; };
    auto raw_ptr = [&](int s) { return smem + C::rawOff + (s % C::nRaw) * C::rawBytes; };
    const uint32_t mslot = lds0 + C4::maskOff + wave * C4::maskSlot;

    // ---- Q^T operands of both row blocks, rounded to f16 like src/utils.h:10
    f16x8 qop[2][NK];
    {
        const auto qs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.q + (int64_t)iq3 * a.q_nb3), 0,
                                                          a.q_span, 0x00020000);
#pragma unroll
        for (int rb = 0; rb < 2; rb++) {
            const uint32_t qoff = row_ok[rb] ? (uint32_t)iq1[rb] * (uint32_t)a.q_nb1 +
                                                   (uint32_t)iq2[rb] * (uint32_t)a.q_nb2 + 32 * h
                                             : a.q_span;
#pragma unroll
            for (int kk = 0; kk < NK; kk++) {
                const f32x4 x0 =
                    __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(qs, qoff + 64 * kk, 0, 0));
                const f32x4 x1 =
                    __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(qs, qoff + 64 * kk + 16, 0, 0));
                f16x8 hq;
                hq.s0 = (f16)x0.x; hq.s1 = (f16)x0.y; hq.s2 = (f16)x0.z; hq.s3 = (f16)x0.w;
                hq.s4 = (f16)x1.x; hq.s5 = (f16)x1.y; hq.s6 = (f16)x1.z; hq.s7 = (f16)x1.w;
                qop[rb][kk] = hq;
            }
        }
    }

    // ---- mask DMA (as fattn_pf.h, 64 rows per wave): instruction k fills slot
    // units 64k .. 64k+63 = rows 8k + i/8, piece (i%8) ^ ((row >> 1) & 7)
    uint32_t moff[C4::NIM];
    if constexpr (HM) {
#pragma unroll
        for (int k = 0; k < C4::NIM; k++) {
            const int rr = 8 * k + (lane >> 3);
            int q1, q2;
            const bool ok = row_of(kPf4RowsW * wave + rr, q1, q2);
            const int pc = (lane & 7) ^ ((rr >> 1) & 7);
            moff[k] = ok ? (uint32_t)q1 * (uint32_t)a.m_nb1 + 16 * pc : a.m_span;
        }
    }
    auto mask_issue = [&](int s) {
        if constexpr (HM) {
#ifndef FATTN_MQ_NOMEM
            const uint32_t n2 = (uint32_t)s * kPfKeys * 2;
#pragma unroll
            for (int k = 0; k < C4::NIM; k++) {
                const uint32_t off = moff[k] == a.m_span ? a.m_span : moff[k] + n2;
                dma<16>(rs.m, mslot + k * 1024, off);
            }
#endif
        }
    };
    // mask reads: row 32rb + c32, piece 4t + u, half h (row block 1 at + 4 KiB)
    uint32_t maddr[2][4];
#pragma unroll
    for (int t = 0; t < 2; t++) {
#pragma unroll
        for (int u = 0; u < 4; u++)
            maddr[t][u] = C4::maskOff + wave * C4::maskSlot + (c32 * 8 + ((4 * t + u) ^ ((c32 >> 1) & 7))) * 16 + 8 * h;
    }

    // per-lane LDS read bases (image pair 0; pair 1 is + pairBytes); see fattn_pf.h
    const uint32_t kbase = c32 * 32 + ((h ^ ((c32 >> 3) & 1)) * 16);
    const int gi = lane & 15, dh = (lane >> 4) & 1;
    uint32_t vbase[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int row = 8 * e + 4 * h + (gi >> 2);
        const int ch = (2 * dh + ((gi & 3) >> 1)) ^ ((h + 2 * e) & 3);
        vbase[e] = C::img + row * 64 + ch * 16 + (gi & 1) * 8;
    }

    // ---- prologue: mask 0, raw tiles 0..2; dequantise tile 0
    if (ntiles > 0) mask_issue(0);
    for (int s = 0; s < 3 && s < ntiles; s++) pf4_issue<KT, D>(rs, s * kPfKeys, raw_lds(s), wave, lane);
    pf4_wait<KT, D>(wave, min(2, ntiles - 1));  // raw 0 and mask 0 landed
    __syncthreads();
    if (ntiles > 0) pf4_dequant<KT, D>(raw_ptr(0), smem, smem + C::img, wave, lane);

    float m_run[2] = {kNegInf, kNegInf};  // reference max (log2 domain) of this lane's rows
    f32x2 l2[2] = {{0.0f, 0.0f}, {0.0f, 0.0f}};
    f32x16 o[2][NDB];
#pragma unroll
    for (int rb = 0; rb < 2; rb++) {
#pragma unroll
        for (int db = 0; db < NDB; db++) {
#pragma unroll
            for (int j = 0; j < 16; j++) o[rb][db][j] = 0.0f;
        }
    }
    const float log2e = 1.4426950408889634f;
    const float scale = a.scale_log2 / log2e;
    const float c = HM ? log2e : a.scale_log2;  // exponent argument x * c - m (scale > 0)

    auto body = [&](int s, auto par) {
        constexpr int P = decltype(par)::value;  // image pair of tile s
        // raw s+1 and mask s landed (raw s+2 may fly on)
        pf4_wait<KT, D>(wave, s + 2 < ntiles ? 1 : 0);
        __syncthreads();
        const uint8_t* img = smem + P * C::pairBytes;  // K image; vbase includes + img

        // mask of tile s -> registers, then refill the slot with tile s+1
        u32x2 mk[2][2][4];
        if constexpr (HM) {
#pragma unroll
            for (int rb = 0; rb < 2; rb++) {
#pragma unroll
                for (int t = 0; t < 2; t++) {
#pragma unroll
                    for (int uu = 0; uu < 4; uu++) mk[rb][t][uu] = *(const u32x2*)(smem + maddr[t][uu] + rb * 4096);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (s + 1 < ntiles) mask_issue(s + 1);
        }
        if (s + 3 < ntiles) pf4_issue<KT, D>(rs, (s + 3) * kPfKeys, raw_lds(s + 3), wave, lane);

        // scores u = scale * s + mask (natural units; raw s without a mask)
        auto scores = [&](int rb, const f32x16 (&st)[2], float (&u)[2][16]) {
#pragma unroll
            for (int t = 0; t < 2; t++) {
#pragma unroll
                for (int uu = 0; uu < 4; uu++) {
                    if constexpr (HM) {
                        const f16x2 m01 = as_h2(mk[rb][t][uu].x), m23 = as_h2(mk[rb][t][uu].y);
                        u[t][4 * uu + 0] = fmaf(st[t][4 * uu + 0], scale, (float)m01.x);
                        u[t][4 * uu + 1] = fmaf(st[t][4 * uu + 1], scale, (float)m01.y);
                        u[t][4 * uu + 2] = fmaf(st[t][4 * uu + 2], scale, (float)m23.x);
                        u[t][4 * uu + 3] = fmaf(st[t][4 * uu + 3], scale, (float)m23.y);
                    } else {
#pragma unroll
                        for (int r = 0; r < 4; r++) u[t][4 * uu + r] = st[t][4 * uu + r];
                    }
                }
            }
        };
        auto s_tile = [&](int rb, f32x16 (&st)[2]) {
#pragma unroll
            for (int t = 0; t < 2; t++) {
#pragma unroll
                for (int j = 0; j < 16; j++) st[t][j] = 0.0f;
#pragma unroll
                for (int kk = 0; kk < NK; kk++) {
                    const f16x8 ka = *(const f16x8*)(img + kbase + kk * (kPfKeys * 32) + t * 1024);
                    st[t] = mfma32(ka, qop[rb][kk], st[t]);
                }
            }
        };
        // row max and the deferred rescale (cdna_hip_programming.md T13)
        auto max_rescale = [&](int rb, const float (&u)[2][16]) {
            float tmax = kNegInf;
#pragma unroll
            for (int t = 0; t < 2; t++) {
#pragma unroll
                for (int j = 0; j < 16; j++) tmax = fmaxf(tmax, u[t][j]);
            }
            tmax = xor32_pair(tmax, true) * c;
            if (__builtin_amdgcn_ballot_w64(tmax > m_run[rb] + kDeferLog2)) {
                const float m_new = fmaxf(m_run[rb], tmax);
                const float alpha = (m_new == kNegInf) ? 1.0f : __builtin_amdgcn_exp2f(m_run[rb] - m_new);
                l2[rb] *= alpha;
#pragma unroll
                for (int db = 0; db < NDB; db++) o[rb][db] *= alpha;
                m_run[rb] = m_new;
            }
        };
        auto exps = [&](int rb, const float (&u)[2][16], f16x8 (&pb)[2][2]) {
            const float nm = (m_run[rb] == kNegInf) ? 0.0f : -m_run[rb];
#pragma unroll
            for (int t = 0; t < 2; t++) {
                float pv[16];
#pragma unroll
                for (int j = 0; j < 16; j++) pv[j] = __builtin_amdgcn_exp2f(fmaf(u[t][j], c, nm));
#pragma unroll
                for (int j = 0; j < 16; j += 2) l2[rb] += f32x2{pv[j], pv[j + 1]};
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    f16x8 x;
                    x.s0 = (f16)pv[8 * q]; x.s1 = (f16)pv[8 * q + 1]; x.s2 = (f16)pv[8 * q + 2]; x.s3 = (f16)pv[8 * q + 3];
                    x.s4 = (f16)pv[8 * q + 4]; x.s5 = (f16)pv[8 * q + 5]; x.s6 = (f16)pv[8 * q + 6]; x.s7 = (f16)pv[8 * q + 7];
                    pb[t][q] = x;
                }
            }
        };
        // O^T += V^T.P^T (k-step (t, q): keys 32t + 16q + 8(i/4) + 4h + (i%4))
        auto o_tile = [&](int rb, const f16x8 (&pb)[2][2]) {
#pragma unroll
            for (int t = 0; t < 2; t++) {
#pragma unroll
                for (int q = 0; q < 2; q++) {
#pragma unroll
                    for (int db = 0; db < NDB; db++) {
                        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
                        const uint32_t off = db * (kPfKeys * 64) + t * 2048 + q * 1024;
                        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + vbase[0] + off));
                        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + vbase[1] + off));
                        const u32x2 a2 = __builtin_bit_cast(u32x2, lo), b2 = __builtin_bit_cast(u32x2, hi);
                        const u32x4 r = {a2.x, a2.y, b2.x, b2.y};
                        o[rb][db] = mfma32(__builtin_bit_cast(f16x8, r), pb[t][q], o[rb][db]);
                    }
                }
            }
        };

        // R1: S^T(rb0) beside the dequantisation of tile s+1 (past the last
        // tile it converts stale bytes into an image nobody reads)
        f32x16 st0[2], st1[2];
        s_tile(0, st0);
        pf4_dequant<KT, D>(raw_ptr(s + 1), smem + (P ^ 1) * C::pairBytes, smem + (P ^ 1) * C::pairBytes + C::img,
                           wave, lane);
        pf4_interleave<16, 6, 2>();
        float u0[2][16];
        scores(0, st0, u0);
        max_rescale(0, u0);
        // R2: S^T(rb1) beside P(rb0)
        f16x8 pb0[2][2];
        s_tile(1, st1);
        exps(0, u0, pb0);
        pf4_interleave<16, 6, 1>();
        float u1[2][16];
        scores(1, st1, u1);
        max_rescale(1, u1);
        // R3: O^T(rb0) beside P(rb1)
        f16x8 pb1[2][2];
        o_tile(0, pb0);
        exps(1, u1, pb1);
        pf4_interleave<16, 6, 2>();
        // R4: O^T(rb1)
        o_tile(1, pb1);
    };
    for (int s = 0; s < ntiles; s += 2) {
        body(s, std::integral_constant<int, 0>());
        if (s + 1 < ntiles) body(s + 1, std::integral_constant<int, 1>());
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    // ---- normalise and store: O^T element j of block db is dim
    // 32db + 8(j/4) + 4h + (j%4) of this lane's row
#pragma unroll
    for (int rb = 0; rb < 2; rb++) {
        const float l_tot = xor32_pair(l2[rb].x + l2[rb].y, false);
        if (row_ok[rb]) {
            float* out = a.dst + (((int64_t)iq3 * a.NQ + iq1[rb]) * a.H + iq2[rb]) * D + 4 * h;
            const float inv = 1.0f / l_tot;  // fully masked row -> NaN like the reference
#pragma unroll
            for (int db = 0; db < NDB; db++) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    f32x4 v;
#pragma unroll
                    for (int r = 0; r < 4; r++) v[r] = l_tot == 0.0f ? __builtin_nanf("") : o[rb][db][4 * u + r] * inv;
                    *(f32x4*)(out + 32 * db + 8 * u) = v;
                }
            }
        }
    }
}

}  // namespace fattn
