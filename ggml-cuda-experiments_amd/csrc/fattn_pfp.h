// fattn_pfp.h -- software-pipelined prefill kernel over f16 K/V images
// (f16 K/V caches directly; Q8_0 / Q4_0 after pf_dequant_rows_kernel).
//
// Same tile, layouts and math as fattn_pf_kernel (fattn_pf.h: 8 waves x 32
// packed rows, 64-key tiles, swapped products on v_mfma_f32_32x32x16_f16,
// deferred-max online softmax), but each wave runs its softmax BESIDE its own
// MFMAs instead of between them.  Per tile s, two phases of 16 MFMAs each:
//
//   phase A:  S^T(s+1) = K(s+1).Q^T      ||  finish softmax(s): p = exp2(u c - m),
//                                             row sums, P(s) -> f16
//   phase B:  O^T += V(s)^T.P(s)^T       ||  start softmax(s+1): mask(s+1),
//                                             u = scale s + mask, row max,
//                                             deferred rescale
//
// so the VALU work (about 24 cycles of issue per MFMA gap, MI355X_MICROARCH.md
// 'Per-instruction cycle constants') fills the gaps of the wave's own MFMA
// stream rather than alternating with it.  The K image of tile s+1 and the V
// image of tile s are read in the same body, hence a 4-deep image ring (tile
// s+1 read, s+2 and s+3 in flight): 4 x 32 KiB + 8 mask slots x 4 KiB = 160 KiB.
//
// Replaces flash_attn_ext_f16<D,Q,C> (src/flash-llama.h:5-438) for long query
// blocks, like fattn_pf_kernel; results are the same math in the same
// accumulation order per element (S^T chains, then P.V k-steps in order), so
// the two kernels agree to rounding of the exp2 argument only.
#pragma once

#include "fattn_pf.h"

namespace fattn {

struct PfpCfg {
    using C = PfCfg<FATTN_TYPE_F16, 128>;
    static constexpr int nPairs = 4;
    static constexpr int maskOff = nPairs * C::pairBytes;           // 128 KiB
    static constexpr int ldsBytes = maskOff + kPfWaves * C::maskSlot;
    static_assert(ldsBytes <= 163840, "");
};

#ifndef FATTN_PFP_FILL_A
#define FATTN_PFP_FILL_A 6   // VALU fillers placed per S^T MFMA (phase A)
#endif
#ifndef FATTN_PFP_AHEAD_A
#define FATTN_PFP_AHEAD_A 2  // K reads placed before the first S^T MFMA (then 1 per MFMA)
#endif
#ifndef FATTN_PFP_AHEAD_B
#define FATTN_PFP_AHEAD_B 4  // V^T reads placed before the first O^T MFMA (then 2 per MFMA)
#endif
#ifndef FATTN_PFP_FILL_B
#define FATTN_PFP_FILL_B 4   // VALU fillers placed per O^T MFMA (phase B)
#endif

template <bool HM>
__global__ __launch_bounds__(kPfWaves* kWave, 1) void fattn_pfp_kernel(const SplitArgs a) {
    constexpr int D = 128;
    using C = PfCfg<FATTN_TYPE_F16, D>;
    using PC = PfpCfg;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NK = D / 16;   // 16-dim k-steps of S^T = K.Q^T
    constexpr int NDB = D / 32;  // 32-dim blocks of O^T
    constexpr int NM = HM ? 1 : 0;
    constexpr float kNegInf = -__builtin_inff();
    constexpr float kDeferLog2 = 8.0f;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (a.pf_stagger & 2) {
        if (wave >= kPfWaves / 2) __builtin_amdgcn_s_setprio(1);
    }
    const int h = lane >> 5;
    const int c32 = lane & 31;

    int y = blockIdx.y;
    if ((a.pf_stagger & 4) && gridDim.y % 8 == 0) y = (y & 7) * (gridDim.y >> 3) + (y >> 3);
    const int iq3 = blockIdx.z;
    int qt = 0, ik2 = y, ik3 = iq3;
    if (a.n_qt != 1) {
        qt = y % a.n_qt;
        ik2 = y / a.n_qt;
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;
    auto row_of = [&](int p, int& iq1, int& iq2) {
        const int mq = div_R(a, p);
        iq1 = qt * a.QPT + mq;
        iq2 = ik2 * a.rk2 + (p - mq * a.R);
        return iq1 < a.NQ;
    };
    int iq1, iq2;
    const bool row_ok = row_of(kPfRowsW * wave + c32, iq1, iq2);
    const int ntiles = a.N / kPfKeys;

    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    rs.m = make_srd(a.mask, HM ? a.m_span : 0);
    const uint32_t lds0 = lds_addr(smem);
    const uint32_t mslot = lds0 + PC::maskOff + wave * C::maskSlot;

    // Q^T operands, rows past n_q read zeros (as fattn_pf_kernel)
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

    // mask DMA and read addresses (fattn_pf_kernel's, slot base moved)
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
    auto mask_issue = [&](int s) {
        if constexpr (HM) {
            const uint32_t n2 = (uint32_t)s * kPfKeys * 2;
#pragma unroll
            for (int k = 0; k < C::NIM; k++) {
                const uint32_t off = moff[k] == a.m_span ? a.m_span : moff[k] + n2;
                dma<16>(rs.m, mslot + k * 1024, off);
            }
        }
    };
    // this lane's mask piece pc = 4t + u of row c32 sits at mrow + ((pc ^ msw) * 16)
    const uint32_t mrow = PC::maskOff + wave * C::maskSlot + c32 * 128 + 8 * h;
    const uint32_t msw = ((c32 >> 1) & 7) * 16;
    const uint32_t kbase = c32 * 32 + ((h ^ ((c32 >> 3) & 1)) * 16);
    const int gi = lane & 15, dh = (lane >> 4) & 1;
    uint32_t vbase[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int row = 8 * e + 4 * h + (gi >> 2);
        const int ch = (2 * dh + ((gi & 3) >> 1)) ^ ((h + 2 * e) & 3);
        vbase[e] = C::img + row * 64 + ch * 16 + (gi & 1) * 8;
    }
    uint32_t doff[4];
    pf_direct_offsets<D>(a, wave, lane, doff);

    const float log2e = 1.4426950408889634f;
    const float scale = a.scale_log2 / log2e;
    const float c = HM ? log2e : a.scale_log2;  // exponent argument = u c - m (log2 domain)

    float m_run = kNegInf;
    float nm = 0.0f;
    f32x2 l2 = {0.0f, 0.0f};
    f32x16 o[NDB];
#pragma unroll
    for (int db = 0; db < NDB; db++) {
#pragma unroll
        for (int j = 0; j < 16; j++) o[db][j] = 0.0f;
    }
    // The pipeline runs over 32-key subtiles j = 2s + t of the 64-key tiles s
    // (half the live score / P state of whole tiles: no spills).
    float u[16];     // scores of the subtile whose softmax is half done
    u32x2 mk1[4];    // mask pieces of the odd subtile of the current tile

    // -- S^T of subtile t of the tile in image `img`
    auto s_sub = [&](const uint8_t* img, int t, f32x16& st) {
#pragma unroll
        for (int j = 0; j < 16; j++) st[j] = 0.0f;
#pragma unroll
        for (int kk = 0; kk < NK; kk++)
            st = mfma32(*(const f16x8*)(img + kbase + kk * (kPfKeys * 32) + t * 1024), qop[kk], st);
    };
    // -- read both subtiles' mask pieces of a tile (landed), then refill the
    //    slot with the next tile's mask
    auto sm_mask = [&](int s, u32x2 (&mk0)[4]) {
        if constexpr (HM) {
#pragma unroll
            for (int uu = 0; uu < 4; uu++) mk0[uu] = *(const u32x2*)(smem + mrow + ((uu * 16) ^ msw));
#pragma unroll
            for (int uu = 0; uu < 4; uu++) mk1[uu] = *(const u32x2*)(smem + mrow + (((4 + uu) * 16) ^ msw));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (s + 1 < ntiles) mask_issue(s + 1);
        }
    };
    // -- scores u = scale s + mask and their max (element j: key 8(j/4) + 4h + j%4)
    auto sm_scores = [&](const f32x16& st, const u32x2 (&mk)[4]) {
        if constexpr (HM) {
#pragma unroll
            for (int uu = 0; uu < 4; uu++) {
                const f16x2 m01 = as_h2(mk[uu].x), m23 = as_h2(mk[uu].y);
                u[4 * uu + 0] = fmaf(st[4 * uu + 0], scale, (float)m01.x);
                u[4 * uu + 1] = fmaf(st[4 * uu + 1], scale, (float)m01.y);
                u[4 * uu + 2] = fmaf(st[4 * uu + 2], scale, (float)m23.x);
                u[4 * uu + 3] = fmaf(st[4 * uu + 3], scale, (float)m23.y);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++) u[j] = st[j];
        }
        float tmax = kNegInf;
#pragma unroll
        for (int j = 0; j < 16; j++) tmax = fmaxf(tmax, u[j]);
        return tmax;
    };
    auto sm_rescale = [&](float tmax) {
        tmax = xor32_pair(tmax, true) * c;
        if (__builtin_amdgcn_ballot_w64(tmax > m_run + kDeferLog2)) {
            const float m_new = fmaxf(m_run, tmax);
            const float alpha = (m_new == kNegInf) ? 1.0f : __builtin_amdgcn_exp2f(m_run - m_new);
            l2 *= alpha;
#pragma unroll
            for (int db = 0; db < NDB; db++) o[db] *= alpha;
            m_run = m_new;
        }
        nm = (m_run == kNegInf) ? 0.0f : -m_run;
    };
    // -- finish softmax of the started subtile: P (f16, two 16-key k-steps) and row sums
    auto sm_finish = [&](f16x8 (&pb)[2]) {
        float pv[16];
#pragma unroll
        for (int j = 0; j < 16; j++) pv[j] = __builtin_amdgcn_exp2f(fmaf(u[j], c, nm));
#pragma unroll
        for (int j = 0; j < 16; j += 2) l2 += f32x2{pv[j], pv[j + 1]};
#pragma unroll
        for (int q = 0; q < 2; q++) {
            f16x8 x;
            x.s0 = (f16)pv[8 * q]; x.s1 = (f16)pv[8 * q + 1]; x.s2 = (f16)pv[8 * q + 2]; x.s3 = (f16)pv[8 * q + 3];
            x.s4 = (f16)pv[8 * q + 4]; x.s5 = (f16)pv[8 * q + 5]; x.s6 = (f16)pv[8 * q + 6]; x.s7 = (f16)pv[8 * q + 7];
            pb[q] = x;
        }
    };
    // -- O^T += V^T.P^T for subtile t of the tile in image `img`
    auto o_sub = [&](const uint8_t* img, int t, const f16x8 (&pb)[2]) {
#pragma unroll
        for (int q = 0; q < 2; q++) {
            typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
            u32x4 va[NDB];
#pragma unroll
            for (int db = 0; db < NDB; db++) {
                const uint32_t off = db * (kPfKeys * 64) + t * 2048 + q * 1024;
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + vbase[0] + off));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + vbase[1] + off));
                const u32x2 a2 = __builtin_bit_cast(u32x2, lo), b2 = __builtin_bit_cast(u32x2, hi);
                va[db] = u32x4{a2.x, a2.y, b2.x, b2.y};
            }
#pragma unroll
            for (int db = 0; db < NDB; db++) o[db] = mfma32(__builtin_bit_cast(f16x8, va[db]), pb[q], o[db]);
        }
    };
    // per phase: `ahead` LDS reads first, then 8 x {MFMA, `per` LDS reads, F VALU}
    [[maybe_unused]] auto interleave = [](auto nfill, auto ahead, auto per, auto id) {
        constexpr int F = decltype(nfill)::value, A = decltype(ahead)::value, R = decltype(per)::value;
        constexpr int I = decltype(id)::value;
        __builtin_amdgcn_sched_group_barrier(0x100, A, I);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, I);
            __builtin_amdgcn_sched_group_barrier(0x100, R, I);
            __builtin_amdgcn_sched_group_barrier(0x002, F, I);
        }
    };

    // ---- prologue: image 0 and mask 0 (waited), images 1, 2 in flight;
    // S^T(subtile 0), start softmax(subtile 0)
    if (ntiles > 0) pf_direct_issue<D>(a, rs, 0, lds0, wave, doff);
    if (ntiles > 0) mask_issue(0);
    for (int s = 1; s < 3 && s < ntiles; s++) pf_direct_issue<D>(a, rs, s * kPfKeys, lds0 + s * C::pairBytes, wave, doff);
    pf_vm_wait<FATTN_TYPE_F16, D>(wave, min(2, max(0, ntiles - 1)), 0);
    __syncthreads();
    const int nsub = 2 * ntiles;
    if (ntiles > 0) {
        f32x16 st;
        s_sub(smem, 0, st);
        u32x2 mk0[4];
        sm_mask(0, mk0);
        sm_rescale(sm_scores(st, mk0));
    }

    auto body = [&](int j, auto par) {
        constexpr int J = decltype(par)::value;  // j mod 8
        constexpr int T = J & 1, P = (J >> 1) & 3;  // subtile of tile s = j / 2, its ring slot
        constexpr int PN = ((J + 1) >> 1) & 3;      // ring slot of subtile j + 1
        const int s = j >> 1;
        if constexpr (T == 1) {
            // image s+1 landed (image s+2 and mask s+1 may fly on); every wave is
            // past tile s-1, so its slot (P + 3) % 4 takes image s+3
            pf_vm_wait<FATTN_TYPE_F16, D>(wave, s + 2 < ntiles ? 1 : 0, s + 1 < ntiles ? NM : 0);
            __syncthreads();
            if (s + 3 < ntiles)
                pf_direct_issue<D>(a, rs, (s + 3) * kPfKeys, lds0 + ((P + 3) % 4) * C::pairBytes, wave, doff);
        }
        const uint8_t* img_s = smem + P * C::pairBytes;
        const uint8_t* img_n = smem + PN * C::pairBytes;
        f16x8 pb[2];
        f32x16 st;
        const bool more = j + 1 < nsub;
        // phase A: S^T(j+1) || finish softmax(j)
        if (more) {
            s_sub(img_n, T ^ 1, st);
            sm_finish(pb);
#ifndef FATTN_PFP_NO_SGB
            interleave(std::integral_constant<int, FATTN_PFP_FILL_A>(), std::integral_constant<int, FATTN_PFP_AHEAD_A>(),
                       std::integral_constant<int, 1>(), std::integral_constant<int, 0>());
#endif
        } else {
            sm_finish(pb);
        }
        // phase B: O^T(j) || start softmax(j+1)
        if (more) {
            u32x2 mk[4];
            if constexpr (T == 1) {
                // subtile j+1 opens tile s+1: its mask landed (image s+3 may fly on)
                if constexpr (HM) pf_vm_wait<FATTN_TYPE_F16, D>(wave, s + 3 < ntiles ? 1 : 0, 0);
                sm_mask(s + 1, mk);
            } else {
#pragma unroll
                for (int uu = 0; uu < 4; uu++) mk[uu] = mk1[uu];
            }
            o_sub(img_s, T, pb);
            const float tmax = sm_scores(st, mk);
#ifndef FATTN_PFP_NO_SGB
            interleave(std::integral_constant<int, FATTN_PFP_FILL_B>(), std::integral_constant<int, FATTN_PFP_AHEAD_B>(),
                       std::integral_constant<int, 2>(), std::integral_constant<int, 1>());
#endif
            sm_rescale(tmax);
        } else {
            o_sub(img_s, T, pb);
        }
    };
    for (int j = 0; j < nsub; j += 8) {
        body(j, std::integral_constant<int, 0>());
        if (j + 1 < nsub) body(j + 1, std::integral_constant<int, 1>());
        if (j + 2 < nsub) body(j + 2, std::integral_constant<int, 2>());
        if (j + 3 < nsub) body(j + 3, std::integral_constant<int, 3>());
        if (j + 4 < nsub) body(j + 4, std::integral_constant<int, 4>());
        if (j + 5 < nsub) body(j + 5, std::integral_constant<int, 5>());
        if (j + 6 < nsub) body(j + 6, std::integral_constant<int, 6>());
        if (j + 7 < nsub) body(j + 7, std::integral_constant<int, 7>());
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    const float l_tot = xor32_pair(l2.x + l2.y, false);
    if (row_ok) {
        float* out = a.dst + (((int64_t)iq3 * a.NQ + iq1) * a.H + iq2) * D + 4 * h;
        const float inv = 1.0f / l_tot;
#pragma unroll
        for (int db = 0; db < NDB; db++) {
#pragma unroll
            for (int uu = 0; uu < 4; uu++) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; r++) v[r] = l_tot == 0.0f ? __builtin_nanf("") : o[db][4 * uu + r] * inv;
                *(f32x4*)(out + 32 * db + 8 * uu) = v;
            }
        }
    }
}

}  // namespace fattn
