// fattn_pf2.h -- prefill over Q8_0 / Q4_0 KV with SIMD-partner ping-pong.
//
// Same math, tile shape and LDS images as fattn_pf_kernel (fattn_pf.h: 8 waves
// x 32 packed rows = 256 rows of one kv head, 64-key tiles, swapped products
// on v_mfma_f32_32x32x16_f16, K / V dequantised once per workgroup into f16
// images; src/flash-llama.h:5-438), but scheduled so that the two waves of a
// SIMD (w and w + 4) never want the same pipe at the same time.
//
// fattn_pf_kernel runs all 8 waves through one barrier per tile in lockstep:
// both waves of a SIMD issue their S^T MFMAs together, then both run the
// softmax on the VALU, then both P.V -- matrix and vector work of a SIMD add
// up instead of overlapping (PMC: 29 % of MFMA-busy cycles co-execute; stamps:
// ~4,870 cycles per tile against 2,048 of MFMA per SIMD).  Here every wave's
// tile work is cut into two segments,
//     X(j) = P.V of tile j-1 + S^T of tile j   (32 MFMAs, matrix pipe)
//     Y(j) = softmax of tile j + a dequantisation share (VALU)
// and the workgroup walks half-phases k separated by s_barrier: waves 0-3 (A)
// run X(j) at k = 2j and Y(j) at k = 2j + 1, waves 4-7 (B) one half-phase
// later, so in every half-phase each SIMD holds one matrix-bound and one
// vector-bound wave (MI355X_MICROARCH.md, two waves per SIMD: the tuned
// attention loop alternates roles between partners across s_barrier).
//
// Images (two of each, by tile parity): K(j) is read by A at k = 2j and by B at
// k = 2j + 1; V(j) by A at k = 2j + 2 and B at k = 2j + 3.  Dequantisation:
// B writes V(j) at k = 2j (its Y(j-1)), A writes K(j+1) at k = 2j + 1 (its
// Y(j)); each is four waves x one 32-element ggml block of every key row.
// Raw tiles: three in flight; raw(j) is free after k = 2j, so raw(j+3) is
// issued at k = 2j + 1 and needed at k = 2j + 5.  Masks: each wave reads its
// 32 x 64 mask block of tile j at k = 2j + 1 into registers and refills its
// slot with tile j + 1 at once (B keeps the registers to k = 2j + 2).
#pragma once

#include "fattn_pf.h"

namespace fattn {

// four waves dequantise one whole K or V tile: wave q takes ggml block q
// (both halves) of key row `lane`, into the image layouts of fattn_pf.h
template <int KT, int D, bool IS_V>
__device__ __forceinline__ void pf2_dequant(const uint8_t* raw, uint8_t* img, int q, int lane) {
#ifdef FATTN_MQ_NODEQ
    return;  // diagnostic build only
#endif
#pragma unroll
    for (int h = 0; h < 2; h++) {
        u32x4 c[2];
        dequant_half<KT, D>(raw, lane, q, h, c);
        if constexpr (!IS_V) {  // K image [8 dim slices][64 keys][32 B], halves swapped on rows with bit 3
            uint8_t* kd = img + (2 * q + h) * (kPfKeys * 32) + lane * 32;
            const int sk = (lane >> 3) & 1;
            *(u32x4*)(kd + sk * 16) = c[0];
            *(u32x4*)(kd + (sk ^ 1) * 16) = c[1];
        } else {  // V image [4 dim blocks][64 keys][64 B], chunk c of row r at c ^ ((r >> 2) & 3)
            uint8_t* vd = img + q * (kPfKeys * 64) + lane * 64;
            const int sv = (lane >> 2) & 3;
            *(u32x4*)(vd + ((2 * h) ^ sv) * 16) = c[0];
            *(u32x4*)(vd + ((2 * h + 1) ^ sv) * 16) = c[1];
        }
    }
}

template <int KT, int D, bool HM>
__global__ __launch_bounds__(kPfWaves* kWave, 1) void fattn_pf2_kernel(const SplitArgs a) {
    using C = PfCfg<KT, D>;
    static_assert(!C::kDirect, "quantised K/V only");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NK = D / 16;   // 16-dim k-steps of S^T = K.Q^T
    constexpr int NDB = D / 32;  // 32-dim blocks of O^T
    constexpr float kNegInf = -__builtin_inff();
    constexpr float kDeferLog2 = 8.0f;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2;  // 0: A (waves 0-3), 1: B (waves 4-7, one half-phase behind)
    const int wq = wave & 3;
    const int h = lane >> 5;      // k-group of the MFMA operands
    const int c32 = lane & 31;    // MFMA column: this lane's packed row within the wave

    // ---- tile decode (as fattn_pf_kernel): y -> (kv head, query tile)
    int y = blockIdx.y;
    const int iq3 = blockIdx.z;
    int qt = 0, ik2 = y, ik3 = iq3;
    if (a.pf_flags) {  // longest query tiles first
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
        return iq1 < a.NQ;
    };
    int iq1, iq2;
    const bool row_ok = row_of(kPfRowsW * wave + c32, iq1, iq2);
    // live KV tile range [t0, t0 + ntiles) of this query tile (pf_mask_flags_kernel)
    int t0 = 0, ntiles = a.N / kPfKeys;
    if (a.pf_flags) {
        const uint8_t* fl = a.pf_flags + (int64_t)qt * ntiles;
        int lo = ntiles, hi = -1;
        for (int b = 0; b < ntiles; b += kWave) {
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

    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    rs.m = make_srd(a.mask, HM ? a.m_span : 0);
    const uint32_t lds0 = lds_addr(smem);
    auto raw_lds = [&](int s) { return lds0 + C::rawOff + (s % 3) * C::rawBytes; };
    auto raw_ptr = [&](int s) { return smem + C::rawOff + (s % 3) * C::rawBytes; };
    auto kimg = [&](int s) { return smem + (s & 1) * C::pairBytes; };
    auto vimg = [&](int s) { return smem + (s & 1) * C::pairBytes + C::img; };
    const uint32_t mslot = lds0 + C::maskOff + wave * C::maskSlot;

    // ---- Q^T operands, rounded to f16 like src/utils.h:10; rows past n_q read zeros
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

    // ---- mask DMA (as fattn_pf_kernel): instruction k fills slot units 64k..64k+63
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
#ifndef FATTN_MQ_NOMEM
            const uint32_t n2 = (uint32_t)(t0 + s) * kPfKeys * 2;
#pragma unroll
            for (int k = 0; k < C::NIM; k++) {
                const uint32_t off = moff[k] == a.m_span ? a.m_span : moff[k] + n2;
                dma<16>(rs.m, mslot + k * 1024, off);
            }
#endif
        }
    };
    uint32_t maddr[2][4];
#pragma unroll
    for (int t = 0; t < 2; t++) {
#pragma unroll
        for (int u = 0; u < 4; u++)
            maddr[t][u] = C::maskOff + wave * C::maskSlot + (c32 * 8 + ((4 * t + u) ^ ((c32 >> 1) & 7))) * 16 + 8 * h;
    }
    // LDS read bases: K slice kk, row 32t + c32, half h; V^T gather (fattn_pf_kernel)
    const uint32_t kbase = c32 * 32 + ((h ^ ((c32 >> 3) & 1)) * 16);
    const int gi = lane & 15, dh = (lane >> 4) & 1;
    uint32_t vbase[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int row = 8 * e + 4 * h + (gi >> 2);
        const int ch = (2 * dh + ((gi & 3) >> 1)) ^ ((h + 2 * e) & 3);
        vbase[e] = row * 64 + ch * 16 + (gi & 1) * 8;
    }

    // counted waits: vmcnt counts this wave's DMA in issue order -- mask(j+1)
    // then raw(j+3) at half-phase 2j+1; the prologue issues mask(0), raw 0..2
    constexpr int NM = HM ? C::NIM : 0;
    auto wait_raw_fly = [&](bool one_raw_flying) {  // at most one raw tile (this wave's pieces) outstanding
        switch (wave) {
#define PF2_W(W)                                                                  \
    case W:                                                                       \
        if (one_raw_flying) wait_vmcnt_c<C::ni_wave(W)>(); else wait_vmcnt_c<0>(); \
        break;
            PF2_W(0) PF2_W(1) PF2_W(2) PF2_W(3) PF2_W(4) PF2_W(5) PF2_W(6)
            default:
                if (one_raw_flying) wait_vmcnt_c<C::ni_wave(7)>(); else wait_vmcnt_c<0>();
                break;
#undef PF2_W
        }
    };
    (void)NM;

    // ---- prologue: mask 0, raw 0..2 in flight; K(0) by the A waves
    if (ntiles > 0) mask_issue(0);
    for (int s = 0; s < 3 && s < ntiles; s++) pf_issue<KT, D>(rs, (t0 + s) * kPfKeys, raw_lds(s), wave, lane);
    // raw 0 landed (raw 1, raw 2 may fly on; mask 0 was issued before them)
    switch (min(2, max(ntiles - 1, 0))) {
        case 0: wait_vmcnt_c<0>(); break;
        case 1: wait_raw_fly(true); break;
        default:
            switch (wave) {
#define PF2_W2(W) case W: wait_vmcnt_c<2 * C::ni_wave(W)>(); break;
                PF2_W2(0) PF2_W2(1) PF2_W2(2) PF2_W2(3) PF2_W2(4) PF2_W2(5) PF2_W2(6)
                default: wait_vmcnt_c<2 * C::ni_wave(7)>(); break;
#undef PF2_W2
            }
    }
    __syncthreads();
    if (ntiles > 0 && grp == 0) pf2_dequant<KT, D, false>(raw_ptr(0), kimg(0), wq, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();

    float m_run = kNegInf;    // reference max (log2 domain) of this lane's row
    f32x2 l2 = {0.0f, 0.0f};  // this lane's partial row sums
    f32x16 o[NDB];
#pragma unroll
    for (int db = 0; db < NDB; db++) {
#pragma unroll
        for (int j = 0; j < 16; j++) o[db][j] = 0.0f;
    }
    const float log2e = 1.4426950408889634f;
    const float scale = a.scale_log2 / log2e;
    const float c = HM ? log2e : a.scale_log2;

    f32x16 st[2];           // S^T of the wave's current tile, then its scores u (X -> Y)
    f16x8 pb[2][2];         // P^T of the previous tile (Y -> X)
    bool live_p = false;    // the last mask-checked tile's block was not all -inf
    bool live_new = true;   // the block just read

    // X(j): P.V of tile j-1 (if any and live), then S^T of tile j (if any)
    auto seg_x = [&](int j) {
        if (j >= 1 && live_p) {
            const uint8_t* vi = vimg(j - 1);
#pragma unroll
            for (int t = 0; t < 2; t++) {
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
                    u32x4 va[NDB];
#pragma unroll
                    for (int db = 0; db < NDB; db++) {
                        const uint32_t off = db * (kPfKeys * 64) + t * 2048 + q * 1024;
                        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vi + vbase[0] + off));
                        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vi + vbase[1] + off));
                        const u32x2 a2 = __builtin_bit_cast(u32x2, lo), b2 = __builtin_bit_cast(u32x2, hi);
                        va[db] = u32x4{a2.x, a2.y, b2.x, b2.y};
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int db = 0; db < NDB; db++) o[db] = mfma32(__builtin_bit_cast(f16x8, va[db]), pb[t][q], o[db]);
                }
            }
        }
        if (j < ntiles) {
            const uint8_t* ki = kimg(j);
#pragma unroll
            for (int t = 0; t < 2; t++) {
                f16x8 ka[NK];
#pragma unroll
                for (int kk = 0; kk < NK; kk++) ka[kk] = *(const f16x8*)(ki + kbase + kk * (kPfKeys * 32) + t * 1024);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int jj = 0; jj < 16; jj++) st[t][jj] = 0.0f;
#pragma unroll
                for (int kk = 0; kk < NK; kk++) st[t] = mfma32(ka[kk], qop[kk], st[t]);
            }
        }
    };

    // scores in place: u = scale * s + mask (natural units; without a mask the
    // raw scores stay and the exponent's factor carries the scale).  The
    // mask block is read from the wave's slot, which is refilled with tile
    // j + 1 at once; live_new: the block has a key above -inf
    auto mask_scores = [&](int j) {
        live_new = true;
        if constexpr (HM) {
            u32x2 mk[2][4];
#pragma unroll
            for (int t = 0; t < 2; t++) {
#pragma unroll
                for (int uu = 0; uu < 4; uu++) mk[t][uu] = *(const u32x2*)(smem + maddr[t][uu]);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (j + 1 < ntiles) mask_issue(j + 1);
            uint32_t open = 0;  // any key not at -inf (f16 0xFC00)
#pragma unroll
            for (int t = 0; t < 2; t++) {
#pragma unroll
                for (int uu = 0; uu < 4; uu++) {
                    open |= (mk[t][uu].x ^ 0xFC00FC00u) | (mk[t][uu].y ^ 0xFC00FC00u);
                    const f16x2 m01 = as_h2(mk[t][uu].x), m23 = as_h2(mk[t][uu].y);
                    st[t][4 * uu + 0] = fmaf(st[t][4 * uu + 0], scale, (float)m01.x);
                    st[t][4 * uu + 1] = fmaf(st[t][4 * uu + 1], scale, (float)m01.y);
                    st[t][4 * uu + 2] = fmaf(st[t][4 * uu + 2], scale, (float)m23.x);
                    st[t][4 * uu + 3] = fmaf(st[t][4 * uu + 3], scale, (float)m23.y);
                }
            }
            live_new = __builtin_amdgcn_ballot_w64(open != 0) != 0;
        }
    };

    // Y: softmax of the scores in st -> pb; a block that is -inf for the
    // whole wave adds nothing (skipped: m, l, O untouched)
    auto seg_y = [&]() {
        if (!live_p) return;
        float tmax = kNegInf;
#pragma unroll
        for (int t = 0; t < 2; t++) {
#pragma unroll
            for (int jj = 0; jj < 16; jj++) tmax = fmaxf(tmax, st[t][jj]);
        }
        tmax = xor32_pair(tmax, true) * c;
        if (__builtin_amdgcn_ballot_w64(tmax > m_run + kDeferLog2)) {  // deferred max (T13)
            const float m_new = fmaxf(m_run, tmax);
            const float alpha = (m_new == kNegInf) ? 1.0f : __builtin_amdgcn_exp2f(m_run - m_new);
            l2 *= alpha;
#pragma unroll
            for (int db = 0; db < NDB; db++) o[db] *= alpha;
            m_run = m_new;
        }
        const float nm = (m_run == kNegInf) ? 0.0f : -m_run;
#pragma unroll
        for (int t = 0; t < 2; t++) {
            float pv[16];
#pragma unroll
            for (int jj = 0; jj < 16; jj++) pv[jj] = __builtin_amdgcn_exp2f(fmaf(st[t][jj], c, nm));
#pragma unroll
            for (int jj = 0; jj < 16; jj += 2) l2 += f32x2{pv[jj], pv[jj + 1]};
#pragma unroll
            for (int q = 0; q < 2; q++) {
                f16x8 x;
                x.s0 = (f16)pv[8 * q]; x.s1 = (f16)pv[8 * q + 1]; x.s2 = (f16)pv[8 * q + 2]; x.s3 = (f16)pv[8 * q + 3];
                x.s4 = (f16)pv[8 * q + 4]; x.s5 = (f16)pv[8 * q + 5]; x.s6 = (f16)pv[8 * q + 6]; x.s7 = (f16)pv[8 * q + 7];
                pb[t][q] = x;
            }
        }
    };

    // ---- half-phases k = 0 .. 2 ntiles + 1, two per loop iteration; the two
    // halves run separate loops (so that only the state one of them carries
    // across a barrier is live there: P^T for A, S^T for B) with the same
    // barrier count.  At odd k = 2j + 1 every wave refills its mask slot
    // (tile j + 1) and issues its pieces of raw tile j + 3.
#ifdef FATTN_STAMPS
    // diagnostic build only: shader-clock cycles per phase, summed over tiles
    // (tools/pf_stamps.py: 0 waits + barriers, 1 DMA issue, 2 dequant, 3 X (P.V + S^T), 4 Y (scores + softmax))
    uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t t_prev = __builtin_amdgcn_s_memtime();
    auto stamp = [&](int k) {
        const uint64_t t_ = __builtin_amdgcn_s_memtime();
        ph[k] += t_ - t_prev;
        t_prev = t_;
    };
    auto settle = [&] {  // results of the phase's MFMAs in registers before its stamp
        float z = st[0][0] + st[1][15];
#pragma unroll
        for (int db = 0; db < NDB; db++) z += o[db][0];
        asm volatile("" ::"v"(z));
    };
#else
    auto stamp = [&](int) {};
    auto settle = [&] {};
#endif
    auto end_even = [&](int j) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // mask(j) and raw(j+1) landed (A dequantises K(j+1) next); raw(j+2),
        // issued after mask(j), may fly on
        wait_raw_fly(j + 2 < ntiles);
        __syncthreads();
    };
    auto end_odd = [&] {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
    };
    auto refill = [&](int j) {  // after this wave's mask block of tile j is read
        if (j + 3 < ntiles) pf_issue<KT, D>(rs, (t0 + j + 3) * kPfKeys, raw_lds(j + 3), wave, lane);
    };
    if (ntiles > 0) {
        if (grp == 0) {
            for (int j = 0; j <= ntiles; j++) {
                seg_x(j);                      // k = 2j: P.V(j-1), S^T(j)
                settle();
                stamp(3);
                end_even(j);
                stamp(0);
                if (j < ntiles) {              // k = 2j + 1: softmax(j), K(j+1)
                    mask_scores(j);
                    refill(j);
                    stamp(1);
                    live_p = live_new;
                    seg_y();
                    stamp(4);
                    if (j + 1 < ntiles) pf2_dequant<KT, D, false>(raw_ptr(j + 1), kimg(j + 1), wq, lane);
                    stamp(2);
                }
                end_odd();
                stamp(0);
            }
        } else {
            for (int j = 0; j <= ntiles; j++) {
                if (j >= 1) seg_y();           // k = 2j: softmax(j-1), V(j)
                stamp(4);
                if (j < ntiles) pf2_dequant<KT, D, true>(raw_ptr(j) + C::kvRaw, vimg(j), wq, lane);
                stamp(2);
                end_even(j);
                stamp(0);
                seg_x(j);                      // k = 2j + 1: P.V(j-1), S^T(j)
                settle();
                stamp(3);
                if (j < ntiles) {
                    mask_scores(j);
                    refill(j);
                    live_p = live_new;
                    stamp(1);
                }
                end_odd();
                stamp(0);
            }
        }
    }
#ifdef FATTN_STAMPS
    if (lane == 0 && g_stamps) {
        const int64_t blk = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        for (int k = 0; k < 8; k++) g_stamps[(blk * kPfWaves + wave) * 16 + k] = ph[k];
        g_stamps[(blk * kPfWaves + wave) * 16 + 8] = (unsigned long long)ntiles;
    }
#endif
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    // ---- normalise and store (as fattn_pf_kernel)
    const float l_tot = xor32_pair(l2.x + l2.y, false);
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
