// fattn_dec.h -- split-KV decode with dedicated loader waves (gfx950).
//
// Same math and the same per-step body as fattn_split_kernel (split_step: the
// flash_attn_row / flash_attn_ext_f16 step of src/flash_row_float.h:4-200 and
// src/flash-llama.h:162-337, merged like fa_reduce, src/flash_row_float.h:
// 415-472), but the HBM stream no longer waits on the compute:
//
//  * A workgroup = 4 compute waves (one per SIMD) + NLW loader waves.  The
//    loaders issue the chunk's K / mask / V steps into an LDS ring of `nslot`
//    step images with global_load_lds_dwordx4 (nt), as far ahead as their
//    vmcnt allows, and publish each landed step by a FULL word in LDS (the
//    issuing wave's counted vmcnt, then a ds_write -- MI355X_MICROARCH.md,
//    'ldsdma-fill' / 'ring-gemm').  With the decode shapes a chunk's whole
//    K/V slice fits the ring (config 3: 16 steps, 155 KB), so every byte of a
//    CU's slice is requested at kernel start and the CU keeps ~100 KB in
//    flight -- the split kernel, whose waves issue their own steps, stalled
//    compute behind issue and capped MLP at two steps per wave.
//  * Step s goes to compute wave s % 4, which polls FULL[slot] (s_sleep), runs
//    split_step on the image and, when the ring wraps, frees the slot with a
//    FREE word.  The last steps to land are spread over all four compute
//    waves, so the exposed tail is one step's compute.
//  * The epilogue is split_epilogue: one-row tiles publish per wave and the
//    last-arriving wave merges; other tiles merge the 4 waves through LDS and
//    the chunks through the last-arriving workgroup (combine_tile).
#pragma once

#include "fattn_split.h"

namespace fattn {

constexpr int kDecCompute = kSplitWaves;  // compute waves per workgroup (default; 8 = two per SIMD)
constexpr int kDecHdr = 256;              // LDS header: FULL[32], FREE[32] words
constexpr int kDecMaxSlots = 32;

// steps one loader keeps in flight (vmcnt is 6 bits: <= 63 instructions)
template <int NI>
constexpr int dec_ahead() {
    return 63 / NI < 1 ? 1 : (63 / NI > 8 ? 8 : 63 / NI);
}

template <int NI>
__device__ __forceinline__ void dec_wait_steps(int outstanding) {
    switch (__builtin_amdgcn_readfirstlane(outstanding)) {
        case 0: wait_vmcnt_c<0>(); break;
        case 1: wait_vmcnt_c<NI>(); break;
        case 2: wait_vmcnt_c<2 * NI>(); break;
        case 3: wait_vmcnt_c<3 * NI>(); break;
        case 4: wait_vmcnt_c<4 * NI>(); break;
        case 5: wait_vmcnt_c<5 * NI>(); break;
        case 6: wait_vmcnt_c<6 * NI>(); break;
        default: wait_vmcnt_c<7 * NI>(); break;
    }
}

// slot of step s: loader l = s % nlw owns slots l, l + nlw, ... (its own ring
// of nslot / nlw), so a loader's FREE waits depend on its own steps only
__device__ __forceinline__ int dec_slot(int s, int nlw, int spl) {
    return nlw == 1 ? s % spl : (s & 1) + ((s >> 1) % spl) * 2;
}

template <int KT, int VT, int D, bool HM, int NLW, int NCW>
__global__ __launch_bounds__((NCW + NLW) * kWave, 1) void fattn_dec_kernel(const SplitArgs a) {
    using C = SplitCfg<KT, VT, D>;
    using P = StepPlan<KT, VT, D, 16>;
    constexpr int NI = P::NIKV + (HM ? P::NIM : 0);  // VMEM instructions per step
    constexpr int AH = dec_ahead<NI>();
    constexpr int NB = D / QK;
    constexpr int NC = D / 16;
    constexpr float kNegInf = -__builtin_inff();
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    volatile uint32_t* full = (volatile uint32_t*)smem;
    volatile uint32_t* freew = full + kDecMaxSlots;
    uint8_t* slots = smem + kDecHdr;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4;
    const int i16 = lane & 15;
    FATTN_STAMP8(0);

    // ---- tile decode: y -> (kv head, head subgroup, query-row tile), as fattn_split_kernel
    const int chunk = blockIdx.x;
    const int y = blockIdx.y;
    const int iq3 = blockIdx.z;
    int qt = 0, hs = 0, ik2 = y, ik3 = iq3;
    if (a.n_qt != 1 || a.n_hsub != 1) {
        qt = y % a.n_qt;
        hs = (y / a.n_qt) % a.n_hsub;
        ik2 = y / (a.n_qt * a.n_hsub);
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;

    const int c_lo = chunk * a.chunk_len;
    const int c_hi = min(a.N, c_lo + a.chunk_len);
    const int ns = (c_hi - c_lo + kStep - 1) / kStep;  // steps of this chunk
    const int nslot = a.nbuf;
    const int spl = nslot / NLW;                        // slots per loader
    const bool ring = ns > nslot;
    const int mrow0 = qt * a.QPT;

    // FULL / FREE words hold step index + 1 of the last publish: clear them
    // (LDS keeps a previous workgroup's bytes)
    if (threadIdx.x < 2 * kDecMaxSlots) full[threadIdx.x] = 0;
    __syncthreads();

    if (wave >= NCW) {
        // ================= loader wave lw: steps lw, lw + NLW, ...
        __builtin_amdgcn_s_setprio(3);
        const int lw = wave - NCW;
        StepSrc rs;
        rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
        rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
        rs.m = make_srd(a.mask, HM ? a.m_span : 0);
        const int my_n = ns > lw ? (ns - lw + NLW - 1) / NLW : 0;
        auto issue = [&](int j) {
            const int s = lw + j * NLW;
            const int slot = dec_slot(s, NLW, spl);
            if (s >= nslot) {  // ring: the consumer of step s - nslot must be done with the slot
                const uint32_t want = (uint32_t)(s - nslot + 1);
                while (__builtin_amdgcn_readfirstlane(freew[slot]) < want) __builtin_amdgcn_s_sleep(1);
            }
            if (a.dec_diag < 2)
                issue_step<KT, VT, D, 16, HM>(a, rs, c_lo + s * kStep, mrow0, slots + slot * C::stepBytes, lane);
        };
        int ni = 0;
        const int ah = min(AH, a.dec_ahead);
        for (; ni < ah && ni < my_n; ni++) issue(ni);
        for (int j = 0; j < my_n; j++) {
            dec_wait_steps<NI>(ni - 1 - j);  // step j of this loader landed in LDS
            const int s = lw + j * NLW;
            if (lane == 0) full[dec_slot(s, NLW, spl)] = (uint32_t)(s + 1);
            if (ni < my_n) {
                issue(ni);
                ni++;
            }
        }
        f32x4 o[NC];
        float corr[NB];
        split_epilogue<KT, VT, D, NCW>(a, o, kNegInf, 0.0f, corr, wave, lane, qt, hs, ik2, iq3, y, chunk, smem,
                                       C::mergeBytes, false, true);
        return;
    }

    // ================= compute wave: steps wave, wave + NCW, ...
    const int m = i16;
    const int mq = div_R(a, m);
    const int mh = hs * a.R + (m - mq * a.R);
    const int iq1 = qt * a.QPT + mq;
    const int iq2 = ik2 * a.rk2 + mh;
    const bool row_ok = (m < a.QPT * a.R) && (iq1 < a.NQ) && (mh < a.rk2);

    // Q^T operand (B of S^T = K.Q^T), rounded to f16 like src/utils.h:10; lanes
    // of unused columns read past the descriptor (zeros, no traffic)
    f16x8 qop[NB];
    {
        u32x4 qraw[NB][2];
        const i32x4 qs = make_srd(a.q + (int64_t)iq3 * a.q_nb3, a.q_span);
        const uint32_t qoff = row_ok ? (uint32_t)iq1 * (uint32_t)a.q_nb1 + (uint32_t)iq2 * (uint32_t)a.q_nb2 + 32 * g
                                     : a.q_span;
#pragma unroll
        for (int b = 0; b < NB; b++) {
            qraw[b][0] = ld_buf(qs, qoff + 128 * b);
            qraw[b][1] = ld_buf(qs, qoff + 128 * b + 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int b = 0; b < NB; b++) {
            reg_fence(qraw[b][0]);
            reg_fence(qraw[b][1]);
            const f32x4 x0 = __builtin_bit_cast(f32x4, qraw[b][0]), x1 = __builtin_bit_cast(f32x4, qraw[b][1]);
            f16x8 h;
            h.s0 = (f16)x0.x; h.s1 = (f16)x0.y; h.s2 = (f16)x0.z; h.s3 = (f16)x0.w;
            h.s4 = (f16)x1.x; h.s5 = (f16)x1.y; h.s6 = (f16)x1.z; h.s7 = (f16)x1.w;
            qop[b] = h;
        }
    }
    FATTN_STAMP8(2);

    float m_run = kNegInf;
    float l_run = 0.0f;
    f32x4 o[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) o[c] = f32x4{0, 0, 0, 0};
    float corr[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) corr[b] = 0.0f;

    bool first = true;
    for (int s = wave; s < ns; s += NCW) {
        const int slot = dec_slot(s, NLW, spl);
        const uint32_t want = (uint32_t)(s + 1);
        while (__builtin_amdgcn_readfirstlane(full[slot]) != want) __builtin_amdgcn_s_sleep(1);
        if (first) FATTN_STAMP8(3);
        if (s + NCW >= ns) FATTN_STAMP8(5);
        const int n0 = c_lo + s * kStep;
        if (a.dec_diag != 1 && a.dec_diag != 3) {
            split_step<KT, VT, D, HM>(a, slots + slot * C::stepBytes, qop, mq, g, i16, min(kStep, c_hi - n0), first,
                                      m_run, l_run, o, corr, [] {});
            first = false;
        }
        if (ring) {  // hand the slot back once every read of it has returned
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) freew[slot] = want;
        }
    }
    FATTN_STAMP8(6);
    split_epilogue<KT, VT, D, NCW>(a, o, m_run, l_run, corr, wave, lane, qt, hs, ik2, iq3, y, chunk, smem,
                                   C::mergeBytes, true, true);
}

}  // namespace fattn
