// fattn_pf4.h -- prefill attention, one wave per SIMD (gfx950).
//
// The f16 prefill body (f16 K/V rows; Q8_0 / Q4_0 caches arrive here staged
// to f16 by kv_stage_f16_kernel).  Same math as fattn_pf_kernel (scale * q.k
// + mask, online softmax with the deferred max, f16 operands, f32
// accumulation; src/flash-llama.h:5-438 is the reference's form of it), laid
// out for one wave per SIMD instead of two:
//
//  * one workgroup = 4 waves = 256 packed (query row x q-head) rows of one kv
//    head, 64 per wave as two 32-row blocks (rb 0, 1); __launch_bounds__(256, 1):
//    each wave owns its SIMD's whole 512-entry register file, so O (2 x 64
//    f32), Q^T (2 x 32 f16x2) and a tile's K or V operands stay in registers;
//  * K and V operands are read from LDS ONCE per wave and tile and used for
//    both row blocks (the 8-wave form reads them once per 32 rows: twice the
//    LDS traffic, which bounded it);
//  * per 64-key tile j, two phases of 32 MFMAs, the vector work of one row
//    block beside the matrix work (cdna_hip_programming.md 'Fused attention
//    prefill', 4-wave structure), P.V one tile behind S:
//      A_j: S_j = K_j . Q^T for both row blocks || rb 0's exponentials of
//           tile j-1, rb 1's scores / max of tile j
//      B_j: O += V_{j-1}^T . P_{j-1}^T for both  || rb 1's decision and
//           exponentials of tile j, rb 0's scores / max / decision of tile j
//    (SCHED 3, "balanced", the default; SCHED 2, "pipelined": each phase's
//    exponentials in one half and its max pieces in the other); one
//    workgroup barrier per tile, mid-A;
//  * HBM -> LDS by LDS-DMA straight into the f16 images (the swizzles of
//    fattn_pf.h, 16-B granular, so each lane's source offset carries them):
//    K and V rings of 3 tiles, per-wave mask rings of 2: V j in A_j, K j+3
//    and mask j+2 in B_j, into the slots their tiles freed; K and V operands
//    are re-read from LDS per phase (256 B/clk: LDS has the bandwidth, the
//    register file not the room).
//
// LDS (D = 128): K ring 3 x 16 KiB, V ring 3 x 16 KiB, mask [4 waves][2][64
// rows][128 B] = 64 KiB: 160 KiB.  The epilogue parks each wave's 64
// normalised rows there ([256 rows][D + 4] f32) and stores whole rows.
#pragma once

#include "fattn_pf.h"

namespace fattn {

constexpr int kPf4Waves = 4;
constexpr int kPf4RowsW = 64;  // packed rows per wave (two 32-row blocks)

template <int D>
struct Pf4Cfg {
    static_assert(D == 128, "the one-wave-per-SIMD prefill body is D = 128 (other head dims: fattn_pf_kernel)");
    static constexpr int img = kPfKeys * D * 2;            // one f16 image (16 KiB)
    static constexpr int KS = 3, VS = 3, MS = 2;           // ring depths
    static constexpr int kOff = 0;
    static constexpr int vOff = KS * img;
    static constexpr int maskSlot = kPf4RowsW * kPfKeys * 2;  // 8 KiB: 64 rows x 64 keys f16
    static constexpr int mOff = vOff + VS * img;
    static constexpr int loopBytes = mOff + kPf4Waves * MS * maskSlot;
    static constexpr int parkBytes = kPf4Waves * kPf4RowsW * (D + 4) * 4;
    static constexpr int ldsBytes = loopBytes > parkBytes ? loopBytes : parkBytes;
    static constexpr int NJ = img / 1024;                  // 1-KiB DMA pieces per image (16)
    static constexpr int NKI = NJ / kPf4Waves;             // K (and V) DMA instructions per wave and tile (4)
    static constexpr int NMI = maskSlot / 1024;            // mask DMA instructions per wave and tile (8)
    static_assert(ldsBytes <= 163840, "");
};

// row-sum add.  Plain C: hipcc places the trans-use wait state after each
// v_exp_f32 only for instructions it sees; an inline-asm v_add_f32 reading an
// exponential one instruction after its v_exp read a stale register in some
// lanes (rows scaled or sign-flipped; FATTN_PF4_ASM_ADD keeps that form for A/B
// and hazard-checker tests only)
__device__ __forceinline__ float add_f32(float x, float y) {
#ifdef FATTN_PF4_ASM_ADD  // diagnostic build only: WRONG results (see above)
    float r;
    asm("v_add_f32_e32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
#else
    // (not contracted with l's rescale multiply into one fma: the 8-wave
    // body rounds the two separately, and the forms must give the same bits)
#pragma clang fp contract(off)
    return x + y;
#endif
}
// O *= alpha on one accumulator block where it lives (AGPRs), in one asm
// statement: v_accvgpr_read, v_mul_f32, v_accvgpr_write per element, inside
// the rare rescale branch.  Written in C the multiply needs O in VGPRs, and
// hipcc hoisted those AGPR -> VGPR copies (128 per tile) out of the branch onto
// every tile.  The trailing s_nop covers the accumulator-write -> MFMA-read
// wait states the compiler cannot see inside the asm (the next P.V MFMAs read
// these registers as srcC).
__device__ __forceinline__ void scale_acc16(f32x16& o, float alpha) {
    float t;
    asm volatile(
        "v_accvgpr_read_b32 %16, %0\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %0, %16\n\t"
        "v_accvgpr_read_b32 %16, %1\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %1, %16\n\t"
        "v_accvgpr_read_b32 %16, %2\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %2, %16\n\t"
        "v_accvgpr_read_b32 %16, %3\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %3, %16\n\t"
        "v_accvgpr_read_b32 %16, %4\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %4, %16\n\t"
        "v_accvgpr_read_b32 %16, %5\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %5, %16\n\t"
        "v_accvgpr_read_b32 %16, %6\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %6, %16\n\t"
        "v_accvgpr_read_b32 %16, %7\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %7, %16\n\t"
        "v_accvgpr_read_b32 %16, %8\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %8, %16\n\t"
        "v_accvgpr_read_b32 %16, %9\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %9, %16\n\t"
        "v_accvgpr_read_b32 %16, %10\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %10, %16\n\t"
        "v_accvgpr_read_b32 %16, %11\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %11, %16\n\t"
        "v_accvgpr_read_b32 %16, %12\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %12, %16\n\t"
        "v_accvgpr_read_b32 %16, %13\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %13, %16\n\t"
        "v_accvgpr_read_b32 %16, %14\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %14, %16\n\t"
        "v_accvgpr_read_b32 %16, %15\n\tv_mul_f32_e32 %16, %17, %16\n\tv_accvgpr_write_b32 %15, %16\n\t"
        "s_nop 7"
        : "+a"(o[0]), "+a"(o[1]), "+a"(o[2]), "+a"(o[3]), "+a"(o[4]), "+a"(o[5]), "+a"(o[6]), "+a"(o[7]),
          "+a"(o[8]), "+a"(o[9]), "+a"(o[10]), "+a"(o[11]), "+a"(o[12]), "+a"(o[13]), "+a"(o[14]), "+a"(o[15]),
          "=&v"(t)
        : "v"(alpha));
}
// S^T chain steps of the lean body with the accumulator in VGPRs and Q^T's
// operand in AGPRs: hipcc puts every MFMA's accumulator of a 512-register
// kernel in AGPRs, so each score cost a v_accvgpr_read beside its multiply
// (64 of the tile's ~380 vector instructions).  Q^T is loop-invariant and an
// MFMA takes srcB from AGPRs, so the two swap files; the chain starts from 0
// and the row's -m enters the exponent argument's fma.  Wait states hipcc
// cannot see (its hazard pass knows only its own MFMAs): the accumulator ->
// first VALU read (an 8-pass XDL write: 12 states) and Q^T's v_accvgpr_write
// -> MFMA read, checked on the .s by tools/isa_hazard_check.py (xdl-vgpr).
#ifndef FATTN_PF4_SAGPR
#define FATTN_PF4_SVGPR 1
#else
#define FATTN_PF4_SVGPR 0
#endif
__device__ __forceinline__ void mfma_s_first(f32x16& d, const f16x8& k, const f16x8& q) {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(d) : "v"(k), "a"(q));
}
__device__ __forceinline__ void mfma_s_next(f32x16& d, const f16x8& k, const f16x8& q) {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(d) : "v"(k), "a"(q));
}

// registers through an empty volatile asm: code that reads them cannot move
// above the asm (pins a phase's VALU below the branches at its start)
__device__ __forceinline__ void pin16(float (&x)[16]) {
    asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                 "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                 "+v"(x[14]), "+v"(x[15]));
}
__device__ __forceinline__ void pin16(f32x16& x) {
    asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                 "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                 "+v"(x[14]), "+v"(x[15]));
}

// (P fragments of one row block: pinned at the end of the phase that made them,
// so hipcc's machine sinking cannot move their exponentials next to the P.V
// that uses them, into the next phase's block)
__device__ __forceinline__ void pin_p(f16x8 (&p)[2][2]) {
    u32x4 a = __builtin_bit_cast(u32x4, p[0][0]), b = __builtin_bit_cast(u32x4, p[0][1]);
    u32x4 c = __builtin_bit_cast(u32x4, p[1][0]), d = __builtin_bit_cast(u32x4, p[1][1]);
    asm volatile("" : "+v"(a.x), "+v"(a.y), "+v"(a.z), "+v"(a.w), "+v"(b.x), "+v"(b.y), "+v"(b.z), "+v"(b.w),
                 "+v"(c.x), "+v"(c.y), "+v"(c.z), "+v"(c.w), "+v"(d.x), "+v"(d.y), "+v"(d.z), "+v"(d.w));
    p[0][0] = __builtin_bit_cast(f16x8, a);
    p[0][1] = __builtin_bit_cast(f16x8, b);
    p[1][0] = __builtin_bit_cast(f16x8, c);
    p[1][1] = __builtin_bit_cast(f16x8, d);
}

// diagnostic builds only: without the opaque bases
#ifdef FATTN_PF4_SHFL
#define PF4_XOR32(x, mx) ((mx) ? fmaxf((x), __shfl_xor((x), 32)) : (x) + __shfl_xor((x), 32))
#else
#define PF4_XOR32(x, mx) xor32_pair((x), (mx))
#endif
#ifdef FATTN_PF4_NO_OPAQUE
#define PF4_OPAQUE_V(x) ((void)0)
#define PF4_OPAQUE_S(x) ((void)0)
#define PF4_OPAQUE_V2(x, y) ((void)0)
#else
#define PF4_OPAQUE_V(x) asm volatile("" : "+v"(x))
#define PF4_OPAQUE_S(x) asm volatile("" : "+s"(x))
#define PF4_OPAQUE_V2(x, y) asm volatile("" : "+v"(x), "+v"(y))
#endif

// the piece q in [0, 16) whose stage of schedule s(q) = C + (A q) / B falls on
// step i, or -1 (s strictly increasing: A >= B)
template <int A, int B, int C>
__device__ __forceinline__ constexpr int sched_inv(int i) {
    static_assert(A >= B, "the schedule must be strictly increasing");
    const int d = i - C;
    if (d < 0) return -1;
    const int q0 = (d * B) / A;
    if (q0 < 16 && (A * q0) / B == d) return q0;
    if (q0 + 1 < 16 && (A * (q0 + 1)) / B == d) return q0 + 1;
    return -1;
}

// SCHED 2: the pipelined schedule (FATTN_OPT_PF_FORM 4); SCHED 3: the balanced
// one (FATTN_OPT_PF_FORM 5, the default).  Same arithmetic, same order per row
// block: both give the same bits as fattn_pf_kernel.  (Round 5's unpipelined
// three-phase forms, SCHED 0 / 1, measured 18-33 % slower and were removed.)
template <int D, bool HM, int SCHED>
__global__ __launch_bounds__(kPf4Waves* kWave, 1) void fattn_pf4_kernel(const SplitArgs a) {
    using C = Pf4Cfg<D>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NK = D / 16;   // 16-dim k-steps of S^T = K.Q^T
    constexpr int NDB = D / 32;  // 32-dim blocks of O^T
    constexpr float kNegInf = -__builtin_inff();
    constexpr float kDeferLog2 = 8.0f;
    // SCHED 4 ("lean"): each S^T chain starts from the row's -m / c (m its
    // running max in log2 units, c = scale * log2(e)) instead of 0, so one
    // multiply by c turns the accumulator into the exponent argument c s - m:
    // per score an accumulator read, that multiply, one max, one exponential,
    // one row-sum add and half a pack -- not the balanced form's separate
    // scale fma and "x * log2(e) - m" (bodies without mask values: the zero
    // mask, no mask; a masked body runs the balanced arithmetic -- its extra
    // fma per score pushed the lean form into scratch); the rescale decisions
    // move to the phase tails, where the rare
    // branch also shifts the tile's arguments and the chains' start.  Q^T
    // stays h(q) (src/utils.h:10): pre-scaling it by c instead (one rounding
    // more) cost 5e-3 on large scores.  Not bit-identical to the 8-wave body
    // (the -m / c enters the f32 chain): the oracle's 1e-3 is the bar.
    constexpr bool LEAN = SCHED == 4;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef FATTN_STAMPS
    // (diagnostic build: the workgroup's timeline -- entry, loop start / end,
    // exit in shader clocks, entry / exit in the 100-MHz real-time clock)
    const uint64_t kt_entry = __builtin_amdgcn_s_memtime();
    const uint64_t kr_entry = __builtin_amdgcn_s_memrealtime();
    uint64_t kt_loop0 = 0, kt_loop1 = 0;
#endif
    const int h = lane >> 5;    // k-group of the MFMA operands
    const int c32 = lane & 31;  // MFMA column: this lane's row within a 32-row block

    // ---- tile decode (as fattn_pf_kernel): y -> (kv head, query tile)
    const int y = blockIdx.y;
    const int iq3 = blockIdx.z;
    int qt = 0, ik2 = y, ik3 = iq3;
    if (a.pf_flags) {  // masked: longest-first dispatch (the last query tile of every head first)
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
        return mq < a.QPT && iq1 < a.NQ;
    };
    // live KV tile range [t0, t0 + nt) and the +-0 mask blocks (flags 2), from
    // pf_mask_flags_kernel (fattn_pf.h)
    int t0 = 0, nt = a.N / kPfKeys;
    uint64_t zb[4] = {0, 0, 0, 0};
    if (a.pf_flags) {
        const uint8_t* fl = a.pf_flags + (int64_t)qt * nt;
        int lo = nt, hi = -1;
        for (int b = 0; b < nt; b += kWave) {  // wave-uniform
            const bool f = b + lane < nt && fl[b + lane] != 0;
            const uint64_t m = __builtin_amdgcn_ballot_w64(f);
            if (m) {
                lo = min(lo, b + (int)__builtin_ctzll(m));
                hi = b + 63 - (int)__builtin_clzll(m);
            }
        }
        t0 = lo;
        const int all = nt;
        nt = hi >= lo ? hi - lo + 1 : 0;
        const uint8_t* fz = a.pf_flags + (int64_t)qt * all + t0;
#pragma unroll
        for (int w = 0; w < 4; w++) zb[w] = __builtin_amdgcn_ballot_w64(64 * w + lane < nt && fz[64 * w + lane] == 2);
    }
    auto zero_of = [&](int s) { return s < 256 && ((zb[s >> 6] >> (s & 63)) & 1); };

    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    rs.m = make_srd(a.mask, HM ? a.m_span : 0);
    const uint32_t lds0 = lds_addr(smem);
    typedef __attribute__((address_space(3))) uint8_t lds_u8;

    // ---- Q^T operands of both row blocks, rounded to f16 (src/utils.h:10)
    f16x8 qop[2][NK];
    {
        const auto qs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.q + (int64_t)iq3 * a.q_nb3), 0,
                                                          a.q_span, 0x00020000);
#pragma unroll
        for (int rb = 0; rb < 2; rb++) {
            int q1, q2;
            const bool ok = row_of(kPf4RowsW * wave + 32 * rb + c32, q1, q2);
            const uint32_t qoff = ok ? (uint32_t)q1 * (uint32_t)a.q_nb1 + (uint32_t)q2 * (uint32_t)a.q_nb2 + 32 * h
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
    if constexpr (LEAN && FATTN_PF4_SVGPR) {
        // (Q^T into AGPRs once, where the lean chains take it as srcB: from
        // VGPRs hipcc copied it there before every MFMA, 64 v_accvgpr_write a tile)
#pragma unroll
        for (int rb = 0; rb < 2; rb++) {
#pragma unroll
            for (int kk = 0; kk < NK; kk++) asm volatile("" : "+a"(qop[rb][kk]));
        }
        // (the accumulator-write -> MFMA-read wait states of those writes)
        asm volatile("s_nop 4");
    }

    // ---- DMA source offsets (tile-relative; + n0 * nb1 per tile): piece
    // j = wave + 4i of the K image and of the V image, laid out as the image
    // swizzles of fattn_pf.h (K [8 slices][64 keys][32 B], 16-B halves swapped
    // on rows with bit 3 set; V [4 dim blocks][64 keys][64 B], chunk c of row r
    // at c ^ ((r >> 2) & 3))
    // piece j = wave + 4i of an image: the K pieces of one wave share their
    // rows (32 (wave & 1) + lane / 2) and step 2 slices (64 B) per i; the V
    // pieces share their rows (16 wave + lane / 4) and step one dim block (64
    // B) per i -- one offset per image and lane, the rest immediates
    static_assert(kPf4Waves == 4 && C::NKI == 4, "");
    uint32_t koff0, voff0;
    {
        const int r = 32 * (wave & 1) + (lane >> 1), hh = lane & 1;
        koff0 = (uint32_t)r * (uint32_t)a.k_nb1 + (wave >> 1) * 32 + (hh ^ ((r >> 3) & 1)) * 16;
    }
    {
        const int r = 16 * wave + (lane >> 2), pc = lane & 3;
        voff0 = (uint32_t)r * (uint32_t)a.v_nb1 + (pc ^ ((r >> 2) & 3)) * 16;
    }
    // mask: instruction k fills rows 8k .. 8k+7 of the wave's 64 (row pr:
    // 16-B piece pc stored at pc ^ ((pr >> 1) & 7)); rows past the mask fall
    // outside its descriptor (zeros, no traffic)
    uint32_t moff[C::NMI];
    if constexpr (HM) {
#pragma unroll
        for (int k = 0; k < C::NMI; k++) {
            const int rr = 8 * k + (lane >> 3);
            int q1, q2;
            const bool ok = row_of(kPf4RowsW * wave + rr, q1, q2);
            const int pc = (lane & 7) ^ ((rr >> 1) & 7);
            moff[k] = ok ? (uint32_t)q1 * (uint32_t)a.m_nb1 + 16 * pc : a.m_span;
        }
    }

    // per-lane LDS read offsets within an image: K slice kk, row 32t + c32,
    // half h; V^T gather (ds_read_b64_tr_b16) as fattn_pf.h
    const uint32_t kbase = c32 * 32 + ((h ^ ((c32 >> 3) & 1)) * 16);
    const int gi = lane & 15, dh = (lane >> 4) & 1;
    uint32_t vbase[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int row = 8 * e + 4 * h + (gi >> 2);
        const int ch = (2 * dh + ((gi & 3) >> 1)) ^ ((h + 2 * e) & 3);
        vbase[e] = row * 64 + ch * 16 + (gi & 1) * 8;
    }
    // mask read offsets: row c32 of the wave's slot, piece 4t + u (keys
    // 32t + 8u .. +7), half h
    // (row block 1: + 32 rows; (pr >> 1) & 7 is the same for both)
    uint32_t mrd[2][4];
#pragma unroll
    for (int t = 0; t < 2; t++) {
#pragma unroll
        for (int u = 0; u < 4; u++) mrd[t][u] = c32 * 128 + (((4 * t + u) ^ ((c32 >> 1) & 7)) * 16) + 8 * h;
    }


    const float log2e = 1.4426950408889634f;
    const float scale = a.scale_log2 / log2e;
    const float cexp = HM ? log2e : a.scale_log2;  // exponent argument x * c - m (log2 domain)
    float m_run[2] = {kNegInf, kNegInf};
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
    f32x16 s0[2], s1[2];  // S^T of rb 0 and rb 1 (both computed in A_j), per subtile
    f32x16 ci[2];         // (SCHED 4) each row block's S^T chain start: -m / c of the row (0 while m = -inf)
#pragma unroll
    for (int rb = 0; rb < 2; rb++) {
#pragma unroll
        for (int j = 0; j < 16; j++) ci[rb][j] = 0.0f;
        // (held in AGPRs, where the MFMAs take it as srcC: from VGPRs hipcc
        // copied it to AGPRs before every chain, 32 v_accvgpr_write a tile)
        if constexpr (SCHED == 4 && !FATTN_PF4_SVGPR) asm volatile("" : "+a"(ci[rb]));
    }

    // mask values of row block rb for tile s (a +-0 block's slot holds the
    // zeros its empty DMA wrote)
    auto mask_reads = [&](int s, int rb, u32x2 (&mk)[2][4]) {
        if constexpr (HM) {
            uint32_t mb = (uint32_t)(C::mOff + (wave * C::MS + s % C::MS) * C::maskSlot + rb * (32 * 128));
            PF4_OPAQUE_S(mb);
            const lds_u8* slot = (const lds_u8*)smem + mb;
#pragma unroll
            for (int t = 0; t < 2; t++) {
#pragma unroll
                for (int u = 0; u < 4; u++) mk[t][u] = *(const __attribute__((address_space(3))) u32x2*)(slot + mrd[t][u]);
            }
        }
    };
    // exponentials of one row block's tile (subtile t): p = exp2(u * c - m) to
    // f16 P^T fragments in the accumulator's own key order (element j of
    // subtile t is key 32t + 8(j/4) + 4h + (j%4)); row sums as scalar f32 adds
    // (the last tile's, after the loop; the loop stages the same operations
    // over its steps, e1 / e2 / e3 below)
    auto sexp = [&](int rb, int t, const float (&us)[2][16], f16x8 (&pb)[2][2], bool lean) {
        const float nm = (m_run[rb] == kNegInf) ? 0.0f : -m_run[rb];
        float la = l2[rb].x, lb = l2[rb].y;
#pragma unroll
        for (int q = 0; q < 2; q++) {
            f16x8 x;
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
                const float pa = __builtin_amdgcn_exp2f(lean ? us[t][8 * q + e] : fmaf(us[t][8 * q + e], cexp, nm));
                const float pb2 =
                    __builtin_amdgcn_exp2f(lean ? us[t][8 * q + e + 1] : fmaf(us[t][8 * q + e + 1], cexp, nm));
                la = add_f32(la, pa);
                lb = add_f32(lb, pb2);
                x[e] = (f16)pa;
                x[e + 1] = (f16)pb2;
            }
            pb[t][q] = x;
        }
        l2[rb] = f32x2{la, lb};
    };
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    // (LDS-space arithmetic: the per-read offsets fold into the instructions'
    // immediate; through a generic pointer every read got its own v_add)
    lds_u8* const lsm = (lds_u8*)smem;

    {
        // A workgroup whose live tiles all hold +-0 masks (the flags pass's 2,
        // SURVEY's zero-mask prefill) runs the body without mask values in
        // LDS (ZM): no mask DMA, reads or waits, scores fma(s, scale, 0) --
        // the masked path's arithmetic on a zero mask, so the same bits.
        bool all_zero = false;
        if constexpr (HM) {
            int nz = 0;
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const int lo = 64 * w;
                const uint64_t in = nt >= lo + 64 ? ~0ull : (nt > lo ? (1ull << (nt - lo)) - 1 : 0ull);
                nz += __builtin_popcountll(zb[w] & in);
            }
            all_zero = nt > 0 && nz == nt;
        }
        auto body2 = [&](auto zm_tag) {
            constexpr bool ZM = decltype(zm_tag)::value;
            constexpr bool MM = HM && !ZM;  // mask values through LDS
            // (the lean arithmetic for the bodies without mask values -- the bench's
            // zero-mask prefill, no mask; masked bodies keep the balanced form's:
            // its extra fma per score pushed the masked lean body into scratch)
            constexpr bool LN = LEAN && !MM;
            // the pipelined schedule (cdna_hip_programming.md 'Fused attention
            // prefill', 4-wave structure): per tile two phases of 32 MFMAs,
            //   A_j: S_j = K_j . Q^T for both row blocks  ||  rb 1's exponentials
            //        of tile j-1, rb 1's scores / max / rescale decision of tile j;
            //   B_j: O += V_{j-1}^T . P_{j-1}^T for both row blocks (each V^T
            //        operand read once, used twice)  ||  rb 0's scores / max /
            //        decision and exponentials of tile j;
            // so both phases carry one row block's exponentials (one v_exp per
            // MFMA gap).  The O rescale a decision of tile j-1 asks for is applied
            // at the start of A_j: after P_{j-2}.V (B_{j-1}), before P_{j-1}.V --
            // the 8-wave body's order of operations on O and l, so the same bits.
            // Rings: V_j is issued in A_j (into V_{j-3}'s slot), K_{j+3} in B_j
            // (after its barrier, into K_j's slot), the wave's mask j+2 in B_j
            // after its reads of mask j.  A_j's counted wait leaves B_{j-1}'s
            // issues in flight: K_{j+1}, V_{j-1} and mask j have landed (this
            // wave's pieces; B_j's barrier then covers everyone's).
            static_assert(C::NKI == 4 && C::NMI == 8, "the wait counts below are multiples of 4");
            constexpr int MI = MM ? C::NMI : 0;
            // Every tile issues the same DMA instructions (K_{j+3}, V_{j+1}, mask
            // j+2 at B_j), a tile past the end through an offset past its
            // descriptor (no traffic; into a slot nothing reads again), so every
            // counted wait is one constant and the issues sit inside B's steps
            // without a branch.
            // (slot: the ring slot s % 3, which the balanced loop carries from tile
            // to tile instead of dividing -- four mod-3 divisions a tile were 16
            // scalar instructions of a one-wave-per-SIMD loop)
            auto k_piece_at = [&](int s, int slot, int i) {
                const uint32_t nk = (uint32_t)(t0 + s) * kPfKeys * (uint32_t)a.k_nb1;
                const uint32_t dst = lds0 + C::kOff + slot * C::img + (wave + kPf4Waves * i) * 1024;
                dma<16, false, 0>(rs.k, dst, s < nt ? nk + koff0 + 64 * i : a.k_span);
            };
            auto v_piece_at = [&](int s, int slot, int i) {
                const uint32_t nv = (uint32_t)(t0 + s) * kPfKeys * (uint32_t)a.v_nb1;
                const uint32_t dst = lds0 + C::vOff + slot * C::img + (wave + kPf4Waves * i) * 1024;
                dma<16, false, 0>(rs.v, dst, s < nt ? nv + voff0 + 64 * i : a.v_span);
            };
            auto k_piece = [&](int s, int i) { k_piece_at(s, s % C::KS, i); };
            auto v_piece = [&](int s, int i) { v_piece_at(s, s % C::VS, i); };
            // (skip: tile s past the end or a +-0 block, decided once per tile --
            // inside B's steps a branch would split the phase)
            auto m_skip = [&](int s) { return s >= nt || zero_of(s); };
            auto m_piece = [&](int s, int k, bool skip) {
                if constexpr (MM) {
                    const uint32_t n2 = (uint32_t)(t0 + s) * kPfKeys * 2;
                    const uint32_t dst = lds0 + C::mOff + (wave * C::MS + s % C::MS) * C::maskSlot + k * 1024;
                    dma<16>(rs.m, dst, (skip || moff[k] == a.m_span) ? a.m_span : moff[k] + n2);
                }
            };
            // prologue: K 0 | K 1, mask 0 | K 2, mask 1 (the last two groups as
            // the steady state's B_{-2} and B_{-1}; V 0 comes in A_0)
            if (nt > 0) {
#pragma unroll
                for (int i = 0; i < C::NKI; i++) k_piece(0, i);
#pragma unroll
                for (int i = 0; i < C::NKI; i++) k_piece(1, i);
#pragma unroll
                for (int k = 0; k < C::NMI; k++) m_piece(0, k, m_skip(0));
#pragma unroll
                for (int i = 0; i < C::NKI; i++) k_piece(2, i);
#pragma unroll
                for (int k = 0; k < C::NMI; k++) m_piece(1, k, m_skip(1));
            }
            // O_rb^T += V_s^T . P_rb^T for both row blocks, each V^T operand read
            // once; per accumulator the 8-wave body's order (t, q)
            auto pv2 = [&](int s, const f16x8 (&pa)[2][2], const f16x8 (&pb)[2][2]) {
                uint32_t b0 = (uint32_t)(C::vOff + (s % C::VS) * C::img) + vbase[0];
                uint32_t b1 = (uint32_t)(C::vOff + (s % C::VS) * C::img) + vbase[1];
                PF4_OPAQUE_V2(b0, b1);
                lds_u8* const img0 = lsm + b0;
                lds_u8* const img1 = lsm + b1;
                // every V^T operand of the tile first (64 VGPRs), so that no MFMA
                // of the phase waits for its own read
                f16x8 va[2][2][NDB];
#pragma unroll
                for (int t = 0; t < 2; t++) {
#pragma unroll
                    for (int q = 0; q < 2; q++) {
#pragma unroll
                        for (int db = 0; db < NDB; db++) {
                            const uint32_t off = db * (kPfKeys * 64) + t * 2048 + q * 1024;
                            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img0 + off));
                            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img1 + off));
                            const u32x2 a2 = __builtin_bit_cast(u32x2, lo), b2 = __builtin_bit_cast(u32x2, hi);
                            va[t][q][db] = __builtin_bit_cast(f16x8, u32x4{a2.x, a2.y, b2.x, b2.y});
                        }
                    }
                }
#pragma unroll
                for (int t = 0; t < 2; t++) {
#pragma unroll
                    for (int q = 0; q < 2; q++) {
#pragma unroll
                        for (int db = 0; db < NDB; db++) {
                            o[0][db] = mfma32(va[t][q][db], pa[t][q], o[0][db]);
                            o[1][db] = mfma32(va[t][q][db], pb[t][q], o[1][db]);
                        }
                    }
                }
            };
            // K_j's operands, read once per tile at the start of A_j for both row blocks
            f16x8 kr[2][NK];
            // (the streamed forms: operand reads placed inside the steps, a few
            // ahead of their MFMA -- with all of a phase's reads at its head the
            // 4-bit lgkmcnt cannot name the first one, and the first MFMA waited
            // for half of them)
            auto k_base_at = [&](int slot) {
                uint32_t kb = (uint32_t)(C::kOff + slot * C::img) + kbase;
                PF4_OPAQUE_V(kb);
                return kb;
            };
            auto k_base = [&](int s) { return k_base_at(s % C::KS); };
            auto k_read1 = [&](uint32_t kb, int t, int kk) {
                kr[t][kk] = *(const __attribute__((address_space(3))) f16x8*)((const lds_u8*)smem + kb + kk * (kPfKeys * 32) +
                                                                           t * 1024);
            };
            if (nt > 0) {
                // K 0 landed: everything issued after it may fly
                wait_vmcnt_c<2 * C::NKI + 2 * MI>();
                __syncthreads();
            }
            float us0[2][16], us1[2][16];
            float al0 = 1.0f, al1 = 1.0f;
            bool rs0 = false, rs1 = false;
            f16x8 p0[2][2], p1[2][2];
            // (the first tile without rb 1's previous exponentials and without a
            // P.V: a compile-time flag, so that no branch splits a phase -- a
            // phase must stay one basic block for its VALU to sit between its MFMAs)
            // O rescale (the decisions of tile j, both made in B_j) at the end of
            // B_j: after P_{j-1}.V, before P_j.V (B_{j+1}); in AGPRs (scale_acc16).
            // There only O is live in AGPRs -- at B_j's start (the old place) S0
            // was, and the branch made hipcc copy all of it to VGPRs in one block
            // behind its last MFMA.  The pad: B_j's last P.V MFMAs may still be
            // writing the O registers the asm reads (wait states hipcc cannot see
            // inside the asm; a rare branch, so the pad is free).
            auto rescale_acc = [&](int rb, bool resc, float alpha) {
                if (__builtin_expect(resc, 0)) {
                    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
                    for (int db = 0; db < NDB; db++) scale_acc16(o[rb][db], alpha);
                }
            };
            // The phases are written as 32 explicit (MFMA, vector piece) steps, each
            // its own scheduling region (sched_barrier): hipcc's scheduling groups
            // left the exponentials behind the MFMA runs (in-order issue then
            // serialises them).  A vector piece = two elements of one row block:
            // scores + running max (smax_piece) or exponentials + row sums + f16
            // pair (sexp_piece) -- the same operations in the same order per row
            // as smax / sexp, so the same bits.
            // (the rescale decision from the lane pair's max, log2 units)
            auto smax_decide = [&](int rb, float tmax, float& alpha, bool& resc) {
                resc = __builtin_amdgcn_ballot_w64(tmax > m_run[rb] + kDeferLog2) != 0;
                const float m_new = resc ? fmaxf(m_run[rb], tmax) : m_run[rb];
                alpha = (!resc || m_new == kNegInf) ? 1.0f : __builtin_amdgcn_exp2f(m_run[rb] - m_new);
                float mn = m_new, lx = l2[rb].x * alpha, ly = l2[rb].y * alpha;
                // (pinned into its step: rb 1's results are next used past B's
                // loop, and hipcc sank the whole chain there)
                asm volatile("" : "+v"(alpha), "+v"(mn), "+v"(lx), "+v"(ly));
                m_run[rb] = mn;
                l2[rb] = f32x2{lx, ly};
            };
            // Staged forms of the pieces: a piece's three dependent instruction
            // groups in three consecutive steps (its exponent arguments, its
            // exponentials, its sums and f16 pair; its accumulator reads, its
            // scores, its max), so that no step waits on its own results --
            // each stage's results pinned into its step like the pieces'.
            float sA[16][2], sE[16][2], mX[16][2];
            auto e1 = [&](const float (&us)[2][16], float nm, int pc) {
                const int t = pc >> 3, k = 2 * (pc & 7);
                sA[pc][0] = fmaf(us[t][k], cexp, nm);
                sA[pc][1] = fmaf(us[t][k + 1], cexp, nm);
                asm volatile("" : "+v"(sA[pc][0]), "+v"(sA[pc][1]));
            };
            auto e2 = [&](int pc) {
                sE[pc][0] = __builtin_amdgcn_exp2f(sA[pc][0]);
                sE[pc][1] = __builtin_amdgcn_exp2f(sA[pc][1]);
                asm volatile("" : "+v"(sE[pc][0]), "+v"(sE[pc][1]));
            };
            auto e2u = [&](const float (&us)[2][16], int pc) {  // (SCHED 4: the argument is the score)
                const int t = pc >> 3, k = 2 * (pc & 7);
                sE[pc][0] = __builtin_amdgcn_exp2f(us[t][k]);
                sE[pc][1] = __builtin_amdgcn_exp2f(us[t][k + 1]);
                asm volatile("" : "+v"(sE[pc][0]), "+v"(sE[pc][1]));
            };
            auto e3 = [&](f16x8 (&pb)[2][2], float& la, float& lb, int pc) {
                const int t = pc >> 3, k = 2 * (pc & 7);
                la = add_f32(la, sE[pc][0]);
                lb = add_f32(lb, sE[pc][1]);
                pb[t][k >> 3][k & 7] = (f16)sE[pc][0];
                pb[t][k >> 3][(k & 7) + 1] = (f16)sE[pc][1];
                asm volatile("" : "+v"(la), "+v"(lb));
            };
            auto m1 = [&](const f32x16 (&st)[2], int pc) {
                const int t = pc >> 3, k = 2 * (pc & 7);
                mX[pc][0] = st[t][k];
                mX[pc][1] = st[t][k + 1];
                // (an accumulator read staged a step ahead; with the chains in VGPRs
                // (lean kernels) there is nothing to stage, and the pin made copies)
                if constexpr (!(LEAN && FATTN_PF4_SVGPR)) asm volatile("" : "+v"(mX[pc][0]), "+v"(mX[pc][1]));
            };
            // (SCHED 4 without mask values: the accumulator times c IS the argument)
            auto m1u = [&](const f32x16 (&st)[2], float (&us)[2][16], float nr, int pc) {
                const int t = pc >> 3, k = 2 * (pc & 7);
#if FATTN_PF4_SVGPR
                us[t][k] = fmaf(st[t][k], a.scale_log2, nr);
                us[t][k + 1] = fmaf(st[t][k + 1], a.scale_log2, nr);
#else
                (void)nr;
                us[t][k] = st[t][k] * a.scale_log2;
                us[t][k + 1] = st[t][k + 1] * a.scale_log2;
#endif
                asm volatile("" : "+v"(us[t][k]), "+v"(us[t][k + 1]));
            };
            auto m2 = [&](const u32x2 (&mk)[2][4], float (&us)[2][16], int pc) {
                const int t = pc >> 3, k0 = 2 * (pc & 7);
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const int k = k0 + e;
                    float x = mX[pc][e];
                    if constexpr (MM) {
                        const int u = k >> 2, ee = k & 3;
                        const f16x2 mm = as_h2(ee < 2 ? mk[t][u].x : mk[t][u].y);
                        x = fmaf(x, scale, (float)(ee & 1 ? mm.y : mm.x));
                    } else if constexpr (HM) {
                        x = fmaf(x, scale, 0.0f);
                    }
                    us[t][k] = x;
                }
                asm volatile("" : "+v"(us[t][k0]), "+v"(us[t][k0 + 1]));
            };
            // (SCHED 4) the rescale decision of row block rb at a phase tail: trel is
            // the tile max relative to the chains' start -m_ref; a rare,
            // wave-uniform branch applies a new max to the tile's arguments,
            // l, and the next chains' start (O's factor: rescale_acc, end of B)
            auto lean_decide = [&](int rb, float trel, float (&us)[2][16], float& alpha, bool& resc) {
                const float mref = m_run[rb] == kNegInf ? 0.0f : m_run[rb];
                const float tabs = trel + mref;
                resc = __builtin_amdgcn_ballot_w64(tabs > m_run[rb] + kDeferLog2) != 0;
                alpha = 1.0f;
                if (__builtin_expect(resc, 0)) {
                    asm volatile("; lean rescale" ::: "memory");
                    const float m_new = fmaxf(m_run[rb], tabs);
                    alpha = m_new == kNegInf ? 1.0f : __builtin_amdgcn_exp2f(m_run[rb] - m_new);
                    const float dlt = m_new == kNegInf ? 0.0f : m_new - mref;
#pragma unroll
                    for (int t = 0; t < 2; t++) {
#pragma unroll
                        for (int k = 0; k < 16; k++) us[t][k] -= dlt;
                    }
                    l2[rb] = f32x2{l2[rb].x * alpha, l2[rb].y * alpha};
                    m_run[rb] = m_new;
                    const float nci = m_new == kNegInf ? 0.0f : -m_new / a.scale_log2;
                    if constexpr (!FATTN_PF4_SVGPR) {
#pragma unroll
                        for (int j = 0; j < 16; j++) ci[rb][j] = nci;
                        asm volatile("" : "+a"(ci[rb]));
                    } else {
                        (void)nci;
                    }
                }
            };
            auto m3 = [&](const float (&us)[2][16], float& tmax, int pc) {
                const int t = pc >> 3, k = 2 * (pc & 7);
                tmax = fmaxf(fmaxf(tmax, us[t][k]), us[t][k + 1]);
                asm volatile("" : "+v"(tmax));
            };
    #ifdef FATTN_STAMPS
            // diagnostic build only (tools/pf_stamps.py): shader-clock cycles per
            // phase part, summed over tiles (0 A's wait, 1 A's steps, 2 A's tail,
            // 3 B's barrier, 4 B's head -- rescale, V^T reads --, 5 B's steps, 6 B's
            // tail, 7 between tiles)
            uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            uint64_t t_prev = __builtin_amdgcn_s_memtime();
    #define PF4_T(k)                                              \
        do {                                                      \
            const uint64_t t_ = __builtin_amdgcn_s_memtime();     \
            ph[k] += t_ - t_prev;                                 \
            t_prev = t_;                                          \
        } while (0)
    #else
    #define PF4_T(k) do { } while (0)
    #endif
            auto iter = [&](int j, auto first) {
                constexpr bool F = decltype(first)::value;
                PF4_T(7);
                // ---- A_j: S_j for rb 1 (steps 0-15) and rb 0 (16-31); rb 1's
                // exponentials of tile j-1 beside steps 0-15, its scores and max of
                // tile j beside 16-31 (its S chains done by then)
                wait_vmcnt_c<C::NKI + MI>();  // B_{j-1}'s issues (K_{j+2}, mask j+1) may fly
                PF4_T(0);
                // V_{j-1}^T operands for B_j, streamed: operand v (= B's MFMAs of
                // steps 2v, 2v+1); the first four read in A_j after its barrier
                f16x8 va[2][2][NDB];
                uint32_t vb0 = (uint32_t)(C::vOff + (((j > 0 ? j : 1) - 1) % C::VS) * C::img) + vbase[0];
                uint32_t vb1 = (uint32_t)(C::vOff + (((j > 0 ? j : 1) - 1) % C::VS) * C::img) + vbase[1];
                PF4_OPAQUE_V2(vb0, vb1);
                auto v_read1 = [&](int v) {
                    const int t = v >> 3, q = (v >> 2) & 1, db = v & 3;
                    const uint32_t off = db * (kPfKeys * 64) + t * 2048 + q * 1024;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lsm + vb0 + off));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lsm + vb1 + off));
                    const u32x2 a2 = __builtin_bit_cast(u32x2, lo), b2 = __builtin_bit_cast(u32x2, hi);
                    va[t][q][db] = __builtin_bit_cast(f16x8, u32x4{a2.x, a2.y, b2.x, b2.y});
                };
                u32x2 mk1[2][4], mk0[2][4];
                const uint32_t kb = k_base(j);
                // the first four operands: read in B_{j-1}'s last steps (here for
                // tile 0); the rest 4 steps ahead, in the steps
                if constexpr (F) {
#pragma unroll
                    for (int kk = 0; kk < 4; kk++) k_read1(kb, 0, kk);
                }
                const float nm1 = (m_run[1] == kNegInf) ? 0.0f : -m_run[1];
                float la1 = l2[1].x, lb1 = l2[1].y, tmax1 = kNegInf;
                if constexpr (!F) e1(us1, nm1, 0);
                __builtin_amdgcn_sched_barrier(0);
                // steps: rb 1's exponentials of tile j-1 (piece p: stages at steps
                // p-1, p, p+1), its scores and max of tile j (piece p: 15+p, 16+p,
                // 17+p -- S1's subtile-0 chain ended at step 7, subtile 1's at 15);
                // then the step's MFMA
#pragma unroll
                for (int i = 0; i < 32; i++) {
                    const int t = (i >> 3) & 1, kk = i & 7;
                    if (i < 12) k_read1(kb, (i + 4) >> 3, (i + 4) & 7);
                    // the tile's one barrier, mid-A (this wave's K_j reads were
                    // all issued by step 11 and are consumed by step 12's MFMA):
                    // every wave is then past its A_j wait -- V_{j-1}, K_{j+1} and
                    // mask j complete for all -- and done with K_j and V_{j-2}
                    if (i == 12) __syncthreads();
                    if constexpr (!F) {
                        if (i >= 24 && !(i & 1)) v_read1((i - 24) >> 1);  // (after the barrier)
                    }
                    // V_j's DMA (into V_{j-3}'s slot, read in B_{j-2}; needed at B_{j+1}):
                    // the other half of the tile's issue cost beside A's MFMAs
#ifdef FATTN_PF4_VDMA_LATE
                    if (i >= 16 && (i & 3) == 1) v_piece(j, (i - 16) >> 2);
#else
                    if (i < 16 && (i & 3) == 1) v_piece(j, i >> 2);
#endif
                    if constexpr (MM) {
                        if (i == 8) mask_reads(j, 1, mk1);   // (for rb 1's scores, steps 16+)
                        if (i == 14) mask_reads(j, 0, mk0);  // (for B_j: this wave's slot, no barrier needed)
                    }
                    if constexpr (!F) {
                        if (i >= 1 && i <= 16) e3(p1, la1, lb1, i - 1);
                        if (i <= 15) e2(i);
                        if (i <= 14) e1(us1, nm1, i + 1);
                    }
                    if (i >= 17) m3(us1, tmax1, i - 17);
                    if (i >= 16) m2(mk1, us1, i - 16);
                    if (i >= 15 && i <= 30) m1(s1, i - 15);
                    if (i < 16) {
                        if (kk == 0) s1[t] = f32x16{};
                        s1[t] = mfma32(kr[t][kk], qop[1][kk], s1[t]);
                    } else {
                        if (kk == 0) s0[t] = f32x16{};
                        s0[t] = mfma32(kr[t][kk], qop[0][kk], s0[t]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                m3(us1, tmax1, 15);
                PF4_T(1);
                if constexpr (!F) l2[1] = f32x2{la1, lb1};
                // (rb 1's decision of tile j: in B_j's steps 12-13)
                // (the phase's results pinned here: hipcc's machine sinking would
                // otherwise move their exponentials next to their uses in B)
                if constexpr (!F) pin_p(p1);
                pin16(us1[0]);
                pin16(us1[1]);
                PF4_T(2);
                // ---- B_j: P_{j-1}.V for both row blocks (each V^T operand read
                // once); rb 0's scores and max of tile j beside steps 0-15, its
                // exponentials beside 16-31
                PF4_T(3);
                float tmax0 = kNegInf, nm0 = 0.0f, la0 = 0.0f, lb0 = 0.0f;
                f16x8 p0n[2][2];
                const bool mskip = MM ? __builtin_amdgcn_readfirstlane(m_skip(j + 2) ? 1 : 0) != 0 : true;
                PF4_T(4);
                __builtin_amdgcn_sched_barrier(0);
                float tred0 = 0.0f, tred1 = 0.0f;
                const uint32_t kbn = k_base(j + 1);
                // steps: rb 0's scores and max (piece p at slot s(p) = p / 2 for
                // p < 8, p - 4 after: stages at s-1, s, s+1), rb 1's max across the
                // lane pair (12) and rescale decision (13), rb 0's (13, 14), rb 0's
                // exponentials (piece p: 15+p, 16+p, 17+p; the last ones after the
                // loop); then the step's MFMA, operand reads (V^T; K_{j+1}'s first
                // four in 28-31 -- past the end a slot nothing uses) and DMA
                auto slot0 = [](int p) { return p < 8 ? p >> 1 : p - 4; };
                m1(s0, 0);
                m1(s0, 1);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < 32; i++) {
#pragma unroll
                    for (int p = 0; p < 16; p++) {
                        if (slot0(p) + 1 == i) m3(us0, tmax0, p);
                        if (slot0(p) == i) m2(mk0, us0, p);
                        if (slot0(p) - 1 == i) m1(s0, p);
                    }
                    if (i == 12) {
                        tred1 = PF4_XOR32(tmax1, true) * cexp;
                        asm volatile("" : "+v"(tred1));
                    }
                    if (i == 13) {
                        smax_decide(1, tred1, al1, rs1);
                        tred0 = PF4_XOR32(tmax0, true) * cexp;
                        asm volatile("" : "+v"(tred0));
                    }
                    if (i == 14) {
                        smax_decide(0, tred0, al0, rs0);
                        nm0 = (m_run[0] == kNegInf) ? 0.0f : -m_run[0];
                        la0 = l2[0].x;
                        lb0 = l2[0].y;
                        asm volatile("" : "+v"(nm0), "+v"(la0), "+v"(lb0));
                    }
                    if (i >= 17) e3(p0n, la0, lb0, i - 17);
                    if (i >= 16) e2(i - 16);
                    if (i >= 15 && i <= 30) e1(us0, nm0, i - 15);
                    if constexpr (!F) {
                        if (!(i & 1) && i < 24) v_read1((i >> 1) + 4);
                        const int t = i >> 4, q = (i >> 3) & 1, db = (i >> 1) & 3, rb = i & 1;
                        o[rb][db] = mfma32(va[t][q][db], rb ? p1[t][q] : p0[t][q], o[rb][db]);
                    }
                    // this tile's DMA: K_{j+3} and V_{j+1} pieces in steps 1, 3, ..., 15
                    // (into slots every wave finished before the barrier), mask j+2
                    // in steps 17, 19, ..., 31 (this wave's reads of mask j are
                    // consumed by then)
                    if (i < 16 && (i & 3) == 1) k_piece(j + 3, i >> 2);  // (K_{j+3} into K_j's slot; V_j went in A_j)
                    if (i >= 16 && (i & 1)) m_piece(j + 2, (i - 16) >> 1, mskip);
#ifdef FATTN_PF4_KREAD_EARLY
                    if (i >= 5 && i < 9) k_read1(kbn, 0, i - 5);
#else
                    if (i >= 28) k_read1(kbn, 0, i - 28);
#endif
                    __builtin_amdgcn_sched_barrier(0);
                }
                e3(p0n, la0, lb0, 15);  // (piece 15's last stage, after the loop)
                PF4_T(5);
                l2[0] = f32x2{la0, lb0};
                pin_p(p0n);
                rescale_acc(0, rs0, al0);  // the decisions of tile j
                rescale_acc(1, rs1, al1);
#pragma unroll
                for (int t = 0; t < 2; t++) {
#pragma unroll
                    for (int q = 0; q < 2; q++) p0[t][q] = p0n[t][q];
                }
                PF4_T(6);
            };
            // The balanced form (SCHED 3): each phase carries one row block's
            // exponentials and the OTHER row block's scores and max, interleaved
            // over all 32 steps (no dependency between them inside the phase):
            //   A_j: S_j (both)  ||  rb 0's exponentials of tile j-1, rb 1's
            //        scores / max of tile j;
            //   B_j: P_{j-1}.V (both)  ||  rb 1's decision and exponentials of
            //        tile j, rb 0's scores / max / decision of tile j.
            // Per row block the same operations in the same order as the other
            // forms (decision, then the tile's exponentials and sums), so the
            // same bits.  P_{j-1} of rb 0 comes from A_j, of rb 1 from B_{j-1}.
            // Stage steps: A's max pieces from step 9 (S1's subtile-0 chain ends
            // at 7), spread to 31; A's exponential pieces one per two steps; B's
            // rb 1 decision in steps 0-1, its exponentials from 2, rb 0's max
            // pieces over 0-28 and its decision in 29-30.
            // (each schedule s(q) = C + (A q) / B is strictly increasing, so a step
            // holds at most one piece's stage: sched_inv finds it without a loop --
            // a loop over the pieces in every step kept hipcc from unrolling)
            // (diagnostic builds only, outputs wrong: the phases without their
            // vector pieces / without their in-loop DMA -- what the skeleton costs)
#ifdef FATTN_PF4_DIAG_NO_VALU
            constexpr bool kDiagNoValu = true;
#else
            constexpr bool kDiagNoValu = false;
#endif
#ifdef FATTN_PF4_DIAG_NO_DMA
            constexpr bool kDiagNoDma = true;
#else
            constexpr bool kDiagNoDma = false;
#endif
            static_assert(C::KS == 3 && C::VS == 3, "the balanced loop carries j % 3");
            // r0 = j % 3 (K_j, V_j, K_{j+3}: ring slot r0; K_{j+1}: r1; V_{j-1}: rm)
            auto iter_bal = [&](int j, auto first, int r0) {
                constexpr bool F = decltype(first)::value;
                const int r1 = r0 == 2 ? 0 : r0 + 1, rm = r0 == 0 ? 2 : r0 - 1;
                PF4_T(7);
                wait_vmcnt_c<C::NKI + MI>();  // B_{j-1}'s issues (K_{j+2}, mask j+1) may fly
                PF4_T(0);
                f16x8 va[2][2][NDB];
                uint32_t vb0 = (uint32_t)(C::vOff + (F ? 0 : rm) * C::img) + vbase[0];
                uint32_t vb1 = (uint32_t)(C::vOff + (F ? 0 : rm) * C::img) + vbase[1];
                PF4_OPAQUE_V2(vb0, vb1);
                auto v_read1 = [&](int v) {
                    const int t = v >> 3, q = (v >> 2) & 1, db = v & 3;
                    const uint32_t off = db * (kPfKeys * 64) + t * 2048 + q * 1024;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lsm + vb0 + off));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lsm + vb1 + off));
                    const u32x2 a2 = __builtin_bit_cast(u32x2, lo), b2 = __builtin_bit_cast(u32x2, hi);
                    va[t][q][db] = __builtin_bit_cast(f16x8, u32x4{a2.x, a2.y, b2.x, b2.y});
                };
                u32x2 mk1[2][4], mk0[2][4];
                const uint32_t kb = k_base_at(r0);
                if constexpr (F) {
#pragma unroll
                    for (int kk = 0; kk < 4; kk++) k_read1(kb, 0, kk);
                }
                // ---- A_j
                const float nm0 = (m_run[0] == kNegInf) ? 0.0f : -m_run[0];
                // (lean, accumulators in VGPRs: rb 1's -m_ref for its arguments of tile j)
                const float nr1 = (m_run[1] == kNegInf) ? 0.0f : -m_run[1];
                float la0 = l2[0].x, lb0 = l2[0].y, tmax1 = kNegInf;
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < 32; i++) {
                    const int t = (i >> 3) & 1, kk = i & 7;
                    if (i < 12) k_read1(kb, (i + 4) >> 3, (i + 4) & 7);
                    if (i == 12) __syncthreads();
                    if constexpr (!F) {
                        if (i >= 24 && !(i & 1)) v_read1((i - 24) >> 1);
                    }
                    if (!kDiagNoDma && i < 16 && (i & 3) == 1) v_piece_at(j, r0, i >> 2);
                    if constexpr (MM) {
                        if (i == 8) mask_reads(j, 1, mk1);
                        if (i == 14) mask_reads(j, 0, mk0);
                    }
                    if constexpr (!F && !kDiagNoValu) {
                        // rb 0's exponentials of tile j-1: piece p at 2p, 2p+1, 2p+2
                        if (i >= 2 && !(i & 1)) e3(p0, la0, lb0, (i - 2) >> 1);
                        if constexpr (LN) {
                            if (i & 1) e2u(us0, i >> 1);
                        } else {
                            if (i & 1) e2(i >> 1);
                            if (!(i & 1)) e1(us0, nm0, i >> 1);
                        }
                    }
                    if constexpr (!kDiagNoValu) {
                        const int q3 = sched_inv<22, 15, 9>(i - 2), q2 = sched_inv<22, 15, 9>(i - 1),
                                  q1 = sched_inv<22, 15, 9>(i);
                        if (q3 >= 0) m3(us1, tmax1, q3);
                        if constexpr (LN && !MM) {
                            // (the first tile's step 9 reads s1[0] two steps after its
                            // chain's last MFMA with no exponentials between: the
                            // remaining accumulator -> VALU wait states)
                            if (F && FATTN_PF4_SVGPR && i == 9) asm volatile("s_nop 3" : "+v"(s1[0]));
                            if (q1 >= 0) m1u(s1, us1, nr1, q1);
                        } else {
                            if (q2 >= 0) m2(mk1, us1, q2);
                            if (q1 >= 0) m1(s1, q1);
                        }
                    }
                    if (i < 16) {
                        if constexpr (LN && FATTN_PF4_SVGPR) {
                            if (kk == 0) mfma_s_first(s1[t], kr[t][kk], qop[1][kk]);
                            else mfma_s_next(s1[t], kr[t][kk], qop[1][kk]);
                        } else if constexpr (LN) {
                            s1[t] = mfma32(kr[t][kk], qop[1][kk], kk == 0 ? ci[1] : s1[t]);
                        } else if constexpr (LEAN && FATTN_PF4_SVGPR) {
                            if (kk == 0) mfma_s_first(s1[t], kr[t][kk], qop[1][kk]);
                            else mfma_s_next(s1[t], kr[t][kk], qop[1][kk]);
                        } else {
                            if (kk == 0) s1[t] = f32x16{};
                            s1[t] = mfma32(kr[t][kk], qop[1][kk], s1[t]);
                        }
                    } else {
                        if constexpr (LN && FATTN_PF4_SVGPR) {
                            if (kk == 0) mfma_s_first(s0[t], kr[t][kk], qop[0][kk]);
                            else mfma_s_next(s0[t], kr[t][kk], qop[0][kk]);
                        } else if constexpr (LN) {
                            s0[t] = mfma32(kr[t][kk], qop[0][kk], kk == 0 ? ci[0] : s0[t]);
                        } else if constexpr (LEAN && FATTN_PF4_SVGPR) {
                            if (kk == 0) mfma_s_first(s0[t], kr[t][kk], qop[0][kk]);
                            else mfma_s_next(s0[t], kr[t][kk], qop[0][kk]);
                        } else {
                            if (kk == 0) s0[t] = f32x16{};
                            s0[t] = mfma32(kr[t][kk], qop[0][kk], s0[t]);
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if constexpr (!F) e3(p0, la0, lb0, 15);
                {
                    // (the stages of the last pieces past step 31)
                    const int q2 = sched_inv<22, 15, 9>(31), q3a = sched_inv<22, 15, 9>(30),
                              q3b = sched_inv<22, 15, 9>(31);
                    if (q2 >= 0 && !(LN && !MM)) m2(mk1, us1, q2);
                    if (q3a >= 0) m3(us1, tmax1, q3a);
                    if (q3b >= 0) m3(us1, tmax1, q3b);
                }
                if constexpr (LN) {
                    // rb 1's decision of tile j, at A's tail (its exponentials run in B)
                    lean_decide(1, PF4_XOR32(tmax1, true), us1, al1, rs1);
                }
                if constexpr (kDiagNoValu) asm volatile("" ::"v"(s1[0][0]), "v"(s1[1][0]), "v"(s0[0][0]), "v"(s0[1][0]));
                PF4_T(1);
                if constexpr (!F) {
                    l2[0] = f32x2{la0, lb0};
                    pin_p(p0);
                }
                pin16(us1[0]);
                pin16(us1[1]);
                PF4_T(2);
                // ---- B_j
                PF4_T(3);
                float tmax0 = kNegInf, nm1 = 0.0f, la1 = LN ? l2[1].x : 0.0f, lb1 = LN ? l2[1].y : 0.0f;
                const float nr0 = (m_run[0] == kNegInf) ? 0.0f : -m_run[0];
                f16x8 p1n[2][2];
                const bool mskip = MM ? __builtin_amdgcn_readfirstlane(m_skip(j + 2) ? 1 : 0) != 0 : true;
                PF4_T(4);
                __builtin_amdgcn_sched_barrier(0);
                float tred0 = 0.0f, tred1 = 0.0f;
                const uint32_t kbn = k_base_at(r1);
#pragma unroll
                for (int i = 0; i < 32; i++) {
                    if (i == 0 && !LN) {
                        tred1 = PF4_XOR32(tmax1, true) * cexp;
                        asm volatile("" : "+v"(tred1));
                    }
                    if (i == 1 && !LN) {
                        smax_decide(1, tred1, al1, rs1);
                        nm1 = (m_run[1] == kNegInf) ? 0.0f : -m_run[1];
                        la1 = l2[1].x;
                        lb1 = l2[1].y;
                        asm volatile("" : "+v"(nm1), "+v"(la1), "+v"(lb1));
                    }
                    if constexpr (!kDiagNoValu) {
                        const int e3p = sched_inv<28, 15, 2>(i - 2), e2p = sched_inv<28, 15, 2>(i - 1),
                                  e1p = sched_inv<28, 15, 2>(i);
                        const int m3p = sched_inv<26, 15, 0>(i - 2), m2p = sched_inv<26, 15, 0>(i - 1),
                                  m1p = sched_inv<26, 15, 0>(i);
                        if (e3p >= 0) e3(p1n, la1, lb1, e3p);
                        if constexpr (LN) {
                            if (e2p >= 0) e2u(us1, e2p);
                        } else {
                            if (e2p >= 0) e2(e2p);
                            if (e1p >= 0) e1(us1, nm1, e1p);
                        }
                        if (m3p >= 0) m3(us0, tmax0, m3p);
                        if constexpr (LN && !MM) {
                            if (m1p >= 0) m1u(s0, us0, nr0, m1p);
                        } else {
                            if (m2p >= 0) m2(mk0, us0, m2p);
                            if (m1p >= 0) m1(s0, m1p);
                        }
                    }
                    if (i == 29 && !LN) {
                        tred0 = PF4_XOR32(tmax0, true) * cexp;
                        asm volatile("" : "+v"(tred0));
                    }
                    if (i == 30 && !LN) smax_decide(0, tred0, al0, rs0);
                    if constexpr (!F) {
                        if (!(i & 1) && i < 24) v_read1((i >> 1) + 4);
                        const int t = i >> 4, q = (i >> 3) & 1, db = (i >> 1) & 3, rb = i & 1;
                        o[rb][db] = mfma32(va[t][q][db], rb ? p1[t][q] : p0[t][q], o[rb][db]);
                    }
                    if (!kDiagNoDma && i < 16 && (i & 3) == 1) k_piece_at(j + 3, r0, i >> 2);
                    if (!kDiagNoDma && i >= 16 && (i & 1)) m_piece(j + 2, (i - 16) >> 1, mskip);
                    if (i >= 28) k_read1(kbn, 0, i - 28);
                    __builtin_amdgcn_sched_barrier(0);
                }
                {
                    // (the stages of the last pieces past step 31)
                    const int e2p = sched_inv<28, 15, 2>(31), e3a = sched_inv<28, 15, 2>(30),
                              e3b = sched_inv<28, 15, 2>(31);
                    if (e2p >= 0) {
                        if constexpr (LN) e2u(us1, e2p);
                        else e2(e2p);
                    }
                    if (e3a >= 0) e3(p1n, la1, lb1, e3a);
                    if (e3b >= 0) e3(p1n, la1, lb1, e3b);
                }
                PF4_T(5);
                l2[1] = f32x2{la1, lb1};
                pin_p(p1n);
                if constexpr (LN) {
                    // rb 0's decision of tile j, at B's tail (its exponentials run in A_{j+1})
                    lean_decide(0, PF4_XOR32(tmax0, true), us0, al0, rs0);
                }
                pin16(us0[0]);
                pin16(us0[1]);
                rescale_acc(0, rs0, al0);  // the decisions of tile j
                rescale_acc(1, rs1, al1);
#pragma unroll
                for (int t = 0; t < 2; t++) {
#pragma unroll
                    for (int q = 0; q < 2; q++) p1[t][q] = p1n[t][q];
                }
                PF4_T(6);
            };
#ifdef FATTN_STAMPS
            kt_loop0 = __builtin_amdgcn_s_memtime();
#endif
            if constexpr (SCHED >= 3) {
                if (nt > 0) iter_bal(0, std::true_type(), 0);
                int r0 = 0;
                for (int j = 1; j < nt; j++) {
                    r0 = r0 == 2 ? 0 : r0 + 1;  // (j % 3)
                    iter_bal(j, std::false_type(), r0);
                }
                if (nt > 0) {
                    // ---- A_nt, B_nt: rb 0's exponentials of the last tile, its P.V
                    wait_vmcnt_c<0>();
                    sexp(0, 0, us0, p0, LN);
                    sexp(0, 1, us0, p0, LN);
                    __syncthreads();  // every wave's pieces of V nt-1 landed
                    pv2(nt - 1, p0, p1);
                }
            } else {
            if (nt > 0) iter(0, std::true_type());
            for (int j = 1; j < nt; j++) iter(j, std::false_type());
            if (nt > 0) {
                // ---- A_nt, B_nt: rb 1's exponentials of the last tile, its P.V
                wait_vmcnt_c<0>();
                sexp(1, 0, us1, p1, false);
                sexp(1, 1, us1, p1, false);
                __syncthreads();  // every wave's pieces of V nt-1 landed
                pv2(nt - 1, p0, p1);  // (tile nt-1's rescale: at the end of B_{nt-1})
            }
            }
    #ifdef FATTN_STAMPS
            kt_loop1 = __builtin_amdgcn_s_memtime();
            if (lane == 0 && g_stamps) {
                const int64_t blk = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
                for (int k = 0; k < 8; k++) g_stamps[(blk * kPfWaves + wave) * 16 + k] = ph[k];
                g_stamps[(blk * kPfWaves + wave) * 16 + 8] = (unsigned long long)nt;
            }
    #endif
    #undef PF4_T
        };
        if constexpr (HM) {
            if (__builtin_amdgcn_readfirstlane(all_zero ? 1 : 0)) body2(std::true_type());
            else body2(std::false_type());
        } else {
            body2(std::false_type());
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

    // ---- normalise, park the wave's 64 rows in LDS, store whole rows
    // (one instruction = 1 KiB of contiguous row bytes: fattn_pf.h's epilogue)
    constexpr int kStride = D + 4;
    __syncthreads();  // every wave is done with the rings
    float* park = (float*)smem + wave * (kPf4RowsW * kStride);
#pragma unroll
    for (int rb = 0; rb < 2; rb++) {
        const float l_tot = PF4_XOR32(l2[rb].x + l2[rb].y, false);
        const float inv = 1.0f / l_tot;  // fully masked row -> NaN like the reference
        float* pk = park + (32 * rb + c32) * kStride + 4 * h;
#pragma unroll
        for (int db = 0; db < NDB; db++) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; r++) v[r] = l_tot == 0.0f ? __builtin_nanf("") : o[rb][db][4 * u + r] * inv;
                *(f32x4*)(pk + 32 * db + 8 * u) = v;
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (the wave reads back only its own rows)
    constexpr int CPR = D / 4;  // 16-B chunks of a dst row
#pragma unroll
    for (int i = 0; i < kPf4RowsW * CPR / kWave; i++) {
        const int g = kWave * i + lane;
        const int r = g / CPR, c = g % CPR;
        int q1, q2;
        if (row_of(kPf4RowsW * wave + r, q1, q2)) {
            const f32x4 v = *(const f32x4*)(park + r * kStride + 4 * c);
            *(f32x4*)(a.dst + (((int64_t)iq3 * a.NQ + q1) * a.H + q2) * D + 4 * c) = v;
        }
    }
#ifdef FATTN_STAMPS
    if (lane == 0 && g_stamps) {
        const uint64_t kt_exit = __builtin_amdgcn_s_memtime(), kr_exit = __builtin_amdgcn_s_memrealtime();
        const int64_t blk = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        unsigned long long* g = g_stamps + (blk * kPfWaves + wave) * 16;
        g[9] = kt_entry;
        g[10] = kt_loop0;
        g[11] = kt_loop1;
        g[12] = kt_exit;
        g[13] = kr_entry;
        g[14] = kr_exit;
        // HW_ID (CU, SIMD, shader engine) and XCC_ID
        g[15] = (unsigned long long)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                ((unsigned long long)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
    }
#endif
}

}  // namespace fattn
