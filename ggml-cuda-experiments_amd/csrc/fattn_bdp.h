// fattn_bdp.h -- batched decode over ggml-quantised KV with the dequantisation
// taken off the compute waves' path (gfx950).  Same problem and math as
// fattn_bd.h (64 packed (query row x q-head) rows of one kv head per
// workgroup, BASELINE config 5 and its head shards; replaces
// flash_attn_ext_f16<D,Q,C>, src/flash-llama.h:5-438, whose 16-row Q tiles
// re-read K/V per 16 rows):
//
//  * one workgroup = 8 waves with fixed roles, one pair per SIMD: waves 0-3
//    COMPUTE (wave c: row group c & 1 = 32 rows, key half c >> 1 = 32 keys of
//    every 64-key tile), waves 4-7 BUILD (wave 4 + w: half-blocks w, w + 4,
//    ... of every key, K and V -- at D = 128 two, at D = 64 one);
//  * per 64-key tile s, between two workgroup barriers, the compute waves run
//    S^T = K.Q^T, the online softmax and O^T += V^T.P^T on tile s (one image
//    pair) while the build waves issue raw tile s + nRaw into the raw slot
//    they all finished reading before the barrier and dequantise raw tile
//    s + 1 into the other pair -- the dequantisation VALU of one SIMD partner
//    runs beside the matrix work of
//    the other, and there is ONE barrier per tile (fattn_bd.h: the whole
//    workgroup dequantises 128-key tile s between two barriers and then
//    computes it, every SIMD idle on one pipe in each phase);
//  * HBM -> LDS by buffer_load ... lds: raw tiles (nRaw in flight -- as many
//    as the LDS holds, Q8_0 4, Q4_0 5 -- issued by the build waves), each
//    compute wave's 32 x 32 mask block (two tiles in
//    flight, by the compute wave itself), Q's 64 f32 rows once before the loop
//    (by all waves, into the second image pair's place);
//  * dequantisation h(q * d) with one f16 rounding (src/utils.h:10-11), images
//    and operand reads exactly as fattn_bd.h / fattn_pf.h (64-key images);
//  * epilogue: bd_finish over the two key halves (whole-row stores; partials
//    merged by fattn_bd_merge_kernel when the KV is split).
//
// LDS (D = 128, Q8_0): [0, 64 KiB) two image pairs (K [8 dim slices][64 keys]
// [32 B], V [4 dim blocks][64 keys][64 B]), then nRaw = 4 raw tiles [K rows |
// V rows] of 17 KiB, then 4 compute waves x 2 mask slots of 2 KiB: 148 KiB.
#pragma once

#include "fattn_bd.h"

namespace fattn {

constexpr int kBdpKeys = 64;      // keys per tile (two 32-key halves)
constexpr int kBdpCompute = 4;    // waves 0..3 compute, 4..7 build
#ifndef FATTN_BDP_MAX_RAW
#define FATTN_BDP_MAX_RAW 5
#endif
constexpr int kBdpMaxRaw = FATTN_BDP_MAX_RAW;  // (diagnostic builds lower it for A/B runs)

template <int KT, int D>
struct BdpCfg {
    static_assert(D == 64 || D == 96 || D == 128, "half-blocks dealt over the build waves; 16-B Q chunks");
    static_assert(KT == FATTN_TYPE_Q8_0 || KT == FATTN_TYPE_Q4_0, "quantised K/V (f16 takes fattn_bd.h's image ring)");
    static constexpr int rowB = row_bytes<KT, D>();
    static constexpr int kvRaw = kBdpKeys * rowB;                // raw K (or V) bytes per tile
    static constexpr int rawBytes = (2 * kvRaw + 15) / 16 * 16;  // [K rows | V rows]
    static constexpr int img = kBdpKeys * D * 2;                 // one f16 image
    static constexpr int pair = 2 * img;
    static constexpr int rawOff = 2 * pair;
    static constexpr int maskSlot = 2048;                        // [4 key octets][32 rows][16 B]
    static constexpr int maskBytes = kBdpCompute * 2 * maskSlot;
    // raw tiles in flight: as many as the LDS holds beside the images and the
    // mask slots, at most kBdpMaxRaw (Q8_0: 4 x 17 KiB, Q4_0: 5 x 9 KiB)
    static constexpr int nRawFit = (163840 - rawOff - maskBytes) / rawBytes;
    static constexpr int nRaw = nRawFit < kBdpMaxRaw ? nRawFit : kBdpMaxRaw;
    static constexpr int maskOff = rawOff + nRaw * rawBytes;
    static constexpr int maskEnd = maskOff + maskBytes;
    static constexpr int ldsBytes = maskEnd > BdPark<D, 2>::bytes ? maskEnd : BdPark<D, 2>::bytes;
    static constexpr int qOff = pair;                            // Q's f32 rows before the loop (pair 1)
    static constexpr int NI = (kvRaw + 1023) / 1024;             // 1-KiB DMA instructions per K (or V) tile
    // Raw instructions j = 0 .. T - 1 (K then V) of a tile, issued by the build
    // waves, j -> 4 + j % 4.  (FATTN_BDP_ALL_ISSUE, A/B builds: from 8 of them
    // on ALL eight waves issue them, j -> wave j % 8, the remainder to the
    // build waves first -- or one more to every compute wave when more than
    // four are left -- so the compute waves' counts are equal: their waits sit
    // right behind the youngest group and must count it exactly.  The issue
    // of the build waves alone stalls ~1.2 us per tile on config 5 (a full
    // memory pipeline), but spreading it over all waves made the compute
    // waves stall as long: 25.1 vs 24.4 us, profiles/r04_e.)  The smallest
    // per-role count counts the waits (a build wave with one more instruction
    // also waits for one of a younger group: fattn_pf.h).
    static constexpr int T = 2 * NI;
#ifdef FATTN_BDP_ALL_ISSUE
    static constexpr bool kAll = T >= 8;  // diagnostic build only (A/B)
#else
    static constexpr bool kAll = false;
#endif
    static constexpr int kBase = T / 8, kRem = T % 8;
    static constexpr int owner(int j) {
        return !kAll ? 4 + j % 4
               : j < 8 * kBase ? j % 8
               : kRem <= 4     ? 4 + (j - 8 * kBase)
               : j - 8 * kBase < 4 ? j - 8 * kBase
                                   : 4 + (j - 8 * kBase - 4);
    }
    static constexpr int R_c = kAll ? kBase + (kRem > 4 ? 1 : 0) : 0;  // per compute wave (exact)
    static constexpr int R_b = kAll ? kBase : T / 4;                   // per build wave (smallest)
    static constexpr int NM = 2;                                 // mask DMA instructions per compute wave and tile
    static_assert(kBdRows * D * 4 <= pair, "Q rows in the second pair's place");
    static_assert(nRaw >= 3, "a compute wave's raw s + 2 is older than its mask s + 1");
    static_assert(ldsBytes <= 163840, "");
};

// (the K/V DMA without the non-temporal policy: config 5 24.4-24.7 vs
// 25.1-25.3 us with it, profiles/r04_d)
constexpr bool kBdpNT = false;

// this wave's raw instructions of the tile at key n0 (BdpCfg::owner)
template <int KT, int D>
__device__ __forceinline__ void bdp_issue(const StepSrc& rs, int n0, uint32_t lds, int wave, int lane) {
#ifdef FATTN_MQ_NOMEM
    return;  // diagnostic build only
#endif
    using C = BdpCfg<KT, D>;
#pragma unroll
    for (int j = 0; j < C::T; j++) {
        if (C::owner(j) != wave) continue;  // wave-uniform
        const bool is_v = j >= C::NI;
        const int i = is_v ? j - C::NI : j;
        const int byte = i * 1024 + lane * 16;
        if (C::kvRaw % 1024 == 0 || byte < C::kvRaw)  // pieces past the tile's bytes idle (the instruction counts)
            dma<16, kBdpNT>(is_v ? rs.v : rs.k, lds + (is_v ? C::kvRaw : 0) + i * 1024, (uint32_t)n0 * C::rowB + byte);
    }
}

// build wave bw: half-blocks hb = bw, bw + 4, ... (< D / 16) of key `lane` --
// half hb & 1 of ggml block hb >> 1 -- K into dim slice hb and V into dim
// block hb >> 1, in the layouts fattn_bd.h / fattn_pf.h read (D = 96: waves 4
// and 5 take two half-blocks, waves 6 and 7 one).  In two steps: the LDS reads
// of the raw words (bdp_dequant_load) go before the wave's DMA issue of the
// next raw tile, which stalls on a full memory pipeline (profiles/r04_c), so
// their latency runs under that stall; bdp_dequant_store converts and writes.
constexpr int kBdpHpw = 2;  // half-blocks per build wave, at most (D <= 128)
// Image swizzles of this kernel's dequantised tiles (tools/lds_model_bdp.py):
// K rows (32 B) hold their two 16-B halves swapped when bit 2 ^ bit 3 of the
// key is set, V rows (64 B) hold chunk c at c ^ ((key >> 1) & 3).  Both make
// the build waves' b128 image writes (8 consecutive keys per bank cycle) AND
// the compute waves' operand reads conflict-free; fattn_bd.h / fattn_pf.h's
// swizzles (bit 3; key >> 2) left the writes 2-way conflicted (27 % + 27 % of
// the modelled excess cycles; round-4 counters: 36 % of LDS-active cycles in
// conflicts).  FATTN_BDP_OLD_SWZ (A/B builds): the old ones.
#ifdef FATTN_BDP_OLD_SWZ
__host__ __device__ constexpr int bdp_kswz(int key) { return (key >> 3) & 1; }
__host__ __device__ constexpr int bdp_vswz(int key) { return (key >> 2) & 3; }
#else
__host__ __device__ constexpr int bdp_kswz(int key) { return ((key >> 2) ^ (key >> 3)) & 1; }
__host__ __device__ constexpr int bdp_vswz(int key) { return (key >> 1) & 3; }
#endif
struct BdpRaw {
    HalfRaw k[kBdpHpw], v[kBdpHpw];
};
template <int KT, int D>
__device__ __forceinline__ BdpRaw bdp_dequant_load(const uint8_t* raw, int bw, int lane) {
    using C = BdpCfg<KT, D>;
    static_assert((D / 16 + 3) / 4 <= kBdpHpw, "");
    BdpRaw r;
#pragma unroll
    for (int i = 0; i < (D / 16 + 3) / 4; i++) {
        const int hb = bw + 4 * i;
        if (hb >= D / 16) break;  // wave-uniform
        r.k[i] = dequant_half_load<KT, D>(raw, lane, hb >> 1, hb & 1);
        r.v[i] = dequant_half_load<KT, D>(raw + C::kvRaw, lane, hb >> 1, hb & 1);
    }
    return r;
}
template <int KT, int D>
__device__ __forceinline__ void bdp_dequant_store(const BdpRaw& r, uint8_t* k16, uint8_t* v16, int bw, int lane) {
#ifdef FATTN_MQ_NODEQ
    return;  // diagnostic build only
#endif
    const int sk = bdp_kswz(lane), sv = bdp_vswz(lane);
#pragma unroll
    for (int i = 0; i < (D / 16 + 3) / 4; i++) {
        const int hb = bw + 4 * i;
        if (hb >= D / 16) break;  // wave-uniform
        const int b = hb >> 1, h = hb & 1;
        u32x4 ck[2], cv[2];
        dequant_half_cvt<KT>(r.k[i], h, ck);
        dequant_half_cvt<KT>(r.v[i], h, cv);
        uint8_t* kd = k16 + hb * (kBdpKeys * 32) + lane * 32;
        *(u32x4*)(kd + sk * 16) = ck[0];
        *(u32x4*)(kd + (sk ^ 1) * 16) = ck[1];
        uint8_t* vd = v16 + b * (kBdpKeys * 64) + lane * 64;
        *(u32x4*)(vd + ((2 * h) ^ sv) * 16) = cv[0];
        *(u32x4*)(vd + ((2 * h + 1) ^ sv) * 16) = cv[1];
    }
}
template <int KT, int D>
__device__ __forceinline__ void bdp_dequant(const uint8_t* raw, uint8_t* k16, uint8_t* v16, int bw, int lane) {
    bdp_dequant_store<KT, D>(bdp_dequant_load<KT, D>(raw, bw, lane), k16, v16, bw, lane);
}

// build waves: at most n (0 .. nRaw - 1) raw groups issued after the awaited one in flight
template <int KT, int D>
__device__ __forceinline__ void bdp_build_wait(int n) {
    constexpr int NI = BdpCfg<KT, D>::R_b;
    constexpr int NR = BdpCfg<KT, D>::nRaw;
    static_assert(NR >= 2 && NR <= 5, "");
    if (NR >= 5 && n >= 4) wait_vmcnt_c<4 * NI>();
    else if (NR >= 4 && n >= 3) wait_vmcnt_c<3 * NI>();
    else if (NR >= 3 && n >= 2) wait_vmcnt_c<2 * NI>();
    else if (n >= 1) wait_vmcnt_c<NI>();
    else wait_vmcnt_c<0>();
}

// compute waves: at most `raws` raw groups (R_c instructions each) and `masks`
// (0 / 1) mask groups issued after the awaited instruction in flight
template <int KT, int D, int NM>
__device__ __forceinline__ void bdp_compute_wait(int raws, int masks) {
    constexpr int R = BdpCfg<KT, D>::R_c;
    switch (__builtin_amdgcn_readfirstlane(2 * raws + masks)) {
        case 0: wait_vmcnt_c<0>(); break;
        case 1: wait_vmcnt_c<NM>(); break;
        case 2: wait_vmcnt_c<R>(); break;
        case 3: wait_vmcnt_c<R + NM>(); break;
        case 4: wait_vmcnt_c<2 * R>(); break;
        case 5: wait_vmcnt_c<2 * R + NM>(); break;
        case 6: wait_vmcnt_c<3 * R>(); break;
        case 7: wait_vmcnt_c<3 * R + NM>(); break;
        case 8: wait_vmcnt_c<4 * R>(); break;
        case 9: wait_vmcnt_c<4 * R + NM>(); break;
        default: wait_vmcnt_c<0>(); break;  // (not reached: raws <= nRaw - 1 <= 4)
    }
}

template <int KT, int D, bool HM>
__global__ __launch_bounds__(kBdWaves* kWave, 2) void fattn_bdp_kernel(const SplitArgs a) {
    using C = BdpCfg<KT, D>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NK = D / 16;   // 16-dim k-steps of S^T = K.Q^T
    constexpr int NDB = D / 32;  // 32-dim blocks of O^T
    constexpr int NM = HM ? C::NM : 0;
    constexpr float kNegInf = -__builtin_inff();
    constexpr float kDeferLog2 = 8.0f;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool compute = wave < kBdpCompute;  // wave-uniform role
    const int rg = wave & 1, kh = (wave >> 1) & 1;  // compute waves: row group, key half
    const int bw = wave - kBdpCompute;              // build waves: ggml block
    const int h = lane >> 5;
    const int c32 = lane & 31;
    FATTN_STAMP(0);

    // ---- tile decode (fattn_bd.h)
    int chunk, y, iq3;
    tile_coords(a, chunk, y, iq3);
    if (a.merge_launch == 2 && tid == 0) arrival_begin(a, (int64_t)iq3 * gridDim.y + y);
    int qt = 0, ik2 = y, ik3 = iq3;
    if (a.n_qt != 1) {
        qt = y % a.n_qt;
        ik2 = y / a.n_qt;
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;
    const int p = kBdRowsW * rg + c32;  // compute waves: this lane's packed row
    const int rq0 = div_R(a, p);
    const int iq1 = qt * a.QPT + rq0;
    const bool row_ok = rq0 < a.QPT && iq1 < a.NQ;  // (R not a power of two: rows past QPT * R are none)

    const int c_lo = chunk * a.chunk_len;
    const int c_hi = min(a.N, c_lo + a.chunk_len);
    const int ntiles = c_hi > c_lo ? (c_hi - c_lo + kBdpKeys - 1) / kBdpKeys : 0;

    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    rs.m = make_srd(a.mask, HM ? a.m_span : 0);
    const uint32_t lds0 = lds_addr(smem);
    auto raw_lds = [&](int s) { return lds0 + C::rawOff + (s % C::nRaw) * C::rawBytes; };
    auto raw_ptr = [&](int s) { return smem + C::rawOff + (s % C::nRaw) * C::rawBytes; };

    // ---- Q: 64 f32 rows -> LDS (pair 1's place) by D / 4 1-KiB DMA
    // instructions, D / 32 per wave; 16-B chunk g = 64 j + lane of the image is
    // chunk c = g % CPR of row g / CPR (CPR = D / 4 chunks a row), holding the
    // row's chunk c ^ (row & SW) (fattn_bd.h's layout; SW = swz_mask(CPR): 31,
    // 15 and 7 at D = 128, 64, 96)
    constexpr int CPR = D / 4;
    constexpr int SW = swz_mask(CPR);
    {
        const i32x4 qs = make_srd(a.q + (int64_t)iq3 * a.q_nb3, a.q_span);
        constexpr int kQInst = kBdRows * D * 4 / 1024;
        static_assert(kQInst % kBdWaves == 0, "");
#pragma unroll
        for (int i = 0; i < kQInst / kBdWaves; i++) {
            const int j = wave + kBdWaves * i;
            const int g = kWave * j + lane;
            const int pr = g / CPR, cc = g % CPR;
            const int rq = div_R(a, pr);
            const int q1 = qt * a.QPT + rq, q2 = ik2 * a.rk2 + (pr - rq * a.R);
            const uint32_t off = rq < a.QPT && q1 < a.NQ ? (uint32_t)q1 * (uint32_t)a.q_nb1 + (uint32_t)q2 * (uint32_t)a.q_nb2 +
                                                 ((cc ^ (pr & SW)) * 16)
                                           : a.q_span;
            dma<16>(qs, lds0 + C::qOff + j * 1024, off);
        }
    }

    // ---- compute waves' mask blocks: rows 32 rg + c32, keys 32 kh .. + 32 of a
    // tile, slot (wave, s & 1); DMA instruction i, lane l: octet 2 i + (l >> 5)
    const uint32_t mslot0 = lds0 + C::maskOff + (wave & 3) * 2 * C::maskSlot;
    uint32_t mrow_l;
    mrow_l = row_ok ? (uint32_t)iq1 * (uint32_t)a.m_nb1 : a.m_span;
    auto mask_issue = [&](int s) {
        if constexpr (HM) {
            const uint32_t n2 = (uint32_t)(c_lo + s * kBdpKeys + 32 * kh) * 2;
#pragma unroll
            for (int i = 0; i < 2; i++)
                dma<16>(rs.m, mslot0 + (s & 1) * C::maskSlot + i * 1024,
                        mrow_l == a.m_span ? a.m_span : mrow_l + n2 + 16 * (2 * i + h));
        }
    };

    // ---- prologue.  Compute waves: Q | mask 0 | mask 1 | their pieces of raw
    // 0 .. nRaw - 1.  Build waves: Q | their pieces of raw 0 .. nRaw - 1; after
    // the barrier that completes raw 0 they dequantise it into pair 0.
    const int npro = min(C::nRaw, ntiles);  // raw tiles of the prologue
    if (compute) {
        if (ntiles > 0) mask_issue(0);
        if (ntiles > 1) mask_issue(1);
    }
    for (int t = 0; t < npro; t++) bdp_issue<KT, D>(rs, c_lo + t * kBdpKeys, raw_lds(t), wave, lane);
    FATTN_STAMP(1);
    // Q, (masks 0 and 1,) this wave's pieces of raw 0 landed
    if (compute) bdp_compute_wait<KT, D, NM>(max(npro - 1, 0), 0);
    else bdp_build_wait<KT, D>(npro - 1);
    __syncthreads();  // Q and raw 0 complete in LDS
    f16x8 qop[NK];
    if (compute) {
#pragma unroll
        for (int kk = 0; kk < NK; kk++) {
            const float* qr = (const float*)(smem + C::qOff) + p * D;
            const f32x4 x0 = *(const f32x4*)(qr + 4 * ((4 * kk + 2 * h) ^ (p & SW)));
            const f32x4 x1 = *(const f32x4*)(qr + 4 * ((4 * kk + 2 * h + 1) ^ (p & SW)));
            f16x8 hq;
            hq.s0 = (f16)x0.x; hq.s1 = (f16)x0.y; hq.s2 = (f16)x0.z; hq.s3 = (f16)x0.w;
            hq.s4 = (f16)x1.x; hq.s5 = (f16)x1.y; hq.s6 = (f16)x1.z; hq.s7 = (f16)x1.w;
            qop[kk] = hq;
        }
        // this wave's pieces of raw 1 landed (the build waves dequantise it
        // after the loop's first barrier)
        if (ntiles > 1) bdp_compute_wait<KT, D, NM>(npro - 2, 0);
    } else {
        if (ntiles > 0) {
            bdp_dequant<KT, D>(raw_ptr(0), smem, smem + C::img, bw, lane);
            // raw 1 landed (raw 2 .. nRaw - 1 may fly on).  Raw nRaw goes into
            // slot 0 after the loop's first barrier: every build wave reads all
            // of a slot's rows, so a slot is free only once they all have.
            if (ntiles > 1) bdp_build_wait<KT, D>(npro - 2);
        }
    }
    FATTN_STAMP(2);

    float m_run = kNegInf;    // compute waves: reference max (log2 domain) of this lane's row
    f32x2 l2 = {0.0f, 0.0f};  // this lane's partial row sums
    f32x16 o[NDB];
#pragma unroll
    for (int db = 0; db < NDB; db++) {
#pragma unroll
        for (int j = 0; j < 16; j++) o[db][j] = 0.0f;
    }
    const float log2e = 1.4426950408889634f;
    const float scale = a.scale;
    // per-lane K read base (key 32 kh + c32, half h; halves swapped per
    // bdp_kswz) and V^T gather bases (fattn_bd.h's gather, 64-key images,
    // chunks swizzled per bdp_vswz: keys 32 kh + 16 q + row, the first two
    // terms leave bits 1-2 alone)
    const uint32_t kbase = kh * 1024 + c32 * 32 + ((h ^ bdp_kswz(c32)) * 16);
    const int gi = lane & 15, dh = (lane >> 4) & 1;
    uint32_t vbase[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int row = 8 * e + 4 * h + (gi >> 2);
        const int ch = (2 * dh + ((gi & 3) >> 1)) ^ bdp_vswz(row);
        vbase[e] = C::img + kh * 2048 + row * 64 + ch * 16 + (gi & 1) * 8;
    }

    // (diagnostic build only, FATTN_STAMPS, tools/stamps_bd.py --form bdp: 0
    // start, 1 prologue issued, 2 prologue done, 3 + s past tile s's barrier,
    // 7 + s tile s's work done -- compute: tile s computed and mask s + 1
    // landed; build: raw s + 1 dequantised and raw s + 2 landed -- (s < 4),
    // 11 loop done, 12 states parked, 13 partials stored; build waves, tile 2:
    // 14 before and 15 after issuing raw 2 + nRaw)
    for (int s = 0; s < ntiles; s++) {
        // pair s % 2 holds tile s (built before this barrier by the build
        // waves); every compute wave is done with tile s - 1, so pair
        // (s + 1) % 2 is free; raw s + 1 is complete (its build waves waited)
        __syncthreads();
        if (s < 4) FATTN_STAMP(3 + s);
        // build waves: the raw words of tile s + 1 read first (their latency
        // runs under the DMA issue below)
        BdpRaw deq;
#ifndef FATTN_BDP_READ_LATE
        if (!compute && s + 1 < ntiles) deq = bdp_dequant_load<KT, D>(raw_ptr(s + 1), bw, lane);
#endif
        // every wave: its pieces of raw s + nRaw into raw s's slot (every build
        // wave read it before this barrier)
        if (s == 2) FATTN_STAMP(14);
        if (s + C::nRaw < ntiles) bdp_issue<KT, D>(rs, c_lo + (s + C::nRaw) * kBdpKeys, raw_lds(s + C::nRaw), wave, lane);
        if (s == 2) FATTN_STAMP(15);
#ifdef FATTN_BDP_READ_LATE
        // diagnostic build only (A/B): the raw words read after the DMA issue
        if (!compute && s + 1 < ntiles) deq = bdp_dequant_load<KT, D>(raw_ptr(s + 1), bw, lane);
#endif
        if (!compute) {
            // ---- build: raw s + 1 -> pair (s + 1) % 2; then wait for this
            // wave's pieces of raw s + 2 (raw s + 3 .. s + nRaw may fly on)
            if (s + 1 < ntiles) {
                bdp_dequant_store<KT, D>(deq, smem + ((s + 1) & 1) * C::pair, smem + ((s + 1) & 1) * C::pair + C::img, bw,
                                         lane);
                if (s + 2 < ntiles) bdp_build_wait<KT, D>(min(C::nRaw - 2, ntiles - 3 - s));
            }
            if (s < 4) FATTN_STAMP(7 + s);
            continue;
        }
        // ---- compute tile s.  This lane's mask values (keys 8 u + 4 h + 0..3 of
        // the half) out of slot s & 1 (landed: waited for before the barrier),
        // then mask s + 2 into that slot
        const uint32_t pofs = (s & 1) * C::pair;
        u32x2 mh[4];
        uint32_t open = 1;  // any key not at -inf (f16 0xFC00)
        if constexpr (HM) {
            open = 0;
            const uint8_t* ms = smem + C::maskOff + (wave & 3) * 2 * C::maskSlot + (s & 1) * C::maskSlot + c32 * 16 + h * 8;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                mh[u] = *(const u32x2*)(ms + u * 512);
                open |= (mh[u].x ^ 0xFC00FC00u) | (mh[u].y ^ 0xFC00FC00u);
            }
#ifndef FATTN_BDP_MASK_LATE
            if (s + 2 < ntiles) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot has been read
                mask_issue(s + 2);
            }
#endif
        }
        // this wave's 32 keys past the chunk, or -inf for every valid row: nothing to add (exact)
        const bool live = c_lo + s * kBdpKeys + 32 * kh < c_hi &&
                          (!HM || __builtin_amdgcn_ballot_w64(open != 0 && row_ok) != 0);
        if (live) {
            f16x8 ka[NK];
#pragma unroll
            for (int kk = 0; kk < NK; kk++) ka[kk] = *(const f16x8*)(smem + pofs + kk * (kBdpKeys * 32) + kbase);
            __builtin_amdgcn_sched_barrier(0);
            f32x16 st;
#pragma unroll
            for (int j = 0; j < 16; j++) st[j] = 0.0f;
#pragma unroll
            for (int kk = 0; kk < NK; kk++) st = mfma32(ka[kk], qop[kk], st);

            // u = scale * s + mask (natural units); element j = key 8 (j/4) + 4 h + j%4
            float u[16];
#pragma unroll
            for (int uu = 0; uu < 4; uu++) {
                if constexpr (HM) {
                    const f16x2 m01 = as_h2(mh[uu].x), m23 = as_h2(mh[uu].y);
                    u[4 * uu + 0] = fmaf(st[4 * uu + 0], scale, (float)m01.x);
                    u[4 * uu + 1] = fmaf(st[4 * uu + 1], scale, (float)m01.y);
                    u[4 * uu + 2] = fmaf(st[4 * uu + 2], scale, (float)m23.x);
                    u[4 * uu + 3] = fmaf(st[4 * uu + 3], scale, (float)m23.y);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; r++) u[4 * uu + r] = st[4 * uu + r] * scale;
                }
            }
            float tmax = kNegInf;
#pragma unroll
            for (int j = 0; j < 16; j++) tmax = fmaxf(tmax, u[j]);
            tmax = xor32_pair(tmax, true) * log2e;
            // deferred max (cdna_hip_programming.md T13), the whole previous
            // tile's P.V already accumulated
            if (__builtin_amdgcn_ballot_w64(tmax > m_run + kDeferLog2)) {
                const float m_new = fmaxf(m_run, tmax);
                const float alpha = (m_new == kNegInf) ? 1.0f : __builtin_amdgcn_exp2f(m_run - m_new);
                l2 *= alpha;
#pragma unroll
                for (int db = 0; db < NDB; db++) o[db] *= alpha;
                m_run = m_new;
            }
            const float nm = (m_run == kNegInf) ? 0.0f : -m_run;
            f16x8 pb[2];
            {
                float pv[16];
#pragma unroll
                for (int j = 0; j < 16; j++) pv[j] = __builtin_amdgcn_exp2f(fmaf(u[j], log2e, nm));
#pragma unroll
                for (int j = 0; j < 16; j += 2) l2 += f32x2{pv[j], pv[j + 1]};
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    f16x8 x;
                    x.s0 = (f16)pv[8 * q]; x.s1 = (f16)pv[8 * q + 1]; x.s2 = (f16)pv[8 * q + 2]; x.s3 = (f16)pv[8 * q + 3];
                    x.s4 = (f16)pv[8 * q + 4]; x.s5 = (f16)pv[8 * q + 5]; x.s6 = (f16)pv[8 * q + 6]; x.s7 = (f16)pv[8 * q + 7];
                    pb[q] = x;
                }
            }
            // O^T += V^T.P^T: k-step q covers keys 32 kh + 16 q + 8 (i/4) + 4 h + i%4
#pragma unroll
            for (int q = 0; q < 2; q++) {
                typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
                u32x4 va[NDB];
#pragma unroll
                for (int db = 0; db < NDB; db++) {
                    const uint32_t off = pofs + db * (kBdpKeys * 64) + q * 1024;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + vbase[0] + off));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + vbase[1] + off));
                    const u32x2 a2 = __builtin_bit_cast(u32x2, lo), b2 = __builtin_bit_cast(u32x2, hi);
                    va[db] = u32x4{a2.x, a2.y, b2.x, b2.y};
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int db = 0; db < NDB; db++) o[db] = mfma32(__builtin_bit_cast(f16x8, va[db]), pb[q], o[db]);
            }
        }
#ifdef FATTN_BDP_MASK_LATE
        // diagnostic build only (A/B): mask s + 2 issued after tile s's compute
        // (config 5: 24.6-25.2 vs 24.7-25.4 us, neutral, profiles/r04_j)
        if constexpr (HM) {
            if (s + 2 < ntiles) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                mask_issue(s + 2);
            }
        }
#endif
        // before the next barrier: mask s + 1 and this wave's pieces of raw s + 2
        // landed.  Issue order per tile: raw s + nRaw, then mask s + 2, so raw
        // s + 2 (issued with tile s + 2 - nRaw <= s - 1, or in the prologue) is
        // older than mask s + 1 (tile s - 1) for s >= 1; tile 0's mask 1 went
        // before the prologue's raw tiles.  Without a mask only the raw counts.
        if constexpr (HM) {
            if (s == 0) {
                if (ntiles > 1)
                    bdp_compute_wait<KT, D, NM>(max(npro - 3, 0) + (C::nRaw < ntiles ? 1 : 0), 2 < ntiles ? 1 : 0);
            } else if (s + 1 < ntiles) {
                bdp_compute_wait<KT, D, NM>(s + C::nRaw < ntiles ? 1 : 0, s + 2 < ntiles ? 1 : 0);
            }
        } else {
            if (s + 2 < ntiles) bdp_compute_wait<KT, D, NM>(min(C::nRaw - 2, ntiles - 3 - s), 0);
        }
#ifdef FATTN_STAMPS
        if (s < 4) {
            float z = 0.0f;
            for (int db = 0; db < NDB; db++) z += o[db][0];
            asm volatile("" ::"v"(z));  // the MFMA results are in before the stamp
            FATTN_STAMP(7 + s);
        }
#endif
    }
    FATTN_STAMP(11);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    bd_finish<D, 2>(a, smem, o, m_run, l2, kh, p, h, compute, tid, lane, wave, qt, ik2, iq3, y, chunk);
}

}  // namespace fattn
