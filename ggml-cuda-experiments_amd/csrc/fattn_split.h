// fattn_split.h -- split-KV ("flash decoding") attention kernel for gfx950.
//
// Replaces flash_attn_row / flash_attn_row_fast (src/flash_row_float.h:4-413)
// and, for small query counts, flash_attn_ext_f16 (src/flash-llama.h:5-438).
// Same math: s = scale*q.k + mask, online softmax (max, sum) per KV chunk,
// unnormalised P.V, merged with the log-sum-exp rule of fa_reduce
// (src/flash_row_float.h:429-471) -- but built MI355X-first:
//
//  * Work unit: one workgroup = 4, 8 or 16 waves = (KV chunk, 16 packed query rows).
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
//  * The waves' states merge through LDS (or, for one-row tiles, per wave);
//    with several chunks the partials (O, m, l) go to the caller's workspace
//    and merge in the last-arriving workgroup or wave (one-row tiles) or in a
//    second launch, fattn_merge_kernel (multi-row tiles).
#pragma once

#include "fattn_common.h"

namespace fattn {

constexpr int kSplitWaves = 4;
constexpr int kStep = 32;   // KV positions per wave step (= one PV k-step)
constexpr int kRows = 16;   // packed query rows per workgroup (MFMA N)
constexpr int VT_F16T = 100;  // V f16 stored transposed ([D][N], flash_row_float.h:177)
constexpr int kCntStride = 64;
// deferred max (cdna_hip_programming.md T13): the exponentials' reference max
// moves only when a score exceeds it by more than 2^3 in p, so p <= 8 (and P*d
// of a V block stays far inside f16 range)
constexpr float kRescaleLog2 = 3.0f;
constexpr float kRescaleNat = kRescaleLog2 * 0.6931471805599453f;
#ifdef FATTN_DMA_NO_NT
constexpr bool kDecodeNT = false;  // diagnostic build only
#else
constexpr bool kDecodeNT = true;   // decode K/V: read once per launch
#endif  // uint32 words between arrival counters (256 B: atomics to one line serialise)

struct SplitArgs {
    const uint8_t* q;
    const uint8_t* k;
    const uint8_t* v;
    const uint8_t* mask;
    float* dst;
    uint32_t* ws_cnt;   // [S][Y] chunk arrival words (64-bit), one per 256-B line (arrival_begin/arrive_last)
    float* ws_o;        // [S][Y][C][16][D] chunk partials
    float* ws_ml;       // [S][Y][C][16][2]
    int64_t q_nb1, q_nb2, q_nb3;
    int64_t k_nb1, k_nb2, k_nb3;
    int64_t v_nb0, v_nb1, v_nb2, v_nb3;
    int64_t m_nb1;
    uint32_t k_span, v_span, m_span, q_span;  // bytes addressed per (kv head, seq) / mask / seq of Q
    int NQ, H, S;       // q ne1, ne2, ne3
    int N;              // kv length
    int rk2, rk3;       // H/Hkv, S/Skv
    int R;              // q-heads packed per tile
    int QPT;            // query rows per tile
    int n_hsub, n_qt;   // head subgroups, query-row tiles
    float R_inv;        // 1/R: m / R == int((m + 0.5) * R_inv) exactly for m, R <= 16
    int chunk_len;      // positions per workgroup (multiple of kStep*kSplitWaves)
    int n_chunks;
    int ncp;            // next power of two >= n_chunks (combine kernel)
    float scale_log2;   // scale * log2(e)
    float scale;        // the softmax scale (split_step works in natural units)
    int has_mask;
    int nbuf;           // steps in flight per wave (1..4); LDS per wave = wave_bytes
    int wave_bytes;
    int pf_stagger;     // prefill kernel: SIMD partner waves run their phases staggered
    const uint8_t* pf_flags;  // prefill: [n_qt][N/64] live-block flags (pf_mask_flags_kernel), or null
    int split_prio;     // split kernel wave priorities: 0 staggered 3/2/1/0, 1 none, 2 staggered while issuing
    int wave_merge;     // split kernel epilogue: 0 = LDS merge of the waves + combine_tile;
                        // 1 = one-row tiles: every wave publishes its own partial and the
                        // last-arriving WAVE merges them (no LDS merge, no barriers);
                        // 2 = one-row tiles: LDS merge, then one partial per workgroup
                        // (wg_row_merge)
    uint64_t arrival_stamp;  // kArrivalTag | launch epoch << kArrivalEpochShift (arrival_begin)
    int merge_launch;   // chunk partials of multi-row tiles: 1 = merged by a second launch (fattn_merge_kernel,
                        // fattn_bd_merge_kernel), 2 = inside the launch (tile_arrive_wait: grid co-resident)
    int step_skip;      // split kernel: 1 = skip steps whose mask is all -inf for the tile (FATTN_OPT_SPLIT_SKIP)
    int xcd_group;      // workgroups in XCD-grouped order (tile_coords; grid size % 8 == 0): batched decode, split kernel
    int part_f16;       // merge_launch 1: each chunk partial stored as O / l in f16 beside its (m, l) in f32
                        // (half the partial bytes; store_part_f16, merge_row_parts_h)
};

// XOR mask of the 16-B chunk swizzle of an LDS row of `cpr` chunks: the largest
// power of two dividing cpr, minus one, so that chunk ^ (x & mask) stays a
// bijection on [0, cpr) (cpr = 16 / 8 for D = 128 / 64 f16 rows; 12 and 10 for
// the D = 96 / 80 rows, whose swizzle works within groups of 4 / 2 chunks)
__host__ __device__ constexpr int swz_mask(int cpr) { return (cpr & -cpr) - 1; }

// epilogue outputs per thread (16 threads per row): D / 16 where that is a
// multiple of 4 (D = 64, 128, 256), else 8 with D / 8 threads of the 16 active
template <int D>
constexpr int epi_ept() { return (D / 16) % 4 == 0 ? D / 16 : 8; }

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
    static constexpr int vscBytes = 0;
    static constexpr int kMergeStride = D + 4;  // floats; +16 B per row spreads rows over banks
    static constexpr int mergeBytes = kRows * kMergeStride * 4 + kRows * 2 * 4;
    // bytes of LDS one wave needs with nbuf steps in flight
    static constexpr int wave_bytes(int nbuf) {
        const int w = (nbuf * stepBytes + vscBytes + 15) / 16 * 16;
        return w > mergeBytes ? w : mergeBytes;
    }
    static constexpr int lds_bytes(int nbuf) { return kSplitWaves * wave_bytes(nbuf); }
};

template <int N>
__device__ __forceinline__ void wait_vmcnt_c() {
    static_assert(N >= 0, "");
    constexpr int n = N > 63 ? 63 : N;  // vmcnt is 6 bits; waiting for fewer is still correct
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory");
}

// wait until at most `outstanding` whole steps (NI instructions each) remain
template <int NI>
__device__ __forceinline__ void wait_steps(int outstanding) {
    switch (__builtin_amdgcn_readfirstlane(outstanding)) {
        case 0: wait_vmcnt_c<0>(); break;
        case 1: wait_vmcnt_c<NI>(); break;
        case 2: wait_vmcnt_c<2 * NI>(); break;
        default: wait_vmcnt_c<3 * NI>(); break;
    }
}

// wait until at most `outstanding` whole steps plus EXTRA instructions remain
// (EXTRA = the V part of the oldest pending step: its K and mask have landed)
template <int NI, int EXTRA>
__device__ __forceinline__ void wait_steps_plus(int outstanding) {
    switch (__builtin_amdgcn_readfirstlane(outstanding)) {
        case 0: wait_vmcnt_c<EXTRA>(); break;
        case 1: wait_vmcnt_c<NI + EXTRA>(); break;
        case 2: wait_vmcnt_c<2 * NI + EXTRA>(); break;
        default: wait_vmcnt_c<3 * NI + EXTRA>(); break;
    }
}

// ---------------------------------------------------------------- HBM -> LDS
template <int KT, int VT, int D, int GRAN>
struct StepPlan {
    using C = SplitCfg<KT, VT, D>;
    static constexpr int PK = C::kBytes / GRAN;
    static constexpr int PV = C::vBytes / GRAN;
    // K and V come through different buffer descriptors: separate instructions
    static constexpr int NIK = (PK + kWave - 1) / kWave;
    static constexpr int NIV = (PV + kWave - 1) / kWave;
    static constexpr int NIKV = NIK + NIV;
    // mask granule: LDS-DMA writes lane*4 bytes for sub-dword sizes, so the
    // generic path moves dwords (2 positions) and needs even-padded mask rows
    static constexpr int MG = GRAN == 16 ? 16 : 4;
    static constexpr int MPR = kStep * 2 / MG;           // mask pieces per row
    // all 16 mask rows are always requested so every step issues the same,
    // compile-time instruction count; rows past n_q fall outside the mask
    // descriptor and cost no memory traffic
    static constexpr int PM = kRows * MPR;
    static constexpr int NIM = PM / kWave;
    static_assert(PM % kWave == 0, "");
};

typedef __attribute__((address_space(3))) void lds_void;
typedef int i32x4 __attribute__((ext_vector_type(4)));

// Buffer descriptor (4 SGPRs): base, stride 0, num_records = bytes, raw dword
// format.  Offsets at or past `bytes` fetch nothing and write ZEROS to LDS
// (tests/test_gpu_prims.py::test_lds_dma_partial_exec).
__device__ __forceinline__ i32x4 make_srd(const void* base, uint32_t bytes) {
    const uint64_t p = (uint64_t)base;
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32));
    r.z = __builtin_amdgcn_readfirstlane((int)bytes);
    r.w = 0x00020000;
    return r;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(const lds_void*)p; }

// Buffer resource for compiler-tracked buffer loads (the hand-off reads of the
// chunk merges): built from readfirstlane'd inputs, so it is provably
// wave-uniform and no waterfall loop wraps the loads (cdna_hip_programming.md
// T20).  Offsets at or past num_records return zeros without memory traffic.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t p = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, (int)n, 0x00020000);
}
constexpr int kAuxSc1 = 16;  // buffer-load cache policy: sc1 (L1 bypass; MI355X_MICROARCH.md sc1 table)

// L1-bypassing (sc1) 16-B / 4-B loads of handed-off partials.  Compiler-tracked
// builtins: hipcc inserts the waits and never reads a register before its data
// landed (round 3's asm forms had three such miscompiles).
__device__ __forceinline__ u32x4 ld_sc1_buf(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxSc1));
}
__device__ __forceinline__ uint32_t ld_sc1_buf_b32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kAuxSc1);
}

// 16-B load into registers through a buffer descriptor, as asm: UNTRACKED --
// hipcc inserts no wait for it, so waiting for it leaves the LDS-DMA issued
// after it in flight (a tracked load would make hipcc drain every DMA with
// vmcnt(0) at its first use, cdna_hip_programming.md §5 trap (b)).  The caller
// retires it with a counted wait and then passes every result through
// reg_fence<TAG>() before any use.  The asm comments "UNTRACKED(tag)" on the
// load and "RETIRED(tag)" on the fence let tools/isa_hazard_check.py prove on
// the ISA that no instruction touches the destination registers between the
// load and its fence on any path (tests/test_isa_hazards.py).
enum : int { kTagQ = 1, kTagMaskWords = 2 };  // bit masks
template <int TAG>
__device__ __forceinline__ u32x4 ld_buf_untracked(const i32x4& srd, uint32_t off) {
    u32x4 v;
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen ; UNTRACKED(%3)"
                 : "=v"(v)
                 : "v"(off), "s"(srd), "i"(TAG)
                 : "memory");
    return v;
}

// HBM -> LDS, one piece per lane at lds + lane*BYTES.  Inline asm: through the
// builtin, hipcc treats the LDS base as a per-lane value, and around an
// exec-masked (partial) instruction it built per-lane phis of (LDS base,
// offset) pairs whose readfirstlane'd M0 no longer matched the inactive
// lanes' offsets -- and it tracks the DMA in its s_waitcnt bookkeeping, so
// the first LDS read after it would wait for every DMA in flight.  Here the
// LDS address is an M0 operand ("{m0}": hipcc writes M0 itself, straight
// from the address arithmetic -- one s_add per DMA where the asm's own
// save / set / restore of the reserved M0 cost three s_mov; the prefill
// body issues 8 DMAs a tile with one wave per SIMD, where every scalar
// instruction takes an issue slot).  s_nop 4 opens the string: hipcc pads
// its own VMEM instructions but not an asm one, and it re-materialises the
// descriptor's words with v_readfirstlane right before the statement -- a
// VALU SGPR write needs 5 wait states before a VMEM instruction reads it
// (cdna_hip_programming.md 'Insert its wait states'; with s_nop 0 multi-chunk
// decodes read through a stale descriptor word; tools/isa_hazard_check.py
// audits every asm VMEM instruction for it).  It also covers M0 -> LDS-DMA
// (1 state).  Not tracked by the compiler's s_waitcnt bookkeeping: every
// consumer waits with an explicit vmcnt.  (-DFATTN_DMA_M0_SAVE: the round-5
// save / restore form, padded the same way, for A/B builds.)
// NT: non-temporal policy for bytes one CU reads once (the decode KV stream,
// MI355X_MICROARCH.md 'nt-weights'); never for tiles other workgroups re-read.
// PAD: the opening s_nop's count -- 4 (5 wait states) unless the caller's
// descriptor is provably not freshly VALU-written (pf4's loop: its descriptors
// are loop-invariant SGPRs; tools/isa_hazard_check.py checks every call site
// on the shipped ISA, so a PAD that is too small fails the CPU test suite)
template <int BYTES, bool NT = false, int PAD = 4>
__device__ __forceinline__ void dma(const i32x4& srd, uint32_t lds_any, uint32_t off) {
    static_assert(BYTES == 16 || BYTES == 4, "");
    static_assert(PAD >= 0 && PAD <= 4, "");
    // wave-uniform by construction; readfirstlane keeps it an SGPR operand even
    // where divergent code around the call hides that from the compiler
    const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_any);
#ifdef FATTN_DMA_M0_SAVE
    uint32_t keep;
#define FATTN_DMA_ASM(INSN, MOD)                                                                         \
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 2\n\t" INSN " %1, %2, 0 offen" MOD \
                 "\n\ts_mov_b32 m0, %0"                                                                \
                 : "=&s"(keep)                                                                           \
                 : "v"(off), "s"(srd), "s"(lds)                                                          \
                 : "memory")
#else
#define FATTN_DMA_ASM(INSN, MOD)                                                                     \
    asm volatile("s_nop %3\n\t" INSN " %0, %1, 0 offen" MOD : : "v"(off), "s"(srd), "{m0}"(lds), "n"(PAD) \
                 : "memory")
#endif
    if constexpr (BYTES == 16 && NT) FATTN_DMA_ASM("buffer_load_dwordx4", " nt lds");
    else if constexpr (BYTES == 16) FATTN_DMA_ASM("buffer_load_dwordx4", " lds");
    else if constexpr (NT) FATTN_DMA_ASM("buffer_load_dword", " nt lds");
    else FATTN_DMA_ASM("buffer_load_dword", " lds");
#undef FATTN_DMA_ASM
}

struct StepSrc {
    i32x4 k, v, m;
};

// ---------------------------------------------------------------- arrivals
// The chunks of a tile meet through one 64-bit arrival word per tile,
// [0xFF | launch epoch : 32 | generation : 8 | arrivals : 16].  Each arriving
// lane first stamps the word with its launch's tag and epoch (atomic max, no
// return; the split kernel issues it right after its prologue's DMA, off every
// critical path): a word left by an earlier launch (re-armed or, after an
// aborted launch, mid-count) or never zeroed (top 8 bits not all ones) is
// superseded and the count restarts at 0.  The last arriver re-arms the word
// (count 0, same epoch, generation + 1), so a replayed graph finds it clean;
// workgroups that wait for a tile's arrivals (bd_tile_merge) watch for the
// count to complete or the generation to move.
// Launches sharing one workspace must be stream-ordered.
constexpr uint64_t kArrivalTag = 0xFFull << 56;
constexpr int kArrivalEpochShift = 24;

__device__ __forceinline__ uint64_t* arrival_word(const SplitArgs& a, int64_t tile) {
    return (uint64_t*)(a.ws_cnt + tile * kCntStride);
}

// by the lane that later calls arrive_last, before it (same-lane order)
__device__ __forceinline__ void arrival_begin(const SplitArgs& a, int64_t tile) {
    (void)__hip_atomic_fetch_max(arrival_word(a, tile), a.arrival_stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one lane: count this arrival; true for the tile's n-th (last) arriver,
// which re-arms the word
__device__ __forceinline__ bool arrive_last(const SplitArgs& a, int64_t tile, int n) {
    uint64_t* w = arrival_word(a, tile);
    const uint64_t old = __hip_atomic_fetch_add(w, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = (old & 0xFFFF) == (uint64_t)(n - 1);
    if (last) {
        const uint64_t gen = ((old >> 16) + 1) & 0xFF;
        __hip_atomic_store(w, (old & ~0xFFFFFFull) | gen << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return last;
}

// In-kernel chunk merge (SplitArgs::merge_launch == 2, every workgroup of the
// grid co-resident): one lane per workgroup, after every storing wave stored
// its partials sc1 and drained and the workgroup met at a barrier, counts the
// workgroup on the tile's arrival word (stamped in the prologue).  The last
// arriver re-arms the word (count 0, generation + 1) and returns at once; the
// others poll it (sc1 loads, relaxed) until the count is complete or the
// generation has moved.  Then every workgroup of the tile may load the tile's
// partials with sc1 loads, the other waves behind a barrier
// (MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1
// table).  Returns 0 only when the bounded poll gave up (a fault: the caller
// writes NaN rows instead of merging).
__device__ __forceinline__ int tile_arrive_wait(const SplitArgs& a, int64_t tile, int n) {
    uint64_t* w = arrival_word(a, tile);
    const uint64_t old = __hip_atomic_fetch_add(w, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t gen = (uint32_t)(old >> 16) & 0xFFu;
    if ((int)(old & 0xFFFF) == n - 1) {
        __hip_atomic_store(w, (old & ~0xFFFFFFull) | (uint64_t)((gen + 1) & 0xFFu) << 16, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        return 1;
    }
    for (uint32_t spins = 0; spins < (1u << 20); spins++) {
        const uint32_t lo = ld_sc1_u32((const uint32_t*)w);
        if (((lo >> 16) & 0xFFu) != gen || (int)(lo & 0xFFFF) >= n) return 1;
        __builtin_amdgcn_s_sleep(2);
    }
    return 0;
}

// One step = [K rows | V rows | mask rows] for positions [n0, n0+32), copied
// as raw bytes.  GRAN = 16: 16-B pieces (quantised rows contiguous, f16 rows
// 16-B aligned); GRAN = 4: dword pieces for any ggml row stride.
template <int KT, int VT, int D, int GRAN, bool HM>
__device__ __forceinline__ void issue_step(const SplitArgs& a, const StepSrc& rs, int n0, int mrow0, uint8_t* buf,
                                           int lane, bool kv_live = true) {
#ifdef FATTN_DIAG_NOMEM
    return;  // diagnostic build only: compute on whatever LDS holds (compute latency)
#endif
    using C = SplitCfg<KT, VT, D>;
    using P = StepPlan<KT, VT, D, GRAN>;
    const uint32_t kn1 = (uint32_t)a.k_nb1, vn1 = (uint32_t)a.v_nb1;
    // a step that is -inf for the whole tile: K and V through empty
    // descriptors (every load out of range: zeros, no traffic)
    i32x4 ksrd = rs.k, vsrd = rs.v;
    ksrd.z = __builtin_amdgcn_readfirstlane(kv_live ? rs.k.z : 0);
    vsrd.z = __builtin_amdgcn_readfirstlane(kv_live ? rs.v.z : 0);
#pragma unroll
    for (int i = 0; i < P::NIK; i++) {
        const int p = i * kWave + lane;
        const int byte = p * GRAN;
        uint32_t off;
        if constexpr (KT == FATTN_TYPE_F16) {
            // f16 rows: 16-B chunks XOR-swizzled by row (conflict-free ds_read_b128)
            constexpr int SW = swz_mask(C::rowK / 16);
            const int row = byte / C::rowK;
            const int chunk = ((byte % C::rowK) / 16) ^ (row & SW);
            off = (uint32_t)(n0 + row) * kn1 + chunk * 16 + (byte & 15);
        } else if constexpr (GRAN == 16) {
            off = (uint32_t)n0 * C::rowK + byte;
        } else {
            const int row = byte / C::rowK;
            off = (uint32_t)(n0 + row) * kn1 + (byte % C::rowK);
        }
        if (P::PK % kWave == 0 || p < P::PK) dma<GRAN, kDecodeNT>(ksrd, lds_addr(buf + i * kWave * GRAN), off);
    }
    // K, then the mask, then V: a step's S^T and softmax start once K and the
    // mask have landed, while V is still in flight
    if constexpr (HM) {
        uint8_t* mbuf = buf + C::kBytes + C::vBytes;
#pragma unroll
        for (int i = 0; i < P::NIM; i++) {
            const int q = i * kWave + lane;
            const int mr = q / P::MPR;
            const int off = (q % P::MPR) * P::MG;
            const uint32_t moff = (uint32_t)(mrow0 + mr) * (uint32_t)a.m_nb1 + (uint32_t)n0 * 2 + off;
            // 16-B path (one instruction, rows 0..15): lanes of rows past the
            // tile's query rows stay idle -- row 0's lanes always issue it, so
            // the per-step instruction count (vmcnt budget) is unchanged
            if (GRAN != 16 || mr < a.QPT) dma<P::MG>(rs.m, lds_addr(mbuf + i * kWave * P::MG), moff);
        }
    }
    uint8_t* vbuf = buf + C::kBytes;
#pragma unroll
    for (int i = 0; i < P::NIV; i++) {
        const int p = i * kWave + lane;
        const int byte = p * GRAN;
        uint32_t off;
        if constexpr (VT == VT_F16T) {
            // V^T tile: D rows (one per head dim) of kStep f16; needs N % 32 == 0
            const int d = byte / (kStep * 2);
            off = (uint32_t)d * (uint32_t)a.v_nb0 + (uint32_t)n0 * 2 + (byte % (kStep * 2));
        } else if constexpr (VT == FATTN_TYPE_F16) {
            constexpr int SW = swz_mask(C::rowV / 16);
            const int row = byte / C::rowV;
            const int chunk = ((byte % C::rowV) / 16) ^ (((row & 7) << 1) & SW);
            off = (uint32_t)(n0 + row) * vn1 + chunk * 16 + (byte & 15);
        } else if constexpr (GRAN == 16) {
            off = (uint32_t)n0 * C::rowV + byte;
        } else {
            const int row = byte / C::rowV;
            off = (uint32_t)(n0 + row) * vn1 + (byte % C::rowV);
        }
        if (P::PV % kWave == 0 || p < P::PV) dma<GRAN, kDecodeNT>(vsrd, lds_addr(vbuf + i * kWave * GRAN), off);
    }
}

// ---------------------------------------------------------------- block scales
// The f16 scale of block b of a raw ggml row sits at byte BB*b.  row_scales()
// fetches the dwords holding all of a row's scales (2 x ds_read2_b32 for 4
// blocks); scale_bits() extracts block b's 16 bits.
template <int T, int D>
struct RowScales {
    uint32_t w[D / QK];
};
// whether block b's scale sits in the high half of its dword (rows that are a
// whole number of dwords); rows that are not (D = 96) read each scale as a u16
template <int T, int D>
__host__ __device__ constexpr bool scale_hi(int b) {
    return row_bytes<T, D>() % 4 == 0 && ((TypeInfo<T>::block_bytes * b) & 2) != 0;
}
template <int T, int D>
__device__ __forceinline__ RowScales<T, D> row_scales(const uint8_t* row) {
    constexpr int BB = TypeInfo<T>::block_bytes;
    RowScales<T, D> s;
#pragma unroll
    for (int b = 0; b < D / QK; b++) {
        if constexpr (row_bytes<T, D>() % 4 != 0) s.w[b] = *(const uint16_t*)(row + BB * b);
        else s.w[b] = *(const uint32_t*)(row + ((BB * b) & ~3));
    }
    return s;
}
template <int T, int D>
__device__ __forceinline__ uint32_t scale_bits(const RowScales<T, D>& s, int b) {
    return scale_hi<T, D>(b) ? (s.w[b] >> 16) : (s.w[b] & 0xffffu);
}
// block b's f16 scale in both halves, by one v_perm (b is unrolled)
template <int T, int D>
__device__ __forceinline__ uint32_t scale_bcast(const RowScales<T, D>& s, int b) {
    return perm_b32(s.w[b], s.w[b], scale_hi<T, D>(b) ? 0x03020302u : 0x01000100u);
}
// f16 pair {scale of row r0, scale of row r1} for block b
template <int T, int D>
__device__ __forceinline__ f16x2 scale_pair(const RowScales<T, D>& s0, const RowScales<T, D>& s1, int b) {
    constexpr int BB = TypeInfo<T>::block_bytes;
    // v_perm: low half from s0.w[b], high half from s1.w[b]
    return as_h2(((BB * b) & 2) ? perm_b32(s1.w[b], s0.w[b], 0x07060302u) : perm_b32(s1.w[b], s0.w[b], 0x05040100u));
}

// 8 bytes at a 2-byte-aligned LDS offset whose alignment is known only at run
// time (Q8_0 / Q4_0 rows of D = 96: 102 / 54 B, so odd rows start 2 B off a
// dword): three dword reads and two v_alignbyte with the shift in a VGPR
__device__ __forceinline__ u32x2 read8_any(const uint8_t* smem, uint32_t off) {
    const uint32_t base = off & ~3u, sh = off & 3u;
    const uint32_t w0 = *(const uint32_t*)(smem + base);
    const uint32_t w1 = *(const uint32_t*)(smem + base + 4);
    const uint32_t w2 = *(const uint32_t*)(smem + base + 8);
    u32x2 r;
    r.x = alignbyte(w1, w0, sh);
    r.y = alignbyte(w2, w1, sh);
    return r;
}

// ---------------------------------------------------------------- operands
// K operand (A of S^T = K.Q^T) for tile t (16 rows), block/k-step b:
// lane l -> row 16t + (l&15), elements d = 32b + 8(l>>4) + j.
template <int KT, int D>
__device__ __forceinline__ f16x8 k_operand(const uint8_t* kb, int row, int g, int b, uint32_t dbits) {
    if constexpr (KT == FATTN_TYPE_F16) {
        constexpr int CPR = D * 2 / 16;
        const int chunk = (4 * b + g) ^ (row & swz_mask(CPR));
        const f16x8 r = *(const f16x8*)(kb + row * (D * 2) + chunk * 16);
        if constexpr (D % QK != 0) {  // D = 80: the last k-step's dims past D read as zero
            if (b == D / QK && 4 * b + g >= CPR) return f16x8{};
        }
        return r;
    } else if constexpr (KT == FATTN_TYPE_Q8_0) {
        constexpr int RB = row_bytes<KT, D>();
        const uint32_t base = row * RB + kQ8Bytes * b;
        u32x2 raw;
        if constexpr (RB % 4 != 0) {
            raw = read8_any(kb, base + 2 + 8 * g);
        } else switch ((kQ8Bytes * b + 2) & 7) {  // b is a compile-time constant after unrolling
            case 0: raw = read8_at<0>(kb, base + 2 + 8 * g); break;
            case 2: raw = read8_at<2>(kb, base + 2 + 8 * g); break;
            case 4: raw = read8_at<4>(kb, base + 2 + 8 * g); break;
            default: raw = read8_at<6>(kb, base + 2 + 8 * g); break;
        }
        const f16x2 d = as_h2(dbits);
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
        if constexpr (RB % 4 != 0) {
            raw = read8_any(kb, base + 2 + 8 * (g & 1));
        } else switch ((kQ4Bytes * b + 2) & 7) {
            case 0: raw = read8_at<0>(kb, base + 2 + 8 * (g & 1)); break;
            case 2: raw = read8_at<2>(kb, base + 2 + 8 * (g & 1)); break;
            case 4: raw = read8_at<4>(kb, base + 2 + 8 * (g & 1)); break;
            default: raw = read8_at<6>(kb, base + 2 + 8 * (g & 1)); break;
        }
        const uint32_t sh = (g >> 1) * 4;
        const f16x2 d = as_h2(dbits);
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
        const int a0 = r0 * RB + ((chunk ^ (((r0 & 7) << 1) & swz_mask(CPR))) * 16) + (p & 1) * 8;
        const int a1 = r1 * RB + ((chunk ^ (((r1 & 7) << 1) & swz_mask(CPR))) * 16) + (p & 1) * 8;
        typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + a0));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + a1));
        u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
        u32x4 r = {l2.x, l2.y, h2.x, h2.y};
        return __builtin_bit_cast(f16x8, r);
    }
}

// ---------------------------------------------------------------- tile geometry
// A tile packs rows m = (query row m / R, head m % R).  No runtime integer
// division (hipcc expands those into long scalar loops).
__device__ __forceinline__ int div_R(const SplitArgs& a, int m) { return (int)(((float)m + 0.5f) * a.R_inv); }

// number of valid rows of tile (qt, hs); they form a prefix [0, rv)
__device__ __forceinline__ int tile_rows(const SplitArgs& a, int qt, int hs) {
    const int rows_q = min(a.QPT, a.NQ - qt * a.QPT);
    const int heads = min(a.R, a.rk2 - hs * a.R);
    return rows_q * heads;  // heads < R only when R == 16 (then QPT == 1)
}

// ---------------------------------------------------------------- diagnostics
// Diagnostic build only (-DFATTN_STAMPS, libfattn_stamps.so, tools/stamps.py):
// lane 0 of every wave records s_memrealtime (100 MHz) at phase boundaries into
// g_stamps[block][16 wave slots][16]: 0 start, 1 first steps issued, 2+s data of
// step s in LDS (s < 8), 10 loop done, 11 waves merged (LDS), 12 partial
// published and drained, 14 arrival atomic returned, 15 merger's loads in,
// 13 tile merged and stored (merging wave).  No stamp executes in the product
// library.
#ifdef FATTN_STAMPS
static __device__ unsigned long long* g_stamps;  // one per translation unit (fattn_launch_d*.hip)
#define FATTN_STAMP(k)                                                                          \
    do {                                                                                        \
        if (lane == 0 && g_stamps) {                                                            \
            const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                     \
            const int64_t blk_ = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x; \
            g_stamps[(blk_ * 16 + wave) * 16 + (k)] = t_;                                \
        }                                                                                       \
    } while (0)
// any lane: slot k of wave 0's record = max(slot, v)
#define FATTN_STAMP_MAX(k, v)                                                                   \
    do {                                                                                        \
        if (g_stamps) {                                                                         \
            const int64_t blk_ = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x; \
            atomicMax(&g_stamps[blk_ * 16 * 16 + (k)], (unsigned long long)(v));      \
        }                                                                                       \
    } while (0)
// The split kernel keeps its stamps in LDS (a static array) and each wave
// stores its own at the kernel's end (FATTN_SSTAMP_FLUSH): a global store per
// stamp would be counted by vmcnt and every counted wait would wait for it
// too, stretching the very timeline it measures (round 3's stamps: a 17 us
// span for an 11 us launch).
__device__ __forceinline__ unsigned long long* split_stamp_slots() {
    __shared__ unsigned long long s[16 * 16];
    return s;
}
#define FATTN_SSTAMP(k)                                                                          \
    do {                                                                                         \
        if (lane == 0) split_stamp_slots()[wave * 16 + (k)] = __builtin_amdgcn_s_memrealtime();  \
    } while (0)
#define FATTN_SSTAMP_INIT()                                                                      \
    do {                                                                                         \
        if (lane < 16) split_stamp_slots()[wave * 16 + lane] = 0ull;                             \
    } while (0)
#define FATTN_SSTAMP_FLUSH()                                                                     \
    do {                                                                                         \
        if (lane < 16 && g_stamps) {                                                             \
            const int64_t blk_ = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x; \
            g_stamps[(blk_ * 16 + wave) * 16 + lane] = split_stamp_slots()[wave * 16 + lane];    \
        }                                                                                        \
    } while (0)
#else
#define FATTN_STAMP(k) do { } while (0)
#define FATTN_STAMP_MAX(k, v) do { } while (0)
#define FATTN_SSTAMP(k) do { } while (0)
#define FATTN_SSTAMP_INIT() do { } while (0)
#define FATTN_SSTAMP_FLUSH() do { } while (0)
#endif

// ---------------------------------------------------------------- kernel

// workgroup -> (KV chunk, tile y, sequence iq3).  Blocks are dealt round-robin
// over the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch: observed placement,
// used for speed only), so in the plain order the chunks of one kv head sit on
// 8 different L2s (batched decode: each fetches the head's Q rows, 32 KB f32,
// from HBM; split kernel: the tile's chunk partials cross XCDs).  The
// XCD-grouped order (a.xcd_group) gives each XCD whole tiles -- all their
// chunks.  Any bijection is correct; the planner sets xcd_group only for
// grids of a multiple of 8 workgroups.
__device__ __forceinline__ void tile_coords(const SplitArgs& a, int& chunk, int& y, int& iq3) {
    chunk = blockIdx.x;
    y = blockIdx.y;
    iq3 = blockIdx.z;
    if (a.xcd_group) {
        const uint32_t gx = gridDim.x, gy = gridDim.y;
        const uint32_t G = gx * gy * gridDim.z;
        const uint32_t L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
        const uint32_t L2 = (L % 8) * (G / 8) + L / 8;
        chunk = (int)(L2 % gx);
        y = (int)((L2 / gx) % gy);
        iq3 = (int)(L2 / (gx * gy));
    }
}


template <int D, int CB = 2>
__device__ __forceinline__ void combine_tile(const SplitArgs& a, int64_t tile, int qt, int hs, int ik2, int iq3,
                                             int rv, int row_base, uint8_t* smem);

// One-row tiles (decode with n_q * H / Hkv == 1 per tile), up to 32 parts per
// tile: each WAVE is a part.  It stores its (O, m, l) write-through (sc1),
// drains, and counts itself on the tile's arrival word; the wave that counts
// last merges all parts alone -- lane i owns dims 2i, 2i+1, every part's
// values come in one round trip, weights by wave reductions -- and writes dst.
// No LDS merge and no workgroup barrier: waves leave as they finish.  Same
// fa_reduce math as combine_tile (src/flash_row_float.h:415-472), fixed order.
constexpr int kWaveMergeParts = 64;  // parts per tile (one (m, l) pair per lane)
constexpr int kWaveMergeBatch = 32;  // parts loaded per round trip
template <int D, bool VQ8, int NW = kSplitWaves>
__device__ __forceinline__ void wave_merge_epilogue(const SplitArgs& a, const f32x4 (&o)[D / 16], float m_run,
                                                    float l_tot, int chunk, int wave, int lane, int qt, int hs,
                                                    int ik2, int iq3, int y) {
    static_assert(D == 128, "lane i <-> dims 2i, 2i+1");
    constexpr int NB = D / QK;
    constexpr int NC = D / 16;
    constexpr float kNegInf = -__builtin_inff();
    const int g = lane >> 4, m = lane & 15;
    const int NP = a.n_chunks * NW;
    const int64_t tile = (int64_t)iq3 * gridDim.y + y;
    const int part = chunk * NW + wave;
    float* po = a.ws_o + (tile * NP + part) * D;  // row 0 of the part: [NP][D] per tile
    auto bits = [](float x) { return __builtin_bit_cast(uint32_t, x); };
    if (m == 0) {  // column 0 = the tile's row; its dims sit on lanes 0, 16, 32, 48
        if constexpr (VQ8) {
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const f32x4 e = o[2 * b], od = o[2 * b + 1];
                st_sc1(po + 32 * b + 8 * g, u32x4{bits(e.x), bits(od.x), bits(e.y), bits(od.y)});
                st_sc1(po + 32 * b + 8 * g + 4, u32x4{bits(e.z), bits(od.z), bits(e.w), bits(od.w)});
            }
        } else {
#pragma unroll
            for (int c = 0; c < NC; c++)
                st_sc1(po + 16 * c + 4 * g, u32x4{bits(o[c].x), bits(o[c].y), bits(o[c].z), bits(o[c].w)});
        }
        if (g == 0) st_sc1_x2(a.ws_ml + 2 * (tile * NP + part), u32x2{bits(m_run), bits(l_tot)});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FATTN_SSTAMP(12);
    int last = 0;
    if (lane == 0) last = arrive_last(a, tile, NP);
    last = __builtin_amdgcn_readfirstlane(last);
    FATTN_SSTAMP(14);
    if (!last) return;
    // ---- merge: lane half h = lane / 32 takes the parts of parity h, dims
    // 4 (lane % 32) .. +3, one 16-B load per part (parts past NP fall outside
    // the descriptor: zeros, no traffic, weight 0); the halves meet by one
    // permlane32 swap.  Every load of a batch is issued before one wait.
    const int h = lane >> 5, d4 = 4 * (lane & 31);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the count)
    const __amdgpu_buffer_rsrc_t osrd = make_rsrc(a.ws_o + tile * NP * D, (uint32_t)(NP * D * 4));
    const __amdgpu_buffer_rsrc_t msrd = make_rsrc(a.ws_ml + 2 * tile * NP, (uint32_t)(NP * 8));
    constexpr int kIt = kWaveMergeBatch / 2;  // part pairs per round trip
    u32x4 v[kIt];
    auto issue = [&](int p0) {
#pragma unroll
        for (int i = 0; i < kIt; i++) v[i] = ld_sc1_buf(osrd, (uint32_t)(((p0 + 2 * i + h) * D + d4) * 4));
    };
    issue(0);
    const uint32_t mlm = ld_sc1_buf_b32(msrd, (uint32_t)(lane * 8));      // lane p: m of part p
    const uint32_t mll = ld_sc1_buf_b32(msrd, (uint32_t)(lane * 8 + 4));  //          l of part p
    FATTN_SSTAMP(15);
    const float mp = lane < NP ? __builtin_bit_cast(float, mlm) : kNegInf;
    const float M = seg_reduce<true>(mp, 64);
    const float w = (mp == kNegInf) ? 0.0f : __builtin_amdgcn_exp2f(mp - M);
    const float L = seg_reduce<false>(lane < NP ? w * __builtin_bit_cast(float, mll) : 0.0f, 64);
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int p0 = 0; p0 < NP; p0 += kWaveMergeBatch) {  // wave-uniform
        if (p0 > 0) issue(p0);
#pragma unroll
        for (int i = 0; i < kIt; i++) {
            const int wi = __builtin_bit_cast(int, w);
            const float we = __builtin_bit_cast(float, __builtin_amdgcn_readlane(wi, p0 + 2 * i));
            const float wo = __builtin_bit_cast(float, __builtin_amdgcn_readlane(wi, p0 + 2 * i + 1));
            const float wp = h ? wo : we;
            acc += wp * __builtin_bit_cast(f32x4, v[i]);
        }
    }
    acc.x = xor32_pair(acc.x, false);
    acc.y = xor32_pair(acc.y, false);
    acc.z = xor32_pair(acc.z, false);
    acc.w = xor32_pair(acc.w, false);
    if (h) return;  // lanes 0..31 store the row, 16 B each
    const int rq = div_R(a, 0);
    const int riq1 = qt * a.QPT + rq;
    const int riq2 = ik2 * a.rk2 + hs * a.R;
    float* out = a.dst + (((int64_t)iq3 * a.NQ + riq1) * a.H + riq2) * D + d4;
    const float inv = L == 0.0f ? __builtin_nanf("") : 1.0f / L;  // L == 0 (row fully masked) -> NaN like the reference
    *(f32x4*)out = acc * inv;
    FATTN_SSTAMP(13);
}

// Log-sum-exp merge of NP <= 64 one-row partials of a tile: O rows [NP][D]
// f32 and (m in log2 units, l) pairs [NP][2], written write-through by other
// workgroups of this launch (sc1 loads: first row of the hand-off table,
// MI355X_MICROARCH.md).  One wave: lane (h, dl) = (lane / (D/4), lane % (D/4))
// loads 16 B of every part p = h (mod 64 / (D/4)); every load of a batch is
// issued before one wait; the lane groups meet by permlane swaps.  Fixed
// order (deterministic).  `out` = the tile's dst row.  fa_reduce math,
// src/flash_row_float.h:415-472, in fp32.
template <int D>
constexpr int merge_ppr() { return 64 % (D / 4) == 0 ? 64 / (D / 4) : 1; }  // parts per lane row (4, 2, 1)

template <int D, int kIt = 16, int AUX = kAuxSc1>  // kIt: loads per lane per round trip; AUX: the loads' cache bits
__device__ __forceinline__ void merge_row_parts(const float* parts_o, const float* parts_ml, int NP, float* out,
                                                int lane, int ostride = D, int mstride = 2) {
    constexpr float kNegInf = -__builtin_inff();
    constexpr int LPP = D / 4;              // lanes per part
    constexpr int PPR = merge_ppr<D>();     // D = 80 / 96: 1
    const int h = lane / LPP, d4 = 4 * (lane % LPP);
    // (part p's O row at p * ostride floats, its (m, l) at p * mstride)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the count)
    const __amdgpu_buffer_rsrc_t osrd = make_rsrc(parts_o, (uint32_t)(NP * ostride * 4));
    const __amdgpu_buffer_rsrc_t msrd = make_rsrc(parts_ml, (uint32_t)(NP * mstride * 4));
    u32x4 v[kIt];
    auto issue = [&](int p0) {
#pragma unroll
        for (int i = 0; i < kIt; i++)
            v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 osrd, (uint32_t)(((p0 + PPR * i + h) * ostride + d4) * 4), 0, AUX));
    };
    issue(0);
    const uint32_t mlm = __builtin_amdgcn_raw_buffer_load_b32(msrd, (uint32_t)(lane * mstride * 4), 0, AUX);  // lane p: m of part p
    const uint32_t mll = __builtin_amdgcn_raw_buffer_load_b32(msrd, (uint32_t)(lane * mstride * 4 + 4), 0, AUX);  // l of part p
    const float mp = lane < NP ? __builtin_bit_cast(float, mlm) : kNegInf;
    const float M = seg_reduce<true>(mp, 64);
    const float w = (mp == kNegInf) ? 0.0f : __builtin_amdgcn_exp2f(mp - M);
    const float L = seg_reduce<false>(lane < NP ? w * __builtin_bit_cast(float, mll) : 0.0f, 64);
    const int wi = __builtin_bit_cast(int, w);
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int p0 = 0; p0 < NP; p0 += kIt * PPR) {  // wave-uniform
        if (p0 > 0) issue(p0);
#pragma unroll
        for (int i = 0; i < kIt; i++) {
            float wp = 0.0f;
#pragma unroll
            for (int j = 0; j < PPR; j++) {
                const float wj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(wi, (p0 + PPR * i + j) & 63));
                wp = (h == j) ? wj : wp;
            }
            acc += wp * __builtin_bit_cast(f32x4, v[i]);
        }
    }
    if constexpr (PPR == 4) {
        acc.x = xor16_pair(acc.x, false);
        acc.y = xor16_pair(acc.y, false);
        acc.z = xor16_pair(acc.z, false);
        acc.w = xor16_pair(acc.w, false);
    }
    if constexpr (PPR >= 2) {
        acc.x = xor32_pair(acc.x, false);
        acc.y = xor32_pair(acc.y, false);
        acc.z = xor32_pair(acc.z, false);
        acc.w = xor32_pair(acc.w, false);
    }
    if (h) return;
    const float inv = L == 0.0f ? __builtin_nanf("") : 1.0f / L;  // L == 0 (row fully masked) -> NaN like the reference
    *(f32x4*)(out + d4) = acc * inv;
}

// f16 chunk partials (SplitArgs::part_f16, second-launch merges): the
// partial's EPT dims of O / l rounded to f16 -- bounded by max |v|, where the
// unnormalised O is not -- (a fully masked chunk, l = 0, stores zeros: its
// merge weight is 0); the (m, l) pair stays f32.  Plain stores: the kernel
// boundary orders them before the merge launch's loads.
template <int EPT>
__device__ __forceinline__ void store_part_f16(uint16_t* dst, const float (&acc)[EPT], float L) {
    static_assert(EPT % 4 == 0, "");
    const float inv = L > 0.0f ? 1.0f / L : 0.0f;
    uint32_t w[EPT / 2];
#pragma unroll
    for (int e = 0; e < EPT; e += 2) {
        const f16x2 hp = {(_Float16)(acc[e] * inv), (_Float16)(acc[e + 1] * inv)};
        w[e / 2] = __builtin_bit_cast(uint32_t, hp);
    }
    // (16-B stores when EPT is a multiple of 8 -- dst is then 16-B aligned --,
    // else 8-B ones: the batched-decode epilogue's 12 dims at D = 96)
    if constexpr (EPT % 8 == 0) {
#pragma unroll
        for (int e = 0; e < EPT / 2; e += 4) *(u32x4*)(dst + 2 * e) = u32x4{w[e], w[e + 1], w[e + 2], w[e + 3]};
    } else {
#pragma unroll
        for (int e = 0; e < EPT / 2; e += 2) *(u32x2*)(dst + 2 * e) = u32x2{w[e], w[e + 1]};
    }
}

// The merge of NP f16 partials of one row (merge_row_parts' fa_reduce LSE
// merge, src/flash_row_float.h:415-472, in fp32, fixed order): lane (h, dl) =
// (lane / (D/8), lane % (D/8)) loads 16 B = 8 dims of every part p = h (mod
// 64 / (D/8)); part p weighs w_p l_p, w_p = 2^(m_p - M), and the row is
// sum_p w_p l_p O~_p / sum_p w_p l_p.  Plain loads (a second launch).  D = 80,
// 96, 128, 256 (D = 64 keeps f32 partials: 8 parts per lane row would need a
// third lane-swap level).
template <int D>
constexpr int merge_ppr_h() { return 64 % (D / 8) == 0 ? 64 / (D / 8) : 1; }  // (4, 2, 1)
template <int D, int kIt>
__device__ __forceinline__ void merge_row_parts_h(const uint16_t* parts_o, const float* parts_ml, int NP, float* out,
                                                  int lane, int ostride, int mstride) {
    constexpr float kNegInf = -__builtin_inff();
    constexpr int LPP = D / 8;
    constexpr int PPR = merge_ppr_h<D>();
    static_assert(PPR == 1 || PPR == 2 || PPR == 4, "");
    const int h = lane / LPP, d8 = 8 * (lane % LPP);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the count)
    const __amdgpu_buffer_rsrc_t osrd = make_rsrc(parts_o, (uint32_t)(NP * ostride * 2));
    const __amdgpu_buffer_rsrc_t msrd = make_rsrc(parts_ml, (uint32_t)(NP * mstride * 4));
    u32x4 v[kIt];
    auto issue = [&](int p0) {
#pragma unroll
        for (int i = 0; i < kIt; i++)
            v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                 osrd, (uint32_t)(((p0 + PPR * i + h) * ostride + d8) * 2), 0, 0));
    };
    issue(0);
    const uint32_t mlm = __builtin_amdgcn_raw_buffer_load_b32(msrd, (uint32_t)(lane * mstride * 4), 0, 0);
    const uint32_t mll = __builtin_amdgcn_raw_buffer_load_b32(msrd, (uint32_t)(lane * mstride * 4 + 4), 0, 0);
    const float mp = lane < NP ? __builtin_bit_cast(float, mlm) : kNegInf;
    const float M = seg_reduce<true>(mp, 64);
    const float w = (mp == kNegInf) ? 0.0f : __builtin_amdgcn_exp2f(mp - M) * __builtin_bit_cast(float, mll);
    const float L = seg_reduce<false>(lane < NP ? w : 0.0f, 64);
    const int wi = __builtin_bit_cast(int, w);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; e++) acc[e] = 0.0f;
    for (int p0 = 0; p0 < NP; p0 += kIt * PPR) {  // wave-uniform
        if (p0 > 0) issue(p0);
#pragma unroll
        for (int i = 0; i < kIt; i++) {
            float wp = 0.0f;
#pragma unroll
            for (int j = 0; j < PPR; j++) {
                const float wj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(wi, (p0 + PPR * i + j) & 63));
                wp = (h == j) ? wj : wp;
            }
            const f16x8 x = __builtin_bit_cast(f16x8, v[i]);
#pragma unroll
            for (int e = 0; e < 8; e++) acc[e] += wp * (float)x[e];
        }
    }
#pragma unroll
    for (int e = 0; e < 8; e++) {
        if constexpr (PPR == 4) acc[e] = xor16_pair(acc[e], false);
        if constexpr (PPR >= 2) acc[e] = xor32_pair(acc[e], false);
    }
    if (h) return;
    const float inv = L == 0.0f ? __builtin_nanf("") : 1.0f / L;  // L == 0 (row fully masked) -> NaN like the reference
    *(f32x4*)(out + d8) = f32x4{acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv};
    *(f32x4*)(out + d8 + 4) = f32x4{acc[4] * inv, acc[5] * inv, acc[6] * inv, acc[7] * inv};
}

// One-row tiles, NW waves per workgroup: every wave writes its row-0 state
// (O, m, l) into its own LDS region (its steps have all landed), one barrier,
// then wave 0 merges the NW states (lane (h, dl): states p = h mod PPR, dims
// 4dl..4dl+3, one ds_read_b128 each).  With one chunk it writes dst; with
// several it publishes the workgroup's row write-through, drains, counts the
// workgroup on the tile's arrival word, and the last workgroup's wave 0 merges
// the chunks (merge_row_parts).  The cross-workgroup hand-off carries one row
// per workgroup instead of one per wave.
template <int D, bool VQ8, int NW>
__device__ __forceinline__ void wg_row_merge(const SplitArgs& a, const f32x4 (&o)[D / 16], float m_run, float l_tot,
                                             int chunk, int wave, int lane, int qt, int hs, int ik2, int iq3,
                                             int y, uint8_t* smem, int region) {
    constexpr int NB = D / QK;
    constexpr int NC = D / 16;
    constexpr float kNegInf = -__builtin_inff();
    constexpr int LPP = D / 4;
    constexpr int PPR = 64 % LPP == 0 ? 64 / LPP : 1;  // (D = 80 / 96: one part per lane row)
    const int g = lane >> 4, m = lane & 15;
    float* so = (float*)(smem + wave * region);  // [D] O row, then (m, l)
    if (m == 0) {  // column 0 = the tile's row; its dims sit on lanes 0, 16, 32, 48
        if constexpr (VQ8) {
#pragma unroll
            for (int b = 0; b < NB; b++) {
                const f32x4 e = o[2 * b], od = o[2 * b + 1];
                *(f32x4*)(so + 32 * b + 8 * g) = f32x4{e.x, od.x, e.y, od.y};
                *(f32x4*)(so + 32 * b + 8 * g + 4) = f32x4{e.z, od.z, e.w, od.w};
            }
        } else {
#pragma unroll
            for (int c = 0; c < NC; c++) *(f32x4*)(so + 16 * c + 4 * g) = o[c];
        }
        if (g == 0) *(f32x2*)(so + D) = f32x2{m_run, l_tot};
    }
    __syncthreads();
    if (wave != 0) return;
    FATTN_SSTAMP(11);
    // ---- wave 0: merge the NW states
    const int h = lane / LPP, d4 = 4 * (lane % LPP);
    const f32x2 ml = lane < NW ? *(const f32x2*)((const float*)(smem + lane * region) + D) : f32x2{kNegInf, 0.0f};
    const float M = seg_reduce<true>(ml.x, 64);
    const float w = (ml.x == kNegInf) ? 0.0f : __builtin_amdgcn_exp2f(ml.x - M);
    const float L = seg_reduce<false>(w * ml.y, 64);
    const int wi = __builtin_bit_cast(int, w);
    constexpr int NI = (NW + PPR - 1) / PPR;
    f32x4 part[NI];
#pragma unroll
    for (int i = 0; i < NI; i++) {
        const int p = PPR * i + h;
        part[i] = p < NW ? *(const f32x4*)((const float*)(smem + p * region) + d4) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < NI; i++) {
        float wp = 0.0f;
#pragma unroll
        for (int j = 0; j < PPR; j++) {
            const float wj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(wi, (PPR * i + j) & 63));
            wp = (h == j && PPR * i + j < NW) ? wj : wp;
        }
        acc += wp * part[i];
    }
    if constexpr (PPR == 4) {
        acc.x = xor16_pair(acc.x, false);
        acc.y = xor16_pair(acc.y, false);
        acc.z = xor16_pair(acc.z, false);
        acc.w = xor16_pair(acc.w, false);
    }
    if constexpr (PPR >= 2) {
        acc.x = xor32_pair(acc.x, false);
        acc.y = xor32_pair(acc.y, false);
        acc.z = xor32_pair(acc.z, false);
        acc.w = xor32_pair(acc.w, false);
    }
    const int riq1 = qt * a.QPT;
    const int riq2 = ik2 * a.rk2 + hs * a.R;
    float* out = a.dst + (((int64_t)iq3 * a.NQ + riq1) * a.H + riq2) * D;
    if (a.n_chunks == 1) {
        if (h == 0) {
            const float inv = L == 0.0f ? __builtin_nanf("") : 1.0f / L;
            *(f32x4*)(out + d4) = acc * inv;
        }
        return;
    }
#ifdef FATTN_DIAG_NOPUBLISH
    if (acc.x == 12345.0f) a.dst[0] = L;  // diagnostic build only: stop after the workgroup merge
    return;
#endif
    const int64_t tile = (int64_t)iq3 * gridDim.y + y;
    float* po = a.ws_o + (tile * a.n_chunks + chunk) * D;
    auto bits = [](float x) { return __builtin_bit_cast(uint32_t, x); };
    if (h == 0) st_sc1(po + d4, u32x4{bits(acc.x), bits(acc.y), bits(acc.z), bits(acc.w)});
    if (lane == 0) st_sc1_x2(a.ws_ml + 2 * (tile * a.n_chunks + chunk), u32x2{bits(M), bits(L)});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FATTN_SSTAMP(12);
#ifdef FATTN_DIAG_NOATOMIC
    return;  // diagnostic build only: stop after the published row drained
#endif
    int last = 0;
    if (lane == 0) last = arrive_last(a, tile, a.n_chunks);
    last = __builtin_amdgcn_readfirstlane(last);
    FATTN_SSTAMP(14);
    if (!last) return;
    // as few load slots per lane as the chunk count needs (a slot past it is
    // still an issued instruction; config 3: 8 chunks = 4 slots)
    const float* po_all = a.ws_o + tile * a.n_chunks * D;
    const float* pml_all = a.ws_ml + 2 * tile * a.n_chunks;
    const int need = (a.n_chunks + merge_ppr<D>() - 1) / merge_ppr<D>();
    if (need <= 4) merge_row_parts<D, 4>(po_all, pml_all, a.n_chunks, out, lane);
    else if (need <= 8) merge_row_parts<D, 8>(po_all, pml_all, a.n_chunks, out, lane);
    else merge_row_parts<D>(po_all, pml_all, a.n_chunks, out, lane);
    FATTN_SSTAMP(13);
}

// Tail of a split-KV workgroup: the waves' (O, m, l) states merge.  EPI (the
// plan's a.wave_merge, a template parameter so that each kernel carries only
// its own epilogue's registers -- combine_tile's in-flight loads made the
// whole kernel spill): 0 = through LDS (wave w's image at smem + w * region)
// and then across the tile's chunks via the last-arriving workgroup
// (combine_tile); 1 = one-row tiles, every wave publishes and the
// last-arriving wave merges (wave_merge_epilogue); 2 = one-row tiles, LDS
// merge and one published row per workgroup (wg_row_merge).  `active`: this
// wave holds a state (waves >= NW must be inactive).  `sync_first`: the images
// alias step buffers, so wait for every wave before writing them.
template <int KT, int VT, int D, int NW, int EPI>
__device__ __forceinline__ void split_epilogue(const SplitArgs& a, f32x4 (&o)[D / 16], float m_run, float l_run,
                                               float (&corr)[(D + QK - 1) / QK], int wave, int lane, int qt, int hs, int ik2,
                                               int iq3, int y, int chunk, uint8_t* smem, int region, bool active,
                                               bool sync_first) {
    using C = SplitCfg<KT, VT, D>;
    constexpr int NB = D / QK;
    constexpr int NC = D / 16;
    constexpr float kNegInf = -__builtin_inff();
    constexpr bool kVQ8 = C::VTT == FATTN_TYPE_Q8_0;
    constexpr bool kVQ = C::VTT != FATTN_TYPE_F16;
    constexpr float kVOff = kVQ8 ? 1152.0f : 1032.0f;
    const int g = lane >> 4;
    const int m = lane & 15;
    // split_step keeps the reference max in natural units; the merges work in log2
    m_run = m_run == kNegInf ? kNegInf : m_run * 1.4426950408889634f;
    const float l_tot = grp4_sum(l_run);
    if constexpr (kVQ) {
        // O^T tiles of block b (columns 32b..32b+31) carry kVOff * sum(P'_b) too
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const float cb = kVOff * grp4_sum(corr[b]);
            o[2 * b] -= cb;
            o[2 * b + 1] -= cb;
        }
    }
    if constexpr (EPI == 1) {
        static_assert(D == 128, "per-wave merge: lane i <-> dims 2i, 2i+1");
        wave_merge_epilogue<D, kVQ8, NW>(a, o, m_run, l_tot, chunk, wave, lane, qt, hs, ik2, iq3, y);
        return;
    } else if constexpr (EPI == 2) {
        wg_row_merge<D, kVQ8, NW>(a, o, m_run, l_tot, chunk, wave, lane, qt, hs, ik2, iq3, y, smem, region);
        return;
    }
    constexpr int MS = C::kMergeStride;
    // the merge images alias step buffers other waves may still be reading
    if (sync_first) __syncthreads();
    float* mo = (float*)(smem + wave * region);    // [16][MS]
    float* mml = (float*)(smem + wave * region + kRows * MS * 4);  // [16][2]
    // valid rows of this tile form a prefix [0, rv); only those are merged
    const int rv = tile_rows(a, qt, hs);
    if (m >= rv || !active) {
        // nothing of this column is needed
    } else if constexpr (kVQ8) {
        // tile E_b holds columns 32b + 2(4g+reg), O_b the odd neighbours
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const f32x4 e = o[2 * b], od = o[2 * b + 1];
            *(f32x4*)(mo + m * MS + 32 * b + 8 * g) = f32x4{e.x, od.x, e.y, od.y};
            *(f32x4*)(mo + m * MS + 32 * b + 8 * g + 4) = f32x4{e.z, od.z, e.w, od.w};
        }
    } else {
#pragma unroll
        for (int c = 0; c < NC; c++) *(f32x4*)(mo + m * MS + 16 * c + 4 * g) = o[c];
    }
    if (g == 0 && m < rv && active) {
        mml[2 * m] = m_run;
        mml[2 * m + 1] = l_tot;
    }
    __syncthreads();
    FATTN_SSTAMP(11);

    constexpr int EPT = epi_ept<D>();  // outputs per thread: 16 rows x D over 256 threads
    const int tm = threadIdx.x / 16;
    const int tj = threadIdx.x % 16;
    const int d0 = tj * EPT;
    const bool dok = d0 < D;  // (D = 80 / 96: the last threads of a row hold no dims)
    float M = kNegInf;
    float mw[NW], lw[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const float* ml = (const float*)(smem + w * region + kRows * MS * 4);
        mw[w] = tm < rv ? ml[2 * tm] : kNegInf;
        lw[w] = tm < rv ? ml[2 * tm + 1] : 0.0f;
        M = fmaxf(M, mw[w]);
    }
    float L = 0.0f;
    float acc[EPT];
#pragma unroll
    for (int e = 0; e < EPT; e++) acc[e] = 0.0f;
    if (tm < rv) {
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const float wt = (mw[w] == kNegInf) ? 0.0f : __builtin_amdgcn_exp2f(mw[w] - M);
            L += wt * lw[w];
            const float* ow = (const float*)(smem + w * region) + tm * MS + (dok ? d0 : 0);
#pragma unroll
            for (int e = 0; e < EPT; e++) acc[e] += wt * ow[e];
        }
    }
    auto dst_row = [&](int r) -> float* {
        const int rq = div_R(a, r);
        const int riq1 = qt * a.QPT + rq;
        const int riq2 = ik2 * a.rk2 + hs * a.R + (r - rq * a.R);
        return a.dst + (((int64_t)iq3 * a.NQ + riq1) * a.H + riq2) * D;
    };
    if (a.n_chunks == 1) {
        if (tm < rv && dok) {
            float* out = dst_row(tm) + d0;
            const float inv = 1.0f / L;  // L == 0 (row fully masked) -> NaN like the reference
#pragma unroll
            for (int e = 0; e < EPT; e += 4) {
                f32x4 v;
                v.x = L == 0.0f ? __builtin_nanf("") : acc[e] * inv;
                v.y = L == 0.0f ? __builtin_nanf("") : acc[e + 1] * inv;
                v.z = L == 0.0f ? __builtin_nanf("") : acc[e + 2] * inv;
                v.w = L == 0.0f ? __builtin_nanf("") : acc[e + 3] * inv;
                *(f32x4*)(out + e) = v;
            }
        }
        FATTN_SSTAMP(12);
        return;
    }

#ifdef FATTN_DIAG_NOPUBLISH
    // diagnostic build only: stop after the 4-wave merge
    if (acc[0] == 12345.0f) a.dst[0] = L;
    return;
#endif
    // ---- several chunks: the workgroup that arrives last for the tile merges
    // all partials (no second launch).  Hand-off (MI355X_MICROARCH.md,
    // inter-workgroup visibility, first row of the sc1 table): partial bytes
    // stored sc1 (write-through), each storing wave drains vmcnt, barrier, ONE
    // agent-scope atomic add per workgroup on the tile's own 256-B line; the
    // last adder reads the others' partials with sc1 loads -- all of them in
    // one round trip -- while its own stays in LDS.
    const int64_t tile = (int64_t)iq3 * gridDim.y + y;
    if (a.merge_launch == 1 && a.part_f16) {
        if constexpr (EPT % 4 == 0) {
            if (tm < rv) {
                const int64_t slot = (tile * a.n_chunks + chunk) * kRows + tm;
                if (dok) store_part_f16<EPT>((uint16_t*)a.ws_o + slot * D + d0, acc, L);
                if (tj == 0) *(f32x2*)(a.ws_ml + 2 * slot) = f32x2{M, L};
            }
        }
        return;
    }
    if (tm < rv) {
        const int64_t slot = (tile * a.n_chunks + chunk) * kRows + tm;
        auto bits = [](float x) { return __builtin_bit_cast(uint32_t, x); };
        if (dok) {
#pragma unroll
            for (int e = 0; e < EPT; e += 4)
                st_sc1(a.ws_o + slot * D + d0 + e,
                       u32x4{bits(acc[e]), bits(acc[e + 1]), bits(acc[e + 2]), bits(acc[e + 3])});
        }
        if (tj == 0) st_sc1_x2(a.ws_ml + 2 * slot, u32x2{bits(M), bits(L)});
    }
    // second-launch merge (fattn_merge_kernel): the kernel boundary orders
    // these stores before its loads; no drain, no counter
    if (a.merge_launch == 1) return;
    if (a.merge_launch == 2) {
        // in-kernel: wait for the tile's chunks, then every workgroup merges a
        // share of the tile's rows, one wave per row (row r: wave r mod NW of
        // chunk (r / NW) mod n_chunks), as fattn_merge_kernel would
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
        __syncthreads();
        int* flag = (int*)smem;  // (every wave is done reading the merge images)
        if (threadIdx.x == 0) *flag = tile_arrive_wait(a, tile, a.n_chunks);
        __syncthreads();
        const bool ok = *flag != 0;
        FATTN_SSTAMP(12);
        for (int r = chunk * NW + wave; r < rv; r += NW * a.n_chunks) {  // wave-uniform
            const int64_t s0 = tile * a.n_chunks * kRows + r;  // chunk 0's row r
            float* out = dst_row(r);
            if (ok) {
                merge_row_parts<D, 8>(a.ws_o + s0 * D, a.ws_ml + 2 * s0, a.n_chunks, out, lane, kRows * D, 2 * kRows);
            } else if (lane < D / 4) {
                *(f32x4*)(out + 4 * lane) = f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""),
                                                  __builtin_nanf("")};
            }
        }
        FATTN_SSTAMP(13);
        return;
    }
    // every storing wave drains: the merging workgroup reads its own partial back too
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef FATTN_DIAG_NOATOMIC
    return;  // diagnostic build only: stop after the published stores drained
#endif
    __syncthreads();  // every storing wave has drained; every wave is done reading the merge image
    int* last_flag = (int*)smem;
    if (threadIdx.x == 0) *last_flag = arrive_last(a, tile, a.n_chunks);
    __syncthreads();
    FATTN_SSTAMP(12);
    if (!*last_flag) return;
    combine_tile<D, (D == 128 && KT != FATTN_TYPE_F16) ? 8 : 2>(a, tile, qt, hs, ik2, iq3, rv, 0, smem);
    FATTN_SSTAMP(13);
}

// One 32-position step of one wave: S^T = K.Q^T for the step's two 16-row
// key tiles, scale + mask, online softmax of the wave's 16 packed columns,
// O^T += V^T.P^T.  `buf` is the step's LDS image [K rows | V rows | mask rows];
// `wait_v()` runs between the softmax and P.V (the split kernel waits there
// for the step's V, which it issues last).  `first`: o, l are still zero.
// Used by fattn_split_kernel.
template <int KT, int VT, int D, bool HM, typename WaitV>
__device__ __forceinline__ void split_step(const SplitArgs& a, const uint8_t* buf, const f16x8 (&qop)[(D + QK - 1) / QK], int mq,
                                           int g, int i16, int nvalid, bool first, float& m_run, float& l_run,
                                           f32x4 (&o)[D / 16], float (&corr)[(D + QK - 1) / QK], WaitV&& wait_v) {
    using C = SplitCfg<KT, VT, D>;
    constexpr int NB = (D + QK - 1) / QK;  // k-steps of S^T (D = 80: the last one half zero)
    constexpr int NC = D / 16;
    constexpr float kNegInf = -__builtin_inff();
    constexpr bool kVQ8 = C::VTT == FATTN_TYPE_Q8_0;
    constexpr bool kVQ = C::VTT != FATTN_TYPE_F16;
    const float log2e = 1.4426950408889634f;
    const uint8_t* kb = buf;
    const uint8_t* vb = buf + C::kBytes;
    const uint8_t* mb = buf + C::kBytes + C::vBytes;

    // -- S^T = K.Q^T for the two 16-row tiles
    f32x4 st[2];
#pragma unroll
    for (int t = 0; t < 2; t++) {
        st[t] = f32x4{0, 0, 0, 0};
        if constexpr (KT == FATTN_TYPE_F16) {
#pragma unroll
            for (int b = 0; b < NB; b++) st[t] = mfma16(k_operand<KT, D>(kb, 16 * t + i16, g, b, 0), qop[b], st[t]);
        } else {
            const RowScales<KT, D> ks = row_scales<KT, D>(kb + (16 * t + i16) * C::rowK);
#pragma unroll
            for (int b = 0; b < NB; b++)
                st[t] = mfma16(k_operand<KT, D>(kb, 16 * t + i16, g, b, scale_bcast(ks, b)), qop[b], st[t]);
        }
    }

    // -- u = s * scale + mask in one v_fma_mix per score (the f16 mask converts
    // inside it); positions past this wave's slice -> -inf
    float sv[8];
#pragma unroll
    for (int t = 0; t < 2; t++) {
        if constexpr (HM) {
            const uint8_t* mp = mb + (mq < a.QPT ? mq : 0) * (kStep * 2) + (16 * t + 4 * g) * 2;
            const u32x2 mw = *(const u32x2*)mp;
            const f16x2 m01 = as_h2(mw.x), m23 = as_h2(mw.y);
            sv[4 * t + 0] = __builtin_fmaf(st[t][0], a.scale, (float)m01.x);
            sv[4 * t + 1] = __builtin_fmaf(st[t][1], a.scale, (float)m01.y);
            sv[4 * t + 2] = __builtin_fmaf(st[t][2], a.scale, (float)m23.x);
            sv[4 * t + 3] = __builtin_fmaf(st[t][3], a.scale, (float)m23.y);
        } else {
#pragma unroll
            for (int r = 0; r < 4; r++) sv[4 * t + r] = st[t][r] * a.scale;
        }
    }
    if (nvalid < kStep) {  // wave-uniform: only a slice's partial last step
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (16 * (j >> 2) + 4 * g + (j & 3) >= nvalid) sv[j] = kNegInf;
    }

    // -- online softmax for column m (the 4 lanes l, l^16, l^32, l^48 share it).
    // m_run is the reference max the exponentials use (natural units); it
    // moves only when a score exceeds it by more than kRescaleNat, so p stays
    // <= 2^kRescaleLog2 and most steps skip the rescale (deferred max).
    float tmax = fmaxf(fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3])),
                       fmaxf(fmaxf(sv[4], sv[5]), fmaxf(sv[6], sv[7])));
    tmax = grp4_max(tmax);
    if (__builtin_amdgcn_ballot_w64(tmax > m_run + kRescaleNat)) {
        const float m_new = fmaxf(m_run, tmax);
        if (!first) {  // o, l are still 0 at a wave's first step
            const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * log2e);  // m_run = -inf: 0
            l_run *= alpha;
#pragma unroll
            for (int c = 0; c < NC; c++) o[c] *= alpha;
            if constexpr (kVQ) {
#pragma unroll
                for (int b = 0; b < NB; b++) corr[b] *= alpha;
            }
        }
        m_run = m_new;
    }
    const float m_off = (m_run == kNegInf) ? 0.0f : -m_run * log2e;
    float pv[8];
#pragma unroll
    for (int j = 0; j < 8; j++) pv[j] = __builtin_amdgcn_exp2f(__builtin_fmaf(sv[j], log2e, m_off));
    l_run += ((pv[0] + pv[1]) + (pv[2] + pv[3])) + ((pv[4] + pv[5]) + (pv[6] + pv[7]));

    f16x8 pb;
    pb.s0 = (f16)pv[0]; pb.s1 = (f16)pv[1]; pb.s2 = (f16)pv[2]; pb.s3 = (f16)pv[3];
    pb.s4 = (f16)pv[4]; pb.s5 = (f16)pv[5]; pb.s6 = (f16)pv[6]; pb.s7 = (f16)pv[7];

    // -- O^T += V^T.P^T (V of step s landed)
    wait_v();
    if constexpr (C::VTT == FATTN_TYPE_F16) {
#pragma unroll
        for (int c = 0; c < NC; c++) o[c] = mfma16(v_operand_f16<VT, D>(vb, c, g, i16), pb, o[c]);
    } else {
        const int rA = 4 * g, rB = 16 + 4 * g;
#pragma unroll
        for (int b = 0; b < NB; b++) {
            constexpr int BB = TypeInfo<C::VTT>::block_bytes;
            // block-b scales of this lane's 8 rows (4g..4g+3, 16+4g..16+4g+3):
            // the dword holding each, then f16 pairs {row r, row r+1}
            uint32_t sw[8];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if constexpr (C::rowV % 4 != 0) {  // D = 96: rows not a whole number of dwords
                    sw[r] = *(const uint16_t*)(vb + (rA + r) * C::rowV + BB * b);
                    sw[4 + r] = *(const uint16_t*)(vb + (rB + r) * C::rowV + BB * b);
                } else {
                    sw[r] = *(const uint32_t*)(vb + (rA + r) * C::rowV + ((BB * b) & ~3));
                    sw[4 + r] = *(const uint32_t*)(vb + (rB + r) * C::rowV + ((BB * b) & ~3));
                }
            }
            const uint32_t sel = scale_hi<C::VTT, D>(b) ? 0x07060302u : 0x05040100u;  // b is unrolled
            const f16x2 d01 = as_h2(perm_b32(sw[1], sw[0], sel)), d23 = as_h2(perm_b32(sw[3], sw[2], sel));
            const f16x2 d45 = as_h2(perm_b32(sw[5], sw[4], sel)), d67 = as_h2(perm_b32(sw[7], sw[6], sel));
            // P'_b = P * d_b (element j <-> row of element j of the A operand)
            f16x8 pbd;
            pbd.s01 = pb.s01 * d01;
            pbd.s23 = pb.s23 * d23;
            pbd.s45 = pb.s45 * d45;
            pbd.s67 = pb.s67 * d67;
            const f16x2 one2 = {(f16)1.0f, (f16)1.0f};
            corr[b] = __builtin_amdgcn_fdot2(pbd.s01, one2, corr[b], false);
            corr[b] = __builtin_amdgcn_fdot2(pbd.s23, one2, corr[b], false);
            corr[b] = __builtin_amdgcn_fdot2(pbd.s45, one2, corr[b], false);
            corr[b] = __builtin_amdgcn_fdot2(pbd.s67, one2, corr[b], false);
            if constexpr (kVQ8) {
                // one u16 per row carries columns 2i (-> tile E_b) and 2i+1 (-> tile O_b)
                const uint8_t* cp = vb + b * BB + 2 + 2 * i16;
                uint32_t w[8];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    w[r] = *(const uint16_t*)(cp + (rA + r) * C::rowV);
                    w[4 + r] = *(const uint16_t*)(cp + (rB + r) * C::rowV);
                }
                u32x4 ae, ao;  // f16 pairs 1152 + q (exact)
#pragma unroll
                for (int pr = 0; pr < 4; pr++) {
                    // bytes [e_r, o_r, e_r+1, o_r+1] -> xor 0x80 -> f16 magic 0x64xx
                    const uint32_t t2 = (w[2 * pr] | (w[2 * pr + 1] << 16)) ^ 0x80808080u;
                    ae[pr] = perm_b32(0x64646464u, t2, 0x04020400u);
                    ao[pr] = perm_b32(0x64646464u, t2, 0x04030401u);
                }
                o[2 * b] = mfma16(__builtin_bit_cast(f16x8, ae), pbd, o[2 * b]);
                o[2 * b + 1] = mfma16(__builtin_bit_cast(f16x8, ao), pbd, o[2 * b + 1]);
            } else {  // Q4_0: byte i carries column i (low nibble) and 16+i (high nibble)
                const uint8_t* cp = vb + b * BB + 2 + i16;
                uint32_t w[8];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    w[r] = cp[(rA + r) * C::rowV];
                    w[4 + r] = cp[(rB + r) * C::rowV];
                }
                u32x4 al, ah;  // f16 pairs 1032 + (nib - 8) (exact)
#pragma unroll
                for (int pr = 0; pr < 4; pr++) {
                    const uint32_t x = w[2 * pr] | (w[2 * pr + 1] << 16);
                    al[pr] = (x & 0x000F000Fu) | 0x64006400u;
                    ah[pr] = ((x >> 4) & 0x000F000Fu) | 0x64006400u;
                }
                o[2 * b] = mfma16(__builtin_bit_cast(f16x8, al), pbd, o[2 * b]);
                o[2 * b + 1] = mfma16(__builtin_bit_cast(f16x8, ah), pbd, o[2 * b + 1]);
            }
        }
    }

}

// waves per SIMD the split kernel's register budget allows (__launch_bounds__)
template <int KT, int D, int GRAN>
constexpr int split_waves_per_simd() {
    return (KT == FATTN_TYPE_F16 || GRAN == 4 || D == 256) ? 2 : 4;
}

// NWV waves per workgroup (4, 8 or 16), each streaming its own slice of the
// chunk.  More waves per CU put more LDS-DMA instructions in flight from more
// issuing waves (tools/hbm_probe: a 35.7 MB read takes 8.3 us from 256 4-wave
// workgroups, 6.4 us from 16 waves per CU) and let the SIMDs interleave the
// steps' dependent LDS -> VALU -> MFMA chains.
template <int KT, int VT, int D, int GRAN, bool HM, int NWV, int EPI>
__global__ __launch_bounds__(NWV * kWave, (KT == FATTN_TYPE_F16 || GRAN == 4 || D == 256) ? 2 : 4) void fattn_split_kernel(
    const SplitArgs a) {
    using C = SplitCfg<KT, VT, D>;
    using P = StepPlan<KT, VT, D, GRAN>;
    constexpr int NI = P::NIKV + (HM ? P::NIM : 0);  // VMEM instructions per step
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NB = (D + QK - 1) / QK;  // 32-wide k-steps of QK^T (= ggml blocks per row; D = 80: 3)
    constexpr int NC = D / 16;   // 16-wide output column groups (MFMA tiles of O^T)
    constexpr float kNegInf = -__builtin_inff();
    // quantised V: the A operand is the exact integer code plus the magic-number
    // offset (1152 for Q8_0, 1032 for Q4_0) with the block scale folded into P;
    // corr[b] accumulates sum(P * d_b) so the offset comes off once in the epilogue

    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane lets the compiler see it, so the
    // slice bounds, loop counts and LDS-DMA bases (M0) stay scalar
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4;
    const int i16 = lane & 15;
    FATTN_SSTAMP_INIT();
    FATTN_SSTAMP(0);

    // ---- tile decode: y -> (kv head, head subgroup, query-row tile)
    int chunk, y, iq3;
    tile_coords(a, chunk, y, iq3);
    int qt = 0, hs = 0, ik2 = y, ik3 = iq3;  // common case without runtime division
    if (a.n_qt != 1 || a.n_hsub != 1) {
        qt = y % a.n_qt;
        hs = (y / a.n_qt) % a.n_hsub;
        ik2 = y / (a.n_qt * a.n_hsub);
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;

    // this lane's MFMA column m = i16 -> (query row, q head)
    const int m = i16;
    const int mq = div_R(a, m);
    const int mh = hs * a.R + (m - mq * a.R);
    const int iq1 = qt * a.QPT + mq;
    const int iq2 = ik2 * a.rk2 + mh;
    const bool row_ok = (m < a.QPT * a.R) && (iq1 < a.NQ) && (mh < a.rk2);

    // ---- this wave's KV slice
    const int wl = a.chunk_len / NWV;
    const int c_hi = min(a.N, (chunk + 1) * a.chunk_len);
    const int w_lo = chunk * a.chunk_len + wave * wl;
    const int w_hi = min(c_hi, w_lo + wl);
    const int nsteps = w_hi > w_lo ? (w_hi - w_lo + kStep - 1) / kStep : 0;
    const int nbuf = a.nbuf;

    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    rs.m = make_srd(a.mask, HM ? a.m_span : 0);
    uint8_t* wbuf = smem + wave * a.wave_bytes;
    const int mrow0 = qt * a.QPT;

    // Staggered priorities: the waves of a CU otherwise interleave their DMA
    // issue, so every wave's last piece lands near the end of the burst and
    // all compute starts late; by priority the first waves' steps land first
    // and their compute overlaps the rest of the stream.
    // (split_prio 1: no priorities; 2: staggered only while the first steps issue)
    // (NWV > 4: by the wave's rank among the waves of its SIMD, wave / 4)
    if (a.split_prio != 1) {
        switch (__builtin_amdgcn_readfirstlane(NWV == 4 ? wave : wave >> 2)) {
            case 0: __builtin_amdgcn_s_setprio(3); break;
            case 1: __builtin_amdgcn_s_setprio(2); break;
            case 2: __builtin_amdgcn_s_setprio(1); break;
            default: break;
        }
    }

    // ---- Q^T operand (B of S^T = K.Q^T), rounded to f16 like src/utils.h:10
    // (lanes of unused columns point past the descriptor: zeros, no traffic).
    // Loaded first, as asm (no compiler wait), so that waiting for Q leaves the
    // steps' LDS-DMA behind it in flight: compute starts as soon as step 0's K
    // and mask land.
    u32x4 qraw[NB][2];
    {
        const i32x4 qs = make_srd(a.q + (int64_t)iq3 * a.q_nb3, a.q_span);
        const uint32_t qoff = row_ok ? (uint32_t)iq1 * (uint32_t)a.q_nb1 + (uint32_t)iq2 * (uint32_t)a.q_nb2 + 32 * g
                                     : a.q_span;
#pragma unroll
        for (int b = 0; b < NB; b++) {
            // (D = 80: dims past D come from past the descriptor, as zeros)
            const uint32_t qb = (D % QK == 0 || 32 * b + 8 * g < D) ? qoff + 128 * b : a.q_span;
            qraw[b][0] = ld_buf_untracked<kTagQ>(qs, qb);
            qraw[b][1] = ld_buf_untracked<kTagQ>(qs, qb + 16);
        }
    }
    // ---- -inf steps (src/flash-llama.h:275-278 skips their compute): a step
    // whose mask is -inf for every key of every query row of the tile adds
    // exp(-inf) = 0 to o and l.  Its K and V are not fetched: their DMA goes
    // through empty descriptors (no HBM traffic, zeros in LDS; the mask still
    // lands, so every score is -inf and the step's compute adds exactly 0).
    // Loop and vmcnt accounting are unchanged.  The mask words of the wave's
    // steps are read here beside Q (their wait is Q's): one (row, step) pair
    // of 64 B per lane, when the tile's rows x steps fit the wave and the
    // wave has at least 4 steps; the prologue's steps are fetched regardless.
    // Measured (profiles/r02_skip): config 3 (2 steps per wave, no prefetch)
    // unchanged; 8 heads x N = 32768 with 70 % of the cache masked 16.1 vs
    // 17.1-17.5 us; the same unmasked 17.6-18.2 vs 16.9-17.5 us (the loads
    // ahead of the first wait).  Reading the words after step 0 instead, or
    // skipping by control flow in the loop, measured slower everywhere.
    const int pro = min(nbuf, nsteps);  // steps issued before the loop
    const int n_rows = HM ? min(a.QPT, a.NQ - mrow0) : 0;
    const bool pre = HM && a.step_skip && nsteps >= 4 && n_rows * nsteps <= kWave;
    u32x4 mraw[4] = {};
    if (pre) {
        const int r = lane / nsteps, st = lane - r * nsteps;
        const uint32_t moff = r < n_rows ? (uint32_t)(mrow0 + r) * (uint32_t)a.m_nb1 + (uint32_t)(w_lo + st * kStep) * 2
                                         : a.m_span;  // past the descriptor: no traffic
#pragma unroll
        for (int j = 0; j < 4; j++) mraw[j] = ld_buf_untracked<kTagMaskWords>(rs.m, moff + 16 * j);
    }
    for (int s = 0; s < pro; s++) {
        issue_step<KT, VT, D, GRAN, HM>(a, rs, w_lo + s * kStep, mrow0, wbuf + s * C::stepBytes, lane);
    }
    // this launch's stamp on the tile's arrival word, by each lane that will
    // count an arrival: issued after the prologue's DMA, so no wait is spent
    // on it (at most one DMA instruction's worth in the counted waits below)
    if (a.n_chunks > 1 && a.merge_launch != 1 && lane == 0 && (EPI == 1 || wave == 0))
        arrival_begin(a, (int64_t)iq3 * gridDim.y + y);

    FATTN_SSTAMP(1);
    if (a.split_prio == 2) __builtin_amdgcn_s_setprio(0);
    wait_steps<NI>(pro);  // Q and the mask words landed (the steps issued after them may fly on)
    // every untracked result, on every path, passes its fence right behind
    // that wait (nothing reads or moves those registers before it)
#pragma unroll
    for (int b = 0; b < NB; b++) {
        reg_fence<kTagQ>(qraw[b][0]);
        reg_fence<kTagQ>(qraw[b][1]);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) reg_fence<kTagMaskWords>(mraw[j]);
    f16x8 qop[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const f32x4 x0 = __builtin_bit_cast(f32x4, qraw[b][0]), x1 = __builtin_bit_cast(f32x4, qraw[b][1]);
        f16x8 h;
        h.s0 = (f16)x0.x; h.s1 = (f16)x0.y; h.s2 = (f16)x0.z; h.s3 = (f16)x0.w;
        h.s4 = (f16)x1.x; h.s5 = (f16)x1.y; h.s6 = (f16)x1.z; h.s7 = (f16)x1.w;
        qop[b] = h;
    }
    // bit s: step s has a live key (steps past 64 and unprefetched waves: all)
    uint64_t live = ~0ull;
    if (pre) {
        constexpr uint32_t kNegInf2 = 0xFC00FC00u;  // two f16 -inf
        bool lv = false;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            lv |= (mraw[j].x != kNegInf2) | (mraw[j].y != kNegInf2) | (mraw[j].z != kNegInf2) | (mraw[j].w != kNegInf2);
        }
        const uint64_t bl = __builtin_amdgcn_ballot_w64(lv && lane < n_rows * nsteps);
        live = 0;
        for (int r = 0; r < n_rows; r++) live |= bl >> (r * nsteps);
    }

    float m_run = kNegInf;  // reference max (natural units) of column m
    float l_run = 0.0f;     // this lane's partial row sum
    f32x4 o[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) o[c] = f32x4{0, 0, 0, 0};
    float corr[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) corr[b] = 0.0f;

    int cur = 0;  // buffer of step s
    for (int s = 0; s < nsteps; s++) {
        const int ahead = min(nbuf - 1, nsteps - 1 - s);  // steps issued after step s
        // K and mask of step s landed (its V and the later steps may fly on)
        wait_steps_plus<NI, P::NIV>(ahead);
        if (s < 8) FATTN_SSTAMP(2 + s);
#ifdef FATTN_DIAG_NOCOMPUTE
        // diagnostic build only: memory-side ceiling of this access pattern
        wait_steps<NI>(ahead);
        if (s + nbuf < nsteps) {
            issue_step<KT, VT, D, GRAN, HM>(a, rs, w_lo + (s + nbuf) * kStep, mrow0, wbuf + cur * C::stepBytes, lane);
        }
        cur = (cur + 1 == nbuf) ? 0 : cur + 1;
        continue;
#endif
        const int n0 = w_lo + s * kStep;
        int s_opaque = s;  // hides "first step" from loop peeling (a second copy of the body)
        asm volatile("" : "+s"(s_opaque));
        split_step<KT, VT, D, HM>(a, wbuf + cur * C::stepBytes, qop, mq, g, i16, min(kStep, w_hi - n0), s_opaque == 0,
                                  m_run, l_run, o, corr, [&] { wait_steps<NI>(ahead); });
        if (nsteps <= 4 && s < 2) FATTN_SSTAMP(6 + 2 * s);  // (stamps build: step s computed)

        // -- refill this buffer with step s + nbuf (K/V not fetched if -inf)
        if (s + nbuf < nsteps) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const int sn = s + nbuf;
            issue_step<KT, VT, D, GRAN, HM>(a, rs, w_lo + sn * kStep, mrow0, wbuf + cur * C::stepBytes, lane,
                                            sn >= 64 || ((live >> sn) & 1));
            if (nsteps <= 4 && s < 2) FATTN_SSTAMP(7 + 2 * s);  // (stamps build: step s + nbuf issued)
        }
        cur = (cur + 1 == nbuf) ? 0 : cur + 1;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#ifdef FATTN_DIAG_NOTAIL
    // diagnostic build only: stop before the merge / publish tail
    {
        float keep = l_run + m_run;  // keep the loop's results (all of O) alive
#pragma unroll
        for (int c = 0; c < NC; c++) keep += o[c].x + o[c].y + o[c].z + o[c].w;
        if (keep == 12345.0f) a.dst[0] = keep;
    }
    return;
#endif
    FATTN_SSTAMP(10);
    split_epilogue<KT, VT, D, NWV, EPI>(a, o, m_run, l_run, corr, wave, lane, qt, hs, ik2, iq3, y, chunk, smem, a.wave_bytes,
                                   true, false);
    FATTN_SSTAMP_FLUSH();
}

// ---------------------------------------------------------------- loader waves
// The split kernel with the refill of its later steps taken off the compute
// waves (one-row tiles whose whole chunk fits the LDS; config 3).  In
// fattn_split_kernel each wave issues its own steps: a wave that issues step
// s + 1 before computing step s stalls on the CU's full memory queue before it
// can compute (both steps in flight: 12.2 vs 11.3 us), and a wave that issues
// it after computing step s leaves that queue idle for the whole of step s's
// compute (stamps, round 6: step 0 lands at 3.9 us, is computed by 5.7, step 1
// issued at 6.2).  Here each compute wave issues its step 0 (as before), the
// workgroup meets at one barrier, and NLD loader waves then issue every later
// step of every compute wave -- into the queue behind all of step 0 -- and hand
// each (wave, step) over by two LDS flags (K + mask landed, V landed), set
// behind counted vmcnt waits; the compute waves never wait on an issue.  (A
// first form whose loaders issued step 0 too took 13.5 us: the loaders could
// flag step 0 only after issuing everything, profiles/r06_c.)  Same compute
// (split_step) and epilogue (wg_row_merge).  Every step of the chunk is
// resident: LDS = NWV x steps x stepBytes + flags.
constexpr int kSplitLoaders = 4;
constexpr int kSplitLdFlagBytes = 256;  // [8 waves][<= 2 steps][2] u32 flags, past the step buffers

// (LDS flag of a (wave, step) hand-off: relaxed atomic load, polled with
// s_sleep; the empty asm keeps every later LDS read below the poll -- LDS
// instructions of one wave execute in order, and the loader set the flag only
// after its counted wait saw the DMA data written)
__device__ __forceinline__ void wait_lds_flag(const uint32_t* f) {
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0)
        __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

template <int KT, int VT, int D, bool HM, int NWV, int NLD>
__global__ __launch_bounds__((NWV + NLD) * kWave, 1) void fattn_split_ld_kernel(const SplitArgs a) {
    using C = SplitCfg<KT, VT, D>;
    using P = StepPlan<KT, VT, D, 16>;
    constexpr int NI = P::NIKV + (HM ? P::NIM : 0);  // VMEM instructions per step
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NB = (D + QK - 1) / QK;
    constexpr int NC = D / 16;
    constexpr float kNegInf = -__builtin_inff();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4;
    const int i16 = lane & 15;
    FATTN_SSTAMP_INIT();
    FATTN_SSTAMP(0);

    int chunk, y, iq3;
    tile_coords(a, chunk, y, iq3);
    int qt = 0, hs = 0, ik2 = y, ik3 = iq3;
    if (a.n_qt != 1 || a.n_hsub != 1) {
        qt = y % a.n_qt;
        hs = (y / a.n_qt) % a.n_hsub;
        ik2 = y / (a.n_qt * a.n_hsub);
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;
    const int wl = a.chunk_len / NWV;    // positions per compute wave
    const int spw = a.nbuf;              // steps per compute wave, all resident (planner: nbuf == steps)
    const int mrow0 = qt * a.QPT;
    const int c_hi = min(a.N, (chunk + 1) * a.chunk_len);
    uint32_t* flags = (uint32_t*)(smem + NWV * a.wave_bytes);  // [NWV][spw][2]: K + mask, V (step 0 unused)
    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    rs.m = make_srd(a.mask, HM ? a.m_span : 0);

    if (wave >= NWV) {
        // ---- loader: zero the flags, meet the compute waves once they have
        // issued their step 0, then units u = (s - 1) * NWV + w, s >= 1, dealt
        // round-robin; U units per loader, issued back to back, handed over
        // oldest first (K + mask when all but the unit's V and the later
        // units landed, V when all but the later units)
        const int L = wave - NWV;
        if (L == 0 && lane < NWV * spw * 2) flags[lane] = 0u;
        __syncthreads();
        const int U = (spw - 1) * NWV / NLD;  // (planner: <= 4, a whole number)
        for (int k = 0; k < U; k++) {
            const int u = L + NLD * k, w = u % NWV, s = 1 + u / NWV;
            const int n0 = chunk * a.chunk_len + w * wl + s * kStep;
            issue_step<KT, VT, D, 16, HM>(a, rs, n0, mrow0, smem + w * a.wave_bytes + s * C::stepBytes, lane);
        }
        FATTN_SSTAMP(1);
        for (int k = 0; k < U; k++) {
            const int u = L + NLD * k, w = u % NWV, s = 1 + u / NWV;
            uint32_t* f = flags + (w * spw + s) * 2;
            wait_steps_plus<NI, P::NIV>(U - 1 - k);
            if (lane == 0) __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            wait_steps<NI>(U - 1 - k);
            if (lane == 0) __hip_atomic_store(f + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();  // wg_row_merge's one barrier (the loaders then leave)
        FATTN_SSTAMP_FLUSH();
        return;
    }

    // ---- compute wave: the split kernel's, its later steps refilled by the loaders
    const int m = i16;
    const int mq = div_R(a, m);
    const int mh = hs * a.R + (m - mq * a.R);
    const int iq1 = qt * a.QPT + mq;
    const int iq2 = ik2 * a.rk2 + mh;
    const bool row_ok = (m < a.QPT * a.R) && (iq1 < a.NQ) && (mh < a.rk2);
    const int w_lo = chunk * a.chunk_len + wave * wl;
    const int w_hi = min(c_hi, w_lo + wl);
    const int nsteps = w_hi > w_lo ? (w_hi - w_lo + kStep - 1) / kStep : 0;
    uint8_t* wbuf = smem + wave * a.wave_bytes;
    // Q first, untracked (its wait leaves step 0's DMA in flight), then step 0
    // (fetched whatever the wave's slice: the loaders' counts assume it)
    u32x4 qraw[NB][2];
    {
        const i32x4 qs = make_srd(a.q + (int64_t)iq3 * a.q_nb3, a.q_span);
        const uint32_t qoff = row_ok ? (uint32_t)iq1 * (uint32_t)a.q_nb1 + (uint32_t)iq2 * (uint32_t)a.q_nb2 + 32 * g
                                     : a.q_span;
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const uint32_t qb = (D % QK == 0 || 32 * b + 8 * g < D) ? qoff + 128 * b : a.q_span;
            qraw[b][0] = ld_buf_untracked<kTagQ>(qs, qb);
            qraw[b][1] = ld_buf_untracked<kTagQ>(qs, qb + 16);
        }
    }
    issue_step<KT, VT, D, 16, HM>(a, rs, w_lo, mrow0, wbuf, lane);
    if (a.n_chunks > 1 && lane == 0 && wave == 0) arrival_begin(a, (int64_t)iq3 * gridDim.y + y);
    FATTN_SSTAMP(1);
    __syncthreads();  // every compute wave's step 0 is in the queue: the loaders may issue
    wait_steps<NI>(1);  // Q landed (step 0 may fly on)
#pragma unroll
    for (int b = 0; b < NB; b++) {
        reg_fence<kTagQ>(qraw[b][0]);
        reg_fence<kTagQ>(qraw[b][1]);
    }
    f16x8 qop[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const f32x4 x0 = __builtin_bit_cast(f32x4, qraw[b][0]), x1 = __builtin_bit_cast(f32x4, qraw[b][1]);
        f16x8 h;
        h.s0 = (f16)x0.x; h.s1 = (f16)x0.y; h.s2 = (f16)x0.z; h.s3 = (f16)x0.w;
        h.s4 = (f16)x1.x; h.s5 = (f16)x1.y; h.s6 = (f16)x1.z; h.s7 = (f16)x1.w;
        qop[b] = h;
    }

    float m_run = kNegInf;
    float l_run = 0.0f;
    f32x4 o[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) o[c] = f32x4{0, 0, 0, 0};
    float corr[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) corr[b] = 0.0f;
    for (int s = 0; s < nsteps; s++) {
        const uint32_t* f = flags + (wave * spw + s) * 2;
        if (s == 0) wait_steps_plus<NI, P::NIV>(0);  // own DMA: K + mask landed
        else wait_lds_flag(f);
        if (s < 2) FATTN_SSTAMP(2 + s);
        const int n0 = w_lo + s * kStep;
        int s_opaque = s;
        asm volatile("" : "+s"(s_opaque));
        split_step<KT, VT, D, HM>(a, wbuf + s * C::stepBytes, qop, mq, g, i16, min(kStep, w_hi - n0), s_opaque == 0,
                                  m_run, l_run, o, corr, [&] {
                                      if (s == 0) wait_vmcnt_c<0>();
                                      else wait_lds_flag(f + 1);
                                  });
        if (s < 2) FATTN_SSTAMP(6 + 2 * s);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    FATTN_SSTAMP(10);
    split_epilogue<KT, VT, D, NWV, 2>(a, o, m_run, l_run, corr, wave, lane, qt, hs, ik2, iq3, y, chunk, smem,
                                      a.wave_bytes, true, false);
    FATTN_SSTAMP_FLUSH();
}

// ---------------------------------------------------------------- merge launch
// Second launch of a multi-row split (SplitArgs::merge_launch): one wave per
// (tile, packed row) merges the row's chunk partials (merge_row_parts: the
// fa_reduce LSE merge of src/flash_row_float.h:415-472 in fp32, fixed order)
// and writes the normalised dst row.  The last-arriver form (combine_tile)
// pulls a whole tile's 16 rows x chunks into ONE workgroup (config 5 shard:
// 128 KB, 6.4 us of a 14.7 us launch); here the same bytes spread over
// (tiles x rows) waves, and the kernel boundary replaces drain + counter.
// PLAIN: the partials read with plain loads instead of sc1 (FATTN_OPT_MERGE_PLAIN;
// the kernel boundary already made the split kernel's stores visible).  F16:
// the f16 partials of SplitArgs::part_f16 (merge_row_parts_h, plain loads).
template <int D, int KIT, bool PLAIN = false, bool F16 = false>  // KIT: loads per lane per round trip, >= the tile's chunks / merge_ppr<D>() when possible
__global__ __launch_bounds__(256) void fattn_merge_kernel(const SplitArgs a) {
    const int lane = threadIdx.x & 63;
    const int tm = blockIdx.x * 4 + (threadIdx.x >> 6);  // packed row of the tile
    const int y = blockIdx.y, iq3 = blockIdx.z;
    int qt = 0, hs = 0, ik2 = y;  // the split kernel's tile decode
    if (a.n_qt != 1 || a.n_hsub != 1) {
        qt = y % a.n_qt;
        hs = (y / a.n_qt) % a.n_hsub;
        ik2 = y / (a.n_qt * a.n_hsub);
    }
    if (tm >= tile_rows(a, qt, hs)) return;
    const int64_t slot0 = ((int64_t)iq3 * gridDim.y + y) * a.n_chunks * kRows + tm;  // chunk 0's row tm
    const int rq = div_R(a, tm);
    const int riq1 = qt * a.QPT + rq;
    const int riq2 = ik2 * a.rk2 + hs * a.R + (tm - rq * a.R);
    float* out = a.dst + (((int64_t)iq3 * a.NQ + riq1) * a.H + riq2) * D;
    if constexpr (F16) {
        merge_row_parts_h<D, KIT>((const uint16_t*)a.ws_o + slot0 * D, a.ws_ml + 2 * slot0, a.n_chunks, out, lane,
                                  kRows * D, 2 * kRows);
    } else {
        merge_row_parts<D, KIT, PLAIN ? 0 : kAuxSc1>(a.ws_o + slot0 * D, a.ws_ml + 2 * slot0, a.n_chunks, out, lane,
                                                    kRows * D, 2 * kRows);
    }
}

// ---------------------------------------------------------------- combine
// Log-sum-exp merge of a tile's chunk partials (fa_reduce,
// flash_row_float.h:415-472, in fp32 and parallel), run by the tile's last
// workgroup.  16 thread groups = rv rows x G chunk subsets.  Every thread
// issues its (m, l) load and its first batch of partial loads before one wait
// (one memory round trip when ceil(n_chunks / G) <= CB); the (m, l) pairs
// reduce with VALU segmented reductions (DPP + permlane swaps); the G subsets
// of a row are summed with all LDS reads in flight at once.  Fixed order:
// deterministic.  Partial row rr is packed row row_base + rr of the tile
// (row_base != 0: the multi-query kernel's 16-row subtiles).  Written for
// 256 threads; in a 512-thread workgroup the upper half only joins the
// barriers (its groups, rows and chunks are all out of range).
template <int D, int CB>
__device__ __forceinline__ void combine_tile(const SplitArgs& a, int64_t tile, int qt, int hs, int ik2, int iq3,
                                             int rv, int row_base, uint8_t* smem) {
    constexpr float kNegInf = -__builtin_inff();
    constexpr int EPT = epi_ept<D>();
    // CB = chunks per load batch: with 8 (the split kernel at D = 128) every
    // thread's partials come in ONE memory round trip up to 8 chunks per thread
    // (config 4: 32 chunks x 4 rows); batch slots past the thread's chunks
    // issue no load
    float(*red)[D] = (float(*)[D])smem;                                // [16][D]
    float(*wts)[64] = (float(*)[64])(smem + kRows * D * 4);            // [16][64]
    float* rowL = (float*)(smem + kRows * D * 4 + kRows * 64 * 4);     // [16]
    const int NCH = a.n_chunks;
    const int G = max(1, kRows / max(rv, 1));
    const int grp = threadIdx.x / 16, tj = threadIdx.x % 16, d0 = tj * EPT;
    const int64_t sb = tile * NCH;
    const int r = grp / G, cg = grp % G;
    const bool active = grp < rv * G && d0 < D;  // (D = 80 / 96: threads past the row's dims idle)
    const int kmax = active ? (NCH - cg + G - 1) / G : 0;
    auto fl = [](uint32_t x) { return __builtin_bit_cast(float, x); };
    // partial loads of chunks cg + (k0 + kk) * G through a buffer descriptor
    // over this tile's partials: slots past kmax use an out-of-range offset
    // (zeros, no memory traffic; zero weight too).  Every lane executes every
    // load -- an asm load under a branch would leave a register copy (phi)
    // reading the destination before its wait.
    const uint32_t obytes = (uint32_t)(NCH * kRows * D * 4);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the count)
    const __amdgpu_buffer_rsrc_t osrd = make_rsrc(a.ws_o + sb * kRows * D, obytes);
    auto issue = [&](u32x4 (&v)[CB][EPT / 4], int k0) {
#pragma unroll
        for (int kk = 0; kk < CB; kk++) {
            const int c = cg + (k0 + kk) * G;
            const uint32_t off =
                (k0 + kk < kmax) ? (uint32_t)(((c * kRows + (active ? r : 0)) * D + d0) * 4) : obytes;
#pragma unroll
            for (int e = 0; e < EPT / 4; e++) v[kk][e] = ld_sc1_buf(osrd, off + 16 * e);
        }
    };
    u32x4 v[CB][EPT / 4];
    issue(v, 0);
    // (m, l) of chunk c of row r in thread r * NCP + c (NCP = next power of
    // two >= NCH, <= 64)
    const int NCP = a.ncp;
    const int mr = threadIdx.x / NCP, mc = threadIdx.x % NCP;
    const bool has_ml = mr < rv && mc < NCH;
    const u32x2 mlb = ld_sc1_x2(a.ws_ml + 2 * ((sb + min(mc, NCH - 1)) * kRows + (has_ml ? mr : 0)));
    const float mlm = has_ml ? fl(mlb.x) : kNegInf;
    const float Mr = seg_reduce<true>(mlm, NCP);
    const float wt = (mlm == kNegInf) ? 0.0f : __builtin_amdgcn_exp2f(mlm - Mr);
    const float Lr = seg_reduce<false>(has_ml ? wt * fl(mlb.y) : 0.0f, NCP);
    if (mr < rv) {
        wts[mr][mc] = wt;
        if (mc == 0) rowL[mr] = Lr;
    }
    __syncthreads();

    // fold this thread's chunks
    if (active) {
        float s8[EPT];
#pragma unroll
        for (int e = 0; e < EPT; e++) s8[e] = 0.0f;
        for (int k0 = 0; k0 < kmax; k0 += CB) {
            if (k0 > 0) issue(v, k0);
#pragma unroll
            for (int kk = 0; kk < CB; kk++) {
                const int c = cg + (k0 + kk) * G;
                const float w = (k0 + kk < kmax) ? wts[r][min(c, NCH - 1)] : 0.0f;
#pragma unroll
                for (int e = 0; e < EPT / 4; e++) {
                    s8[4 * e] += w * fl(v[kk][e].x);
                    s8[4 * e + 1] += w * fl(v[kk][e].y);
                    s8[4 * e + 2] += w * fl(v[kk][e].z);
                    s8[4 * e + 3] += w * fl(v[kk][e].w);
                }
            }
        }
#pragma unroll
        for (int e = 0; e < EPT; e += 4) *(f32x4*)&red[grp][d0 + e] = f32x4{s8[e], s8[e + 1], s8[e + 2], s8[e + 3]};
    }
    __syncthreads();

    // sum the G subsets of each row, normalise, store: thread -> (row, 4 dims),
    // all of its 16-B LDS reads issued before any is consumed
    // (a 512-thread workgroup's upper half takes no part)
    for (int t = threadIdx.x; t < rv * (D / 4) && threadIdx.x < kSplitWaves * kWave; t += kSplitWaves * kWave) {
        const int rr = t / (D / 4), dq = (t % (D / 4)) * 4;
        f32x4 part[kRows];
#pragma unroll
        for (int k = 0; k < kRows; k++) part[k] = *(const f32x4*)&red[min(rr * G + k, kRows - 1)][dq];
        f32x4 x = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int k = 0; k < kRows; k++) x += (k < G) ? part[k] : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        const float Lrow = rowL[rr];
        const float inv = 1.0f / Lrow;
        const int pr = row_base + rr;  // packed row within the tile
        const int rq = div_R(a, pr);
        const int riq1 = qt * a.QPT + rq;
        const int riq2 = ik2 * a.rk2 + hs * a.R + (pr - rq * a.R);
        f32x4 o4;
#pragma unroll
        for (int j = 0; j < 4; j++) o4[j] = (Lrow == 0.0f) ? __builtin_nanf("") : x[j] * inv;
        *(f32x4*)(a.dst + (((int64_t)iq3 * a.NQ + riq1) * a.H + riq2) * D + dq) = o4;
    }
}

}  // namespace fattn
