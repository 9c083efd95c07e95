// fattn_bd.h -- batched decode over ggml-quantised KV for gfx950: 64 packed
// (query row x q-head) rows per kv head and workgroup (BASELINE config 5: 64
// query rows x 32 heads over a 4096-position Q8_0 cache, and its per-GPU head
// shards).
//
// Replaces flash_attn_ext_f16<D,Q,C> (src/flash-llama.h:5-438; its 16-row Q
// tiles read K/V once per 16 rows) for the batched-decode shape.  Same math as
// the other kernels (scale * q.k + mask, online softmax, P.V; f16 operands,
// f32 accumulation; chunk partials merged by the fa_reduce LSE rule,
// src/flash_row_float.h:415-472):
//
//  * one workgroup = 8 waves = 64 packed rows of one kv head x one KV chunk;
//    wave w takes row group rg = w & 1 (32 rows: the 32 MFMA columns) and key
//    quarter kq = w >> 1 of every 128-key tile, so each K / V byte of the tile
//    is read from HBM once for all 64 rows;
//  * HBM -> LDS: the tile's raw ggml K and V rows by buffer_load ... lds (1-KiB
//    wave instructions dealt round-robin over the waves), two raw slots: tile
//    s + 2 is issued into tile s's slot once s is dequantised, so two tiles
//    are in flight while the waves compute;
//  * the workgroup dequantises each tile ONCE -- wave w takes half block w of
//    every key, K and V -- into f16 K and V images (the prefill kernel's
//    layouts), h(q * d) with one f16 rounding, exactly the oracle's
//    (src/utils.h:10-11);
//  * "swapped" products on v_mfma_f32_32x32x16_f16: S^T = K.Q^T (K rows from
//    the image by ds_read_b128, all eight read before the chain; Q^T in
//    registers), then O^T = V^T.P^T with P^T the S^T accumulator itself
//    converted to f16 (no lane movement) and V^T gathered by ds_read_b64_tr_b16;
//  * Q: the workgroup's 64 f32 rows staged HBM -> LDS once by DMA (in the K
//    image's place), not re-read per wave;
//  * the mask: each wave's 32 rows x 32 keys per tile by two 1-KiB LDS-DMA
//    instructions into the wave's own 2-KiB slot, one tile ahead (issued once
//    the wave has read the previous tile's values out of the slot).  Not by
//    register loads: a load the compiler does not track, carried around the
//    tile loop, gets copied at the loop's back edge before it has landed;
//  * online softmax in the log2 domain with the deferred max (T13); a wave
//    whose 32 x 32 mask block is -inf everywhere skips the block (exact);
//  * epilogue: every wave parks its rows' (O, m, l) in LDS, then all 512
//    threads merge the four key quarters of a row and store whole rows (no
//    row-per-lane store tail); one chunk: normalised dst rows; several:
//    (O, m, l) partials merged by fattn_bd_merge_kernel in a second launch.
//
// LDS (D = 128, Q8_0): [0, 32 KiB) K image, [32, 64 KiB) V image, then 2 raw
// tiles [K rows | V rows] of 34 KiB, then 8 mask slots of 2 KiB; the epilogue
// reuses it all (148 KiB): one workgroup per CU, two waves per SIMD.
#pragma once

#include "fattn_pf.h"

namespace fattn {

constexpr int kBdWaves = 8;
constexpr int kBdRowsW = 32;                   // packed rows per wave (MFMA columns)
constexpr int kBdRows = 2 * kBdRowsW;          // per workgroup (two row groups)
constexpr int kBdKeys = 128;                   // keys per tile (four 32-key quarters)

template <int KT, int D>
struct BdCfg {
    // f16 K/V (the reference's own cache type): no raw tiles and no
    // dequantisation -- the LDS-DMA writes the images straight from the rows,
    // into a ring of two image pairs (tile s computes while s + 1 lands);
    // head dims 64, 96, 128 (quantised K/V: 128, one ggml block per V image
    // block and wave pair; fattn_bdp.h takes the others)
    static constexpr bool kF16 = KT == FATTN_TYPE_F16;
    static_assert(D == 128 || (kF16 && (D == 64 || D == 96)), "");
    static constexpr int rowB = row_bytes<KT, D>();
    static constexpr int kvRaw = kBdKeys * rowB;                 // raw K (or V) bytes per tile
    static constexpr int rawBytes = (2 * kvRaw + 15) / 16 * 16;  // [K rows | V rows]
    static constexpr int nRaw = kF16 ? 0 : 2;
    static constexpr int img = kBdKeys * D * 2;                  // one f16 image (K, then V)
    static constexpr int nPair = kF16 ? 2 : 1;                   // [K image | V image] pairs
    static constexpr int rawOff = nPair * 2 * img;
    static constexpr int ringEnd = rawOff + nRaw * rawBytes;
    // where Q's f32 rows are staged before the first tile: the K image of the
    // pair tile 0 does not use (f16: pair 1, whose tile is issued once Q is read)
    static constexpr int qOff = kF16 ? 2 * img : 0;
    static constexpr int NI = (kvRaw + 1023) / 1024;             // 1-KiB DMA instructions per K (or V) tile
    // instructions j = 0 .. 2 NI - 1 (K then V) go to wave j % 8
    static constexpr int ni_wave(int w) { return (2 * NI - w + kBdWaves - 1) / kBdWaves; }
    static constexpr int NM = 2;                                 // mask DMA instructions per wave and tile
    // mask slot of wave w: [4 key octets u][32 rows][16 B] (8 keys per 16 B), so
    // the lanes' 8-B reads of one octet are contiguous (conflict-free)
    static constexpr int maskSlot = 2048;
    static constexpr int maskOff = ringEnd;
    static constexpr int maskEnd = maskOff + kBdWaves * maskSlot;
    // epilogue: every wave parks its (O, m, l) rows at the front, [4 key
    // quarters][64 rows][D + 4] f32 then [4][64] (m, l) (BdPark)
    static constexpr int parkBytes = 4 * kBdRows * (D + 4) * 4 + 4 * kBdRows * 8;
    static constexpr int ldsBytes = maskEnd > parkBytes ? maskEnd : parkBytes;
    // Q staged as f32 rows [64][D] in the K image's place before the first tile
    static_assert(kBdRows * D * 4 <= img, "Q rows in the image's place");
    static_assert(ldsBytes <= 163840, "");
};

template <int KT, int D>
__device__ __forceinline__ void bd_issue(const StepSrc& rs, int n0, uint32_t lds, int wave, int lane) {
#ifdef FATTN_MQ_NOMEM
    return;  // diagnostic build only
#endif
    using C = BdCfg<KT, D>;
    for (int j = wave; j < 2 * C::NI; j += kBdWaves) {  // wave-uniform
        const bool is_v = j >= C::NI;
        const int i = is_v ? j - C::NI : j;
        const int byte = i * 1024 + lane * 16;
        // pieces past the tile's bytes stay idle (the instruction still counts)
        if (C::kvRaw % 1024 == 0 || byte < C::kvRaw)
            dma<16, kDecodeNT>(is_v ? rs.v : rs.k, lds + (is_v ? C::kvRaw : 0) + i * 1024,
                               (uint32_t)n0 * C::rowB + byte);
    }
}

// f16 K/V: tile rows -> the pair's f16 images by LDS-DMA, laid out exactly as
// bd_dequant writes them (so the compute reads one layout).  D / 2 1-KiB
// instructions per tile (64 at D = 128), instruction j = wave + 8 i: j < D / 4
// K (dim slice j / 4, keys 32 (j % 4) ..: lane l = key pair half), else V (dim
// block (j - D / 4) / 8, keys 16 ((j - D / 4) % 8) ..: lane l = key quarter chunk).  Each lane's SOURCE
// offset carries the image swizzle (the LDS side of a DMA is lane-linear,
// cdna_hip_programming.md rule 21); rows are addressed by nb1, so llama.cpp's
// [N][Hkv] cache works too.  Keys past N read past the descriptor: zeros.
template <int D>
__device__ __forceinline__ void bd_issue_f16(const StepSrc& rs, uint32_t k_nb1, uint32_t v_nb1, int n0, uint32_t lds,
                                             int wave, int lane) {
#ifdef FATTN_MQ_NOMEM
    return;  // diagnostic build only
#endif
    constexpr int img = kBdKeys * D * 2;
    constexpr int NJK = D / 4;  // K instructions per tile (a multiple of 8)
#pragma unroll
    for (int i = 0; i < D / 16; i++) {
        const int j = wave + kBdWaves * i;  // (i < D / 32: K; wave-uniform)
        if (j < NJK) {
            const int w = j >> 2, kb = j & 3;
            const int key = 32 * kb + (lane >> 1);
            const int q = (lane & 1) ^ ((key >> 3) & 1);
            dma<16, kDecodeNT>(rs.k, lds + w * (kBdKeys * 32) + kb * 1024,
                               (uint32_t)(n0 + key) * k_nb1 + 32 * w + 16 * q);
        } else {
            const int jj = j - NJK, b = jj >> 3, kb = jj & 7;
            const int key = 16 * kb + (lane >> 2);
            const int c = (lane & 3) ^ ((key >> 2) & 3);
            dma<16, kDecodeNT>(rs.v, lds + img + b * (kBdKeys * 64) + kb * 1024,
                               (uint32_t)(n0 + key) * v_nb1 + 64 * b + 16 * c);
        }
    }
}

// counted wait: the awaited group is done once at most the `nraw` raw-tile
// DMA groups and `nmask` mask groups this wave issued after it are still in
// flight (vmcnt counts in issue order)
template <int KT, int D, bool HM, int W>
__device__ __forceinline__ void bd_vm_wait_w(int nraw, int nmask) {
    constexpr int NI = BdCfg<KT, D>::ni_wave(W);
    constexpr int NM = HM ? BdCfg<KT, D>::NM : 0;
    switch (nraw * 4 + nmask) {
        case 0: wait_vmcnt_c<0>(); break;
        case 1: wait_vmcnt_c<NM>(); break;
        case 2: wait_vmcnt_c<2 * NM>(); break;
        case 4: wait_vmcnt_c<NI>(); break;
        case 5: wait_vmcnt_c<NI + NM>(); break;
        case 6: wait_vmcnt_c<NI + 2 * NM>(); break;
        case 8: wait_vmcnt_c<2 * NI>(); break;
        case 9: wait_vmcnt_c<2 * NI + NM>(); break;
        default: wait_vmcnt_c<2 * NI + 2 * NM>(); break;  // 10
    }
}
template <int KT, int D, bool HM>
__device__ __forceinline__ void bd_vm_wait(int wave, int nraw, int nmask) {
    switch (wave) {
        case 0: bd_vm_wait_w<KT, D, HM, 0>(nraw, nmask); break;
        case 1: bd_vm_wait_w<KT, D, HM, 1>(nraw, nmask); break;
        case 2: bd_vm_wait_w<KT, D, HM, 2>(nraw, nmask); break;
        case 3: bd_vm_wait_w<KT, D, HM, 3>(nraw, nmask); break;
        case 4: bd_vm_wait_w<KT, D, HM, 4>(nraw, nmask); break;
        case 5: bd_vm_wait_w<KT, D, HM, 5>(nraw, nmask); break;
        case 6: bd_vm_wait_w<KT, D, HM, 6>(nraw, nmask); break;
        default: bd_vm_wait_w<KT, D, HM, 7>(nraw, nmask); break;
    }
}

// raw tile -> f16 K and V images (the prefill kernel's layouts, 128 keys):
// wave w dequantises half h = w & 1 of block b = w >> 1 -- K dim slice w and V
// dim block b, chunks 2h, 2h + 1 -- of keys lane and 64 + lane; h(q * d), one
// f16 rounding (src/utils.h:10-11).
//   K image [8 dim slices][128 keys][32 B], 16-B halves swapped on keys with bit 3 set
//   V image [4 dim blocks][128 keys][64 B], chunk c of key r at c ^ ((r >> 2) & 3)
template <int KT, int D>
__device__ __forceinline__ void bd_dequant(const uint8_t* raw, uint8_t* k16, uint8_t* v16, int wave, int lane) {
#ifdef FATTN_MQ_NODEQ
    return;  // diagnostic build only
#endif
    using C = BdCfg<KT, D>;
    const int b = wave >> 1, h = wave & 1;
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const int r = 64 * i + lane;
        u32x4 ck[2], cv[2];
        dequant_half<KT, D>(raw, r, b, h, ck);
        dequant_half<KT, D>(raw + C::kvRaw, r, b, h, cv);
        uint8_t* kd = k16 + wave * (kBdKeys * 32) + r * 32;
        const int sk = (r >> 3) & 1;
        *(u32x4*)(kd + sk * 16) = ck[0];
        *(u32x4*)(kd + (sk ^ 1) * 16) = ck[1];
        uint8_t* vd = v16 + b * (kBdKeys * 64) + r * 64;
        const int sv = (r >> 2) & 3;
        *(u32x4*)(vd + ((2 * h) ^ sv) * 16) = cv[0];
        *(u32x4*)(vd + ((2 * h + 1) ^ sv) * 16) = cv[1];
    }
}

// ---- in-kernel chunk merge (SplitArgs::merge_launch == 2; every workgroup of
// the grid co-resident, size_bd checks): the tile's workgroups publish their
// partial rows write-through (sc1) and drain, one lane per workgroup counts on
// the tile's arrival word (the prologue stamped it), and every workgroup then
// merges its share of the tile's rows -- the workgroup whose add came last at
// once, the others once their sc1 poll of the word sees the count complete
// (or the last arriver's re-arm: generation + 1).  MI355X_MICROARCH.md,
// inter-workgroup visibility, first row of the sc1 table: sc1 stores, every
// storing wave drained, then the add; sc1 loads after the poll / add, the other
// waves behind a barrier.  Row r of the tile goes to wave (r mod 8) of chunk
// (r / 8) mod n, one merge_row_parts each: the fa_reduce LSE merge
// (src/flash_row_float.h:415-472) in fp32, fixed order.  This replaces the
// second launch (fattn_bd_merge_kernel) and its kernel boundary.
template <int D>
__device__ __forceinline__ void bd_tile_merge(const SplitArgs& a, uint8_t* smem, const float* acc, float M, float L,
                                              int pr, int c0, bool row_valid, int tid, int lane, int wave, int qt,
                                              int iq3, int y, int chunk) {
    constexpr int kDpt = kBdRows * D / (kBdWaves * kWave);
    const int64_t tile = (int64_t)iq3 * gridDim.y + y;
    const int n = a.n_chunks;
    const int64_t slot = (tile * n + chunk) * kBdRows + pr;
    auto bits = [](float x) { return __builtin_bit_cast(uint32_t, x); };
    if (row_valid) {
        float* po = a.ws_o + slot * D + c0;
#pragma unroll
        for (int e = 0; e < kDpt; e += 4) st_sc1(po + e, u32x4{bits(acc[e]), bits(acc[e + 1]), bits(acc[e + 2]), bits(acc[e + 3])});
        if (c0 == 0) st_sc1_x2(a.ws_ml + 2 * slot, u32x2{bits(M), bits(L)});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
    __syncthreads();
    int* flag = (int*)smem;  // (the park images were read before the barrier)
    if (tid == 0) *flag = tile_arrive_wait(a, tile, n);
    __syncthreads();
    const bool ok = *flag != 0;
    int qt_rows = min(a.QPT, a.NQ - qt * a.QPT) * a.R;
    int ik2 = a.n_qt != 1 ? y / a.n_qt : y;
    for (int r = chunk * kBdWaves + wave; r < qt_rows; r += kBdWaves * n) {  // wave-uniform
        const int64_t s0 = tile * n * kBdRows + r;  // chunk 0's row r
        const int rq = div_R(a, r);
        float* out = a.dst + (((int64_t)iq3 * a.NQ + qt * a.QPT + rq) * a.H + ik2 * a.rk2 + (r - rq * a.R)) * D;
        if (ok) {
            merge_row_parts<D, 8>(a.ws_o + s0 * D, a.ws_ml + 2 * s0, n, out, lane, kBdRows * D, 2 * kBdRows);
        } else if (lane < D / 4) {
            *(f32x4*)(out + 4 * lane) = f32x4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
        }
    }
}

// ---- epilogue of the batched-decode kernels (all memory traffic of the tile
// loop drained): merge the NKG key groups of each row (bd: four key quarters;
// bdp: two key halves).  Every wave that holds a state parks its rows' (O, m,
// l) in LDS (accumulator layout -> [kg][row][D + 4]); then each of the 512
// threads merges 16 dims of one row (fixed order, kg = 0..NKG-1) and stores
// them as 64 contiguous bytes, so every store instruction writes whole rows
// (row-per-lane stores from the accumulator layout issue 32 lines per
// instruction: MI355X_MICROARCH.md, epilogue store tail)
template <int D, int NKG>
struct BdPark {
    static constexpr int stride = D + 4;  // floats (+16 B per row: the accumulator-layout writes are conflict-free)
    static constexpr int ml = NKG * kBdRows * stride * 4;
    static constexpr int bytes = ml + NKG * kBdRows * 8;
};
template <int D, int NKG>
__device__ __forceinline__ void bd_finish(const SplitArgs& a, uint8_t* smem, const f32x16 (&o)[D / 32], float m_run,
                                          f32x2 l2, int kq, int p, int h, bool has_state, int tid, int lane, int wave,
                                          int qt, int ik2, int iq3, int y, int chunk) {
    using PK = BdPark<D, NKG>;
    constexpr int NDB = D / 32;
    constexpr float kNegInf = -__builtin_inff();
    (void)lane; (void)wave;  // (stamps)
    const float l_own = xor32_pair(l2.x + l2.y, false);
    __syncthreads();  // every wave is done with the tiles' LDS
    if (has_state) {
        float* pk = (float*)smem + (kq * kBdRows + p) * PK::stride + 4 * h;
#pragma unroll
        for (int db = 0; db < NDB; db++) {
#pragma unroll
            for (int uu = 0; uu < 4; uu++)
                *(f32x4*)(pk + 32 * db + 8 * uu) = f32x4{o[db][4 * uu], o[db][4 * uu + 1], o[db][4 * uu + 2],
                                                         o[db][4 * uu + 3]};
        }
        if (h == 0) ((f32x2*)(smem + PK::ml))[kq * kBdRows + p] = f32x2{m_run, l_own};
    }
    __syncthreads();
    FATTN_STAMP(12);
    constexpr int kDpt = kBdRows * D / (kBdWaves * kWave);  // dims per thread: 16
    const int pr = tid / (D / kDpt), c0 = (tid % (D / kDpt)) * kDpt;
    const f32x2* pml = (const f32x2*)(smem + PK::ml);
    f32x2 mlk[NKG];
    float M = kNegInf;
#pragma unroll
    for (int k = 0; k < NKG; k++) {
        mlk[k] = pml[k * kBdRows + pr];
        M = fmaxf(M, mlk[k].x);
    }
    float L = 0.0f;
    float acc[kDpt];
#pragma unroll
    for (int e = 0; e < kDpt; e++) acc[e] = 0.0f;
#pragma unroll
    for (int k = 0; k < NKG; k++) {
        const float wk = (mlk[k].x == kNegInf) ? 0.0f : __builtin_amdgcn_exp2f(mlk[k].x - M);
        L += wk * mlk[k].y;
        const float* src = (const float*)smem + (k * kBdRows + pr) * PK::stride + c0;
#pragma unroll
        for (int e = 0; e < kDpt; e += 4) {
            const f32x4 x = *(const f32x4*)(src + e);
            acc[e] += wk * x.x;
            acc[e + 1] += wk * x.y;
            acc[e + 2] += wk * x.z;
            acc[e + 3] += wk * x.w;
        }
    }
    const int rq = div_R(a, pr);
    const int q1 = qt * a.QPT + rq;
    const bool pr_ok = rq < a.QPT && q1 < a.NQ;  // (R not a power of two: rows past QPT * R are none)
    if (a.merge_launch == 2) {
        bd_tile_merge<D>(a, smem, acc, M, L, pr, c0, pr_ok, tid, lane, wave, qt, iq3, y, chunk);
        return;
    }
    if (!pr_ok) return;
    if (a.n_chunks == 1) {
        const int q2 = ik2 * a.rk2 + (pr - rq * a.R);
        float* out = a.dst + (((int64_t)iq3 * a.NQ + q1) * a.H + q2) * D + c0;
        const float inv = 1.0f / L;  // fully masked row -> NaN like the reference
#pragma unroll
        for (int e = 0; e < kDpt; e += 4) {
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; r++) v[r] = L == 0.0f ? __builtin_nanf("") : acc[e + r] * inv;
            *(f32x4*)(out + e) = v;
        }
        return;
    }
    // several chunks: the partial (O, m, l) of packed row pr for
    // fattn_bd_merge_kernel, [tile][chunk][64 rows][D] and [..][64 rows][2] (the
    // kernel boundary orders these stores before the merge's loads)
    const int64_t slot = (((int64_t)iq3 * gridDim.y + y) * a.n_chunks + chunk) * kBdRows + pr;
    if (a.part_f16) {  // (SplitArgs::part_f16: O / l in f16)
        store_part_f16<kDpt>((uint16_t*)a.ws_o + slot * D + c0, acc, L);
    } else {
        float* po = a.ws_o + slot * D + c0;
#pragma unroll
        for (int e = 0; e < kDpt; e += 4) *(f32x4*)(po + e) = f32x4{acc[e], acc[e + 1], acc[e + 2], acc[e + 3]};
    }
    if (c0 == 0) *(f32x2*)(a.ws_ml + 2 * slot) = f32x2{M, L};
#ifdef FATTN_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FATTN_STAMP(13);
#endif
}

template <int KT, int D, bool HM>
__global__ __launch_bounds__(kBdWaves* kWave, 2) void fattn_bd_kernel(const SplitArgs a) {
    using C = BdCfg<KT, D>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NK = D / 16;   // 16-dim k-steps of S^T = K.Q^T
    constexpr int NDB = D / 32;  // 32-dim blocks of O^T (= ggml blocks of a row)
    constexpr float kNegInf = -__builtin_inff();
    constexpr float kDeferLog2 = 8.0f;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rg = wave & 1, kq = wave >> 1;  // row group, key quarter
    const int h = lane >> 5;                  // k-group of the MFMA operands
    const int c32 = lane & 31;                // MFMA column: packed row 32 rg + c32; MFMA row: key 32 kq + c32
    // diagnostic build only (FATTN_STAMPS, tools/stamps_bd.py): 0 start, 1 prologue
    // issued, 2 Q ready, 3 + 2s / 4 + 2s tile s (< 4) landed / computed, 14 / 15
    // tile 0 barriers passed, 11 loop done, 12 states parked, 13 stores drained
    FATTN_STAMP(0);

    // ---- tile decode: y -> (kv head, 64-row query tile); R = rk2
    int chunk, y, iq3;
    tile_coords(a, chunk, y, iq3);
    // in-kernel merge: stamp the tile's arrival word with this launch's epoch
    // (no return; it is older than every counted DMA wait below, which it
    // therefore only joins)
    if (a.merge_launch == 2 && tid == 0) arrival_begin(a, (int64_t)iq3 * gridDim.y + y);
    int qt = 0, ik2 = y, ik3 = iq3;
    if (a.n_qt != 1) {
        qt = y % a.n_qt;
        ik2 = y / a.n_qt;
    }
    if (a.rk3 != 1) ik3 = iq3 / a.rk3;
    const int p = kBdRowsW * rg + c32;  // packed row of the workgroup tile (its q head only
    const int rq0 = div_R(a, p);        // matters to Q and dst, both addressed per row below)
    const int iq1 = qt * a.QPT + rq0;
    const bool row_ok = rq0 < a.QPT && iq1 < a.NQ;  // (R not a power of two: rows past QPT * R are none)

    // ---- this workgroup's KV chunk: 128-key tiles (N % 32 == 0; a tile's
    // quarters past the chunk are idle)
    const int c_lo = chunk * a.chunk_len;
    const int c_hi = min(a.N, c_lo + a.chunk_len);
    const int ntiles = c_hi > c_lo ? (c_hi - c_lo + kBdKeys - 1) / kBdKeys : 0;

    StepSrc rs;
    rs.k = make_srd(a.k + (int64_t)ik2 * a.k_nb2 + (int64_t)ik3 * a.k_nb3, a.k_span);
    rs.v = make_srd(a.v + (int64_t)ik2 * a.v_nb2 + (int64_t)ik3 * a.v_nb3, a.v_span);
    rs.m = make_srd(a.mask, HM ? a.m_span : 0);
    const uint32_t lds0 = lds_addr(smem);
    constexpr int kRing = C::nRaw ? C::nRaw : 1;  // (f16: no raw slots)
    auto raw_lds = [&](int s) { return lds0 + C::rawOff + (s % kRing) * C::rawBytes; };
    auto raw_ptr = [&](int s) { return smem + C::rawOff + (s % kRing) * C::rawBytes; };

    // ---- Q: the workgroup's 64 rows (f32, D per row) copied HBM -> LDS into the
    // V image's place by 1-KiB LDS-DMA instructions (2 rows each, dealt over
    // the waves); each wave then reads its rows' Q^T operands from there.
    // Rows past n_q come from past the descriptor: zeros.
    const i32x4 qs = make_srd(a.q + (int64_t)iq3 * a.q_nb3, a.q_span);
    constexpr int CPR = D / 4;             // 16-B chunks of an f32 Q row
    constexpr int SW = swz_mask(CPR);      // 31, 15, 7 at D = 128, 64, 96
    {
        constexpr int kQInst = kBdRows * D * 4 / 1024;  // 32 at D = 128
        static_assert(kQInst % kBdWaves == 0, "");
#pragma unroll
        for (int i = 0; i < kQInst / kBdWaves; i++) {
            const int j = wave + kBdWaves * i;              // instruction: image chunks 64 j ..
            const int g = kWave * j + lane;
            const int pr = g / CPR, cc = g % CPR;            // packed row, chunk of this lane's 16 B
            const int rq = div_R(a, pr);
            const int q1 = qt * a.QPT + rq, q2 = ik2 * a.rk2 + (pr - rq * a.R);
            // LDS chunk cc of row pr holds the row's chunk cc ^ (pr & SW): the
            // operand reads below (32 rows at once) then spread over the banks
            const uint32_t off = rq < a.QPT && q1 < a.NQ ? (uint32_t)q1 * (uint32_t)a.q_nb1 + (uint32_t)q2 * (uint32_t)a.q_nb2 +
                                                 ((cc ^ (pr & SW)) * 16)
                                           : a.q_span;
            dma<16>(qs, lds0 + C::qOff + j * 1024, off);
        }
    }
    constexpr int kQInstW = kBdRows * D * 4 / 1024 / kBdWaves;  // Q DMA instructions per wave

    // ---- mask: the wave's 32 rows x keys 32 kq .. + 32 of a tile into its slot.
    // DMA instruction i, lane l: octet u = 2 i + (l >> 5) of row l & 31 (rows
    // past n_q come from past the descriptor: zeros, and count as not open)
    const uint32_t mslot = lds0 + C::maskOff + wave * C::maskSlot;
    uint32_t mrow_l;
    {
        mrow_l = row_ok ? (uint32_t)iq1 * (uint32_t)a.m_nb1 : a.m_span;
    }
    auto mask_issue = [&](int s) {
        if constexpr (HM) {
            const uint32_t n2 = (uint32_t)(c_lo + s * kBdKeys + 32 * kq) * 2;
#pragma unroll
            for (int i = 0; i < 2; i++)
                dma<16>(rs.m, mslot + i * 1024, mrow_l == a.m_span ? a.m_span : mrow_l + n2 + 16 * (2 * i + h));
        }
    };

    // per-lane K read base (prefill kernel's): key 32 kq + c32, half h (swapped on keys with bit 3 set)
    const uint32_t kbase = c32 * 32 + ((h ^ ((c32 >> 3) & 1)) * 16);
    // per-lane V^T gather bases (prefill kernel's, 128-key image):
    // 16-lane group (h, dh), lane gi: key 32 kq + 16 q + 8 e + 4 h + gi / 4
    const int gi = lane & 15, dh = (lane >> 4) & 1;
    uint32_t vbase[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const int row = 8 * e + 4 * h + (gi >> 2);
        const int ch = (2 * dh + ((gi & 3) >> 1)) ^ ((h + 2 * e) & 3);
        vbase[e] = C::img + kq * 2048 + row * 64 + ch * 16 + (gi & 1) * 8;
    }

    // ---- this wave's issue order: prologue mask 0 | raw 0 | raw 1, then per
    // tile s, once the images are built and mask s has been read out of the
    // slot: mask s + 1 | raw s + 2.  vmcnt retires in issue order, so each
    // mask goes BEFORE the raw tile that is two ahead: at the top of tile s
    // only mask s and raw s + 1 were issued after raw s, and only raw s + 1
    // after mask s -- tile s computes while tile s + 1 is still in flight.
    // f16: Q | mask 0 | tile 0 into pair 0, then per tile s, right after the
    // barrier that ends tile s - 1's compute (and, for s = 0, the Q reads):
    // tile s + 1 into pair (s + 1) % 2 | mask s + 1
    const uint32_t k_nb1 = (uint32_t)a.k_nb1, v_nb1 = (uint32_t)a.v_nb1;
    auto tile_issue = [&](int s) {
        if constexpr (C::kF16)
            bd_issue_f16<D>(rs, k_nb1, v_nb1, c_lo + s * kBdKeys, lds0 + (s & 1) * 2 * C::img, wave, lane);
        else
            bd_issue<KT, D>(rs, c_lo + s * kBdKeys, raw_lds(s), wave, lane);
    };
    if (ntiles > 0) mask_issue(0);
    if (ntiles > 0) tile_issue(0);
    if (!C::kF16 && ntiles > 1) tile_issue(1);

    float m_run = kNegInf;    // reference max (log2 domain) of this lane's row
    f32x2 l2 = {0.0f, 0.0f};  // this lane's partial row sums (16 of every 32 keys)
    f32x16 o[NDB];
#pragma unroll
    for (int db = 0; db < NDB; db++) {
#pragma unroll
        for (int j = 0; j < 16; j++) o[db][j] = 0.0f;
    }
    const float log2e = 1.4426950408889634f;
    const float scale = a.scale;

    FATTN_STAMP(1);
    // Q landed (mask 0, raw 0 and raw 1 may fly on); every wave's Q pieces in LDS
    {
        const int n1 = (!C::kF16 && ntiles > 1) ? 1 : 0, n0 = ntiles > 0 ? 1 : 0;
        bd_vm_wait<KT, D, HM>(wave, n0 + n1, n0);
    }
    __syncthreads();
    // Q^T operands (B of S^T = K.Q^T): dims 16 kk + 8 h .. + 8 of this lane's
    // row, rounded to f16 like src/utils.h:10
    f16x8 qop[NK];
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
    (void)kQInstW;
    FATTN_STAMP(2);

    for (int s = 0; s < ntiles; s++) {
        // quantised: raw s landed (mask s (s >= 1) and raw s + 1 may fly on);
        // f16: tile s landed (mask s (s >= 1) may fly on; tile s + 1 is
        // issued below)
        bd_vm_wait<KT, D, HM>(wave, (!C::kF16 && s + 1 < ntiles) ? 1 : 0, s > 0 ? 1 : 0);
        if (s < 4) FATTN_STAMP(3 + 2 * s);
        // every wave's pieces of tile s landed; every wave is done with tile
        // s - 1 (quantised: the images are free; f16: pair (s + 1) % 2 is)
        __syncthreads();
        if (s == 0) FATTN_STAMP(14);
        if constexpr (C::kF16) {
            if (s + 1 < ntiles) tile_issue(s + 1);
        } else {
            bd_dequant<KT, D>(raw_ptr(s), smem, smem + C::img, wave, lane);
            // the images are complete and raw s's slot is free
            __syncthreads();
        }
        if (s == 0) FATTN_STAMP(15);
        const int pofs = C::kF16 ? (s & 1) * 2 * C::img : 0;  // this tile's image pair
        // this lane's mask values of tile s (keys 8 u + 4 h + 0..3 of the
        // quarter) out of the wave's slot (mask s landed: only raw s + 1 was
        // issued after it; mask 0 went before raw 0), then mask s + 1 into the
        // slot, then tile s + 2 into raw s's slot (a DMA issue that stalls on
        // a full memory queue overlaps the other waves' compute instead of
        // holding a barrier)
        u32x2 mh[4];
        uint32_t open = 1;  // any key not at -inf (f16 0xFC00)
        if constexpr (HM) {
            // (f16, s = 0: the wait above was vmcnt(0); mask 0 went before tile 0)
            if (s > 0) bd_vm_wait<KT, D, HM>(wave, s + 1 < ntiles ? 1 : 0, 0);
            open = 0;
            const uint8_t* ms = smem + C::maskOff + wave * C::maskSlot + c32 * 16 + h * 8;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                mh[u] = *(const u32x2*)(ms + u * 512);
                open |= (mh[u].x ^ 0xFC00FC00u) | (mh[u].y ^ 0xFC00FC00u);
            }
            if (s + 1 < ntiles) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot has been read
                mask_issue(s + 1);
            }
        }
        if (!C::kF16 && s + 2 < ntiles) tile_issue(s + 2);
#ifdef FATTN_MQ_NOCOMPUTE
        continue;  // diagnostic build only: copies, V dequant and barriers
#endif
        // this wave's 32 keys past the chunk: nothing to compute (N % 32 == 0)
        if (c_lo + s * kBdKeys + 32 * kq >= c_hi) continue;
        // a 32 x 32 block that is -inf for every valid row adds nothing (exact skip)
        if (HM && __builtin_amdgcn_ballot_w64(open != 0 && row_ok) == 0) continue;

        // -- S^T = K.Q^T for this wave's 32 keys: the 8 K operands are read
        // from the image before the MFMA chain (one LDS wait, not eight)
        f16x8 ka[NK];
#pragma unroll
        for (int kk = 0; kk < NK; kk++) ka[kk] = *(const f16x8*)(smem + pofs + kk * (kBdKeys * 32) + kq * 1024 + kbase);
        __builtin_amdgcn_sched_barrier(0);
        f32x16 st;
#pragma unroll
        for (int j = 0; j < 16; j++) st[j] = 0.0f;
#pragma unroll
        for (int kk = 0; kk < NK; kk++) st = mfma32(ka[kk], qop[kk], st);

        // -- u = scale * s + mask (natural units); element j = key 8 (j/4) + 4 h + j%4
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
        // deferred max (cdna_hip_programming.md T13): the reference max moves
        // only when the row's block max passes it by more than 2^8 in p
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

        // -- O^T += V^T.P^T: k-step q covers keys 32 kq + 16 q + 8 (i/4) + 4 h + i%4
        // (i = 0..7); V^T gathered from the image in that order
#pragma unroll
        for (int q = 0; q < 2; q++) {
            typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
            u32x4 va[NDB];
#pragma unroll
            for (int db = 0; db < NDB; db++) {
                const uint32_t off = pofs + db * (kBdKeys * 64) + q * 1024;
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + vbase[0] + off));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + vbase[1] + off));
                const u32x2 a2 = __builtin_bit_cast(u32x2, lo), b2 = __builtin_bit_cast(u32x2, hi);
                va[db] = u32x4{a2.x, a2.y, b2.x, b2.y};
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int db = 0; db < NDB; db++) o[db] = mfma32(__builtin_bit_cast(f16x8, va[db]), pb[q], o[db]);
        }
#ifdef FATTN_STAMPS
        if (s < 4) {
            float z = 0.0f;
            for (int db = 0; db < NDB; db++) z += o[db][0];
            asm volatile("" ::"v"(z));  // the MFMA results are in before the stamp
            FATTN_STAMP(4 + 2 * s);
        }
#endif
    }
    FATTN_STAMP(11);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    bd_finish<D, 4>(a, smem, o, m_run, l2, kq, p, h, true, tid, lane, wave, qt, ik2, iq3, y, chunk);
}

// Second launch of a split batched-decode plan: one wave per (tile, packed
// row) merges the row's chunk partials (merge_row_parts: the fa_reduce LSE
// merge of src/flash_row_float.h:415-472 in fp32, fixed order) and writes the
// normalised dst row.
template <int D, int KIT, bool PLAIN = false, bool F16 = false>  // PLAIN, F16: as fattn_merge_kernel
__global__ __launch_bounds__(256) void fattn_bd_merge_kernel(const SplitArgs a) {
    const int lane = threadIdx.x & 63;
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6);  // packed row of the tile
    const int y = blockIdx.y, iq3 = blockIdx.z;
    int qt = 0, ik2 = y;
    if (a.n_qt != 1) {
        qt = y % a.n_qt;
        ik2 = y / a.n_qt;
    }
    if (p >= min(a.QPT, a.NQ - qt * a.QPT) * a.R) return;
    const int64_t slot0 = ((int64_t)iq3 * gridDim.y + y) * a.n_chunks * kBdRows + p;  // chunk 0's row
    const int rq = div_R(a, p);
    float* out = a.dst + (((int64_t)iq3 * a.NQ + qt * a.QPT + rq) * a.H + ik2 * a.rk2 + (p - rq * a.R)) * D;
    if constexpr (F16) {
        merge_row_parts_h<D, KIT>((const uint16_t*)a.ws_o + slot0 * D, a.ws_ml + 2 * slot0, a.n_chunks, out, lane,
                                  kBdRows * D, 2 * kBdRows);
    } else {
        merge_row_parts<D, KIT, PLAIN ? 0 : kAuxSc1>(a.ws_o + slot0 * D, a.ws_ml + 2 * slot0, a.n_chunks, out, lane,
                                                    kBdRows * D, 2 * kBdRows);
    }
}

}  // namespace fattn
