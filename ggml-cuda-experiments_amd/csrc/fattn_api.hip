// fattn_api.hip -- C-ABI entry points (include/fattn.h) and host-side dispatch.
//
// The reference launches its kernels inline from host code with hard-coded
// template parameters (src/kernel_test.h:157-199, src/flash-matrix.cu:179-255).
// Here the host side validates the ggml views, picks the instantiation
// (head dim x K type x V type x addressing granule), sizes the split-KV grid
// for 256 CUs, and launches on the caller's stream.  Nothing allocates;
// nothing synchronises (graph-capturable).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "fattn_launch.h"

using namespace fattn;

namespace {

constexpr int kCUsDefault = 256;  // MI355X; used when no device can be queried (host-only planning)

// compute units of the current device, queried once per device
int device_cus() {
    static std::atomic<int> cache[kMaxDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
        (void)hipGetLastError();
        return kCUsDefault;
    }
    int n = cache[dev].load(std::memory_order_relaxed);
    if (n > 0) return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        n = kCUsDefault;
    }
    cache[dev].store(n, std::memory_order_relaxed);
    return n;
}

// fattn_set_option overrides (process-wide; atomics, so a planner running on
// another host thread never reads a torn or stale-forever value -- overrides
// are still meant to be set before launches, by tests and benchmarks)
std::atomic<int> g_opt_mq_rpw{0};
std::atomic<int> g_opt_mq_disable{0};
std::atomic<int> g_opt_split_spw{0};
std::atomic<int> g_opt_split_nbuf{0};
std::atomic<int> g_opt_pf{0};  // 0 auto, 1 never, 2 whenever eligible
std::atomic<int> g_opt_pf_stagger{2};
constexpr int kMqMinRowsDefault = 64;
std::atomic<int> g_opt_mq_min_rows{kMqMinRowsDefault};  // multi-query kernel from this many packed rows per kv head (>= 32)
std::atomic<int> g_opt_mq_min_rows_set{0};  // 1: FATTN_OPT_MQ_MIN_ROWS was given explicitly (bypasses the `wide` gate)
std::atomic<int> g_opt_pf_no_skip{0};     // 1: masked prefill without the live-block pre-pass (FATTN_OPT_PF_SKIP)
std::atomic<int> g_opt_split_prio{0};     // split kernel wave priorities (FATTN_OPT_SPLIT_PRIO)
std::atomic<int> g_opt_no_wave_merge{0};  // 1: one-row split tiles merge through LDS + combine_tile as other tiles
std::atomic<int> g_opt_split_waves{0};      // split kernel waves per workgroup (FATTN_OPT_SPLIT_WAVES), 0 = planner
std::atomic<int> g_opt_split_no_skip{0};    // 1: split kernel loads and computes every step (FATTN_OPT_SPLIT_SKIP)
std::atomic<int> g_opt_split_fused_merge{0};  // 1: multi-row split tiles merge in the last-arriving workgroup
std::atomic<int> g_opt_bd{0};               // batched-decode kernel: 0 auto, 1 never, 2 whenever eligible
std::atomic<int> g_opt_bd_xcd{0};           // batched decode, XCD-grouped workgroup order: 0 auto (on), 1 off, 2 on
std::atomic<int> g_opt_gqa_unpack{0};       // GQA one-row decode: 0 auto (packed), 1 packed, 2 one q head per tile
std::atomic<int> g_opt_part_f16{0};         // second-launch merges' partials: 0 auto (f16 where supported), 1 f32, 2 f16
std::atomic<int> g_opt_merge_plain{0};      // second-launch merges: 0 auto (sc1 loads), 1 sc1, 2 plain loads
std::atomic<int> g_opt_split_loaders{0};    // split kernel, one-row tiles: loader waves (FATTN_OPT_SPLIT_LOADERS): 0 auto, 1 off, 2 on
std::atomic<int> g_opt_split_xcd{0};        // split kernel, XCD-grouped workgroup order: 0 auto, 1 off, 2 on
std::atomic<int> g_opt_pf_form{0};          // prefill body at D = 128 over f16 rows: 0 auto (5), 1 the 8-wave form, 4-5 one wave per SIMD (fattn_pf4.h)
std::atomic<int> g_opt_pf_stage{0};         // prefill over Q8_0 / Q4_0: 0 auto (staged to f16), 1 in-kernel dequantisation, 2 staged
std::atomic<int> g_opt_merge_in_kernel{0};  // 1: multi-row chunk partials merge in-kernel when co-resident (FATTN_OPT_MERGE_IN_KERNEL)
// launch epochs for the arrival words (SplitArgs::arrival_stamp); 32 bits, 0 skipped
std::atomic<uint32_t> g_epoch{0};

inline bool is_quant(int t) { return t == FATTN_TYPE_Q8_0 || t == FATTN_TYPE_Q4_0; }
inline int type_size_elem(int t) { return t == FATTN_TYPE_F32 ? 4 : t == FATTN_TYPE_F16 ? 2 : 0; }

// LDS geometry of one instantiation (type-erased for the planner)
struct Geom {
    int step_bytes, vsc_bytes, merge_bytes;
    int wave_bytes(int nbuf) const {
        const int w = (nbuf * step_bytes + vsc_bytes + 15) / 16 * 16;
        return w > merge_bytes ? w : merge_bytes;
    }
    int lds_bytes(int nbuf, int nwv) const { return nwv * wave_bytes(nbuf); }
};

template <int KT, int VT, int D>
Geom geom_of() {
    using C = SplitCfg<KT, VT, D>;
    return Geom{C::stepBytes, C::vscBytes, C::mergeBytes};
}

Geom geom(int kt, int vt, int D) {
    auto pick = [&](auto d) -> Geom {
        constexpr int DD = decltype(d)::value;
        auto with_v = [&](auto k) -> Geom {
            constexpr int KK = decltype(k)::value;
            if (vt == FATTN_TYPE_Q8_0) return geom_of<KK, FATTN_TYPE_Q8_0, DD>();
            if (vt == FATTN_TYPE_Q4_0) return geom_of<KK, FATTN_TYPE_Q4_0, DD>();
            if (vt == VT_F16T) return geom_of<KK, VT_F16T, DD>();
            return geom_of<KK, FATTN_TYPE_F16, DD>();
        };
        if (kt == FATTN_TYPE_Q8_0) return with_v(std::integral_constant<int, FATTN_TYPE_Q8_0>());
        if (kt == FATTN_TYPE_Q4_0) return with_v(std::integral_constant<int, FATTN_TYPE_Q4_0>());
        return with_v(std::integral_constant<int, FATTN_TYPE_F16>());
    };
    switch (D) {
        case 64: return pick(std::integral_constant<int, 64>());
        case 80:  // f16 only (80 is not a whole number of 32-element ggml blocks)
            return vt == VT_F16T ? geom_of<FATTN_TYPE_F16, VT_F16T, 80>() : geom_of<FATTN_TYPE_F16, FATTN_TYPE_F16, 80>();
        case 96: return pick(std::integral_constant<int, 96>());
        case 128: return pick(std::integral_constant<int, 128>());
        default: return pick(std::integral_constant<int, 256>());
    }
}

constexpr int kLdsPerCU = 163840;

// combine_tile limits: one (chunk, row) pair per thread for the (m, l) loads
bool combine_ok(int64_t nch, int rv, int D) {
    (void)D;
    int ncp = 1;
    while (ncp < nch) ncp <<= 1;
    return nch <= 64 && ncp * rv <= 256;
}

// Split-KV sizing.  A workgroup has nwv waves (4, 8 or 16); every wave streams
// `spw` steps of 32 positions.  One-row tiles (decode without GQA packing) with
// at least 6 steps per CU take 8 waves per workgroup, one step in flight each
// (config 3: 8 waves x 2 steps, 11.3 us against 11.8 with 16 waves x 1 step
// all requested at once, 12.4 with both steps of the 8 waves in flight, 12.6
// for the 4-wave form; config 2: 8 x 1); multi-row tiles keep 4 waves up to 8
// steps per CU (config 4: 10.8 vs 11.3 us; config 5's 8-rank shard, 4 heads:
// 11.7 vs 12.0) and take 8 from 16 (round 5, same box: 4-rank shard 14.0 vs
// 15.2 us, 2-rank shard 19.6 vs 19.9; profiles/r05_l).  The grid is sized so that
// all (Y x S x chunks) workgroups are co-resident, limited by LDS (steps in
// flight) and registers.
// f16 chunk partials (SplitArgs::part_f16) for the second-launch merges of the
// split kernel's multi-row tiles and the batched-decode kernels: not at D = 64
// (merge_row_parts_h), not with the in-kernel merges
bool part_f16_ok(int merge_launch, int D) { return merge_launch == 1 && D != 64 && g_opt_part_f16 != 1; }

int size_split(Plan& pl, int kv_chunk, int64_t Y, int64_t S, int64_t N, int64_t NQ) {
    SplitArgs& a = pl.a;
    const Geom G = geom(pl.kt, pl.vt, pl.D);
    const int64_t steps = (N + kStep - 1) / kStep;
    const int wps = (pl.kt == FATTN_TYPE_F16 || pl.gran == 4 || pl.D == 256) ? 2 : 4;  // __launch_bounds__ waves/SIMD
    const int rv_max = std::min<int64_t>(kRows, (int64_t)a.R * std::min<int64_t>(a.QPT, NQ));
    const int64_t total = steps * Y * S;
    int nwv = 4;
    if (pl.gran == 16) {
        if (g_opt_split_waves > 0) {
            nwv = g_opt_split_waves;
        } else if (kv_chunk <= 0) {
            const int64_t per_cu = total / pl.cus;
            nwv = ((rv_max == 1 && per_cu >= 6) || (rv_max > 1 && per_cu >= 16)) ? 8 : 4;
        }
        nwv = std::min(nwv, 4 * wps);
        while (nwv > 4 && G.lds_bytes(1, nwv) > kLdsPerCU) nwv /= 2;
    }
    const int quantum = kStep * nwv;
    // steps in flight per wave: 2 with 4 waves, 1 with more (the measured
    // optima; more bytes requested at once land later for every wave)
    auto inflight = [&](int spw_) {
        int nb = std::min(spw_, nwv == 4 ? 2 : 1);
        while (nb > 1 && G.lds_bytes(nb, nwv) > kLdsPerCU) nb--;
        return nb;
    };
    int spw = 1;
    if (kv_chunk > 0) {
        spw = (int)((kv_chunk + quantum - 1) / quantum);
        for (;;) {  // a forced chunk is a lower bound: grow it until the combine fits
            const int64_t nch = (N + (int64_t)spw * quantum - 1) / ((int64_t)spw * quantum);
            if (nch == 1 || combine_ok(nch, rv_max, pl.D)) break;
            spw++;
        }
    } else {
        spw = (int)std::max<int64_t>(1, (total + (int64_t)pl.cus * nwv / 2) / ((int64_t)pl.cus * nwv));
        spw = (int)std::min<int64_t>(spw, (steps + nwv - 1) / nwv);
        for (;;) {
            const int nb = inflight(spw);
            const int wgs_cu = std::max(1, std::min(4 * wps / nwv, kLdsPerCU / G.lds_bytes(nb, nwv)));
            const int64_t slots = (int64_t)pl.cus * wgs_cu * nwv;
            const int64_t need = (int64_t)((steps + spw - 1) / spw) * Y * S;  // waves at this spw
            const int64_t nch = (N + (int64_t)spw * quantum - 1) / ((int64_t)spw * quantum);
            const bool reducer_ok = nch == 1 || combine_ok(nch, rv_max, pl.D);
            if ((need <= slots && reducer_ok) || nch == 1) break;
            spw++;
        }
        // multi-row tiles with long per-wave slices: twice the chunks (two
        // workgroups per CU); their merge is a second launch from 4 chunks on
        // (config 5 on one GPU: 16 -> 8 steps per wave, 2 -> 4 chunks, 36.5 ->
        // 30.0 us; halving again, 8 chunks: 36.1)
        if (rv_max > 1 && spw >= 8 && !g_opt_split_fused_merge) {
            const int64_t nch2 = (N + (int64_t)(spw / 2) * quantum - 1) / ((int64_t)(spw / 2) * quantum);
            if (combine_ok(nch2, rv_max, pl.D)) spw /= 2;
        }
        if (g_opt_split_spw > 0) {
            spw = (int)std::min<int64_t>(g_opt_split_spw, (steps + nwv - 1) / nwv);
            const int64_t nch = (N + (int64_t)spw * quantum - 1) / ((int64_t)spw * quantum);
            if (nch > 1 && !combine_ok(nch, rv_max, pl.D)) return FATTN_ERR_INVALID_ARG;
        }
    }
    int nbuf = inflight(spw);
    if (g_opt_split_nbuf > 0) {
        nbuf = std::min(spw, (int)g_opt_split_nbuf);
        while (nbuf > 1 && G.lds_bytes(nbuf, nwv) > kLdsPerCU) nbuf--;
    }
    pl.nwv = nwv;
    a.step_skip = g_opt_split_no_skip ? 0 : 1;
    a.nbuf = nbuf;
    a.split_prio = g_opt_split_prio;
    a.wave_bytes = G.wave_bytes(nbuf);
    a.chunk_len = spw * quantum;
    a.n_chunks = (int)((N + a.chunk_len - 1) / a.chunk_len);
    a.ncp = 1;
    while (a.ncp < a.n_chunks) a.ncp <<= 1;
    if (a.n_chunks > 1 && !combine_ok(a.n_chunks, rv_max, pl.D)) return FATTN_ERR_INVALID_ARG;
    // epilogue: one-row tiles with few parts publish per wave and the last wave
    // merges (4-wave form, D = 128); other one-row tiles merge their waves in
    // LDS and publish one row per workgroup; multi-row tiles: combine_tile
    a.wave_merge = 0;
    if (rv_max == 1 && !g_opt_no_wave_merge) {
        if (nwv == 4 && a.n_chunks > 1 && pl.D == 128 && a.n_chunks * nwv <= kWaveMergeParts) a.wave_merge = 1;
        else if (nwv > 4 || a.n_chunks > 1) a.wave_merge = 2;
    }
    // multi-row tiles (and one-row tiles forced onto the same epilogue) with 4
    // or more chunks: the chunk partials merge in a second launch, one wave per
    // (tile, row) instead of one workgroup per tile (config 5 shard: 11.8 vs
    // 14.8 us, config 4: 10.0 vs 10.7; with 2 chunks per tile, config 5 on
    // one GPU, the extra launch costs more than it saves: 36.6 vs 35.6).
    // FATTN_OPT_SPLIT_MERGE = 1: always the last-arriving workgroup (combine_tile).
    // FATTN_OPT_MERGE_IN_KERNEL = 1, with the whole grid co-resident: inside
    // the launch instead, the tile's workgroups waiting for each other and each
    // merging a share of the rows (tile_arrive_wait): measured 0.6-1.1 us
    // slower than the second launch (config 4 10.7-10.9 vs 10.0-10.3 us, the
    // config-5 8-rank shard 12.2 vs 11.6-11.7; profiles/r03_merge)
    pl.lds = G.lds_bytes(nbuf, nwv);
    // loader waves (fattn_split_ld_kernel): one-row tiles on 8 waves whose
    // whole chunk fits the LDS (every step resident), 16-B rows, D = 64 / 128,
    // one K / V type; 4 loader waves issue it all up front
    pl.nld = 0;
    if (g_opt_split_loaders == 2 && pl.gran == 16 && a.wave_merge == 2 && nwv == 8 && spw >= 2 && spw <= 3 &&
        (pl.D == 64 || pl.D == 128) && pl.kt == pl.vt && g_opt_split_nbuf == 0 &&
        G.lds_bytes(spw, nwv) + kSplitLdFlagBytes <= kLdsPerCU) {
        pl.nld = kSplitLoaders;
        a.nbuf = nbuf = spw;
        a.wave_bytes = G.wave_bytes(spw);
        pl.lds = G.lds_bytes(spw, nwv) + kSplitLdFlagBytes;
    }
    const int64_t wgs_cu = std::max(1, std::min(4 * wps / nwv, kLdsPerCU / pl.lds));
    const bool resident = (int64_t)a.n_chunks * Y * S <= (int64_t)pl.cus * wgs_cu;
    a.merge_launch = (a.n_chunks >= 4 && a.wave_merge == 0 && !g_opt_split_fused_merge)
                         ? ((resident && g_opt_merge_in_kernel) ? 2 : 1) : 0;
    // (auto: f16 partials for tiles of 8+ rows -- the 8-rank config-5 shard
    // 11.67 -> 11.50 us; config 4's 4-row tiles were 10.09 -> 10.33 us, so
    // they keep f32; profiles/r06_f)
    a.part_f16 = part_f16_ok(a.merge_launch, pl.D) && (g_opt_part_f16 == 2 || rv_max >= 8) ? 1 : 0;
    pl.grid = dim3(a.n_chunks, (unsigned)Y, (unsigned)S);
    // XCD-grouped order (tile_coords): a tile's chunk workgroups on one XCD.
    // Default for the one-row tiles that merge in-kernel (wg_row_merge):
    // config 3 11.80 vs 11.95 us, six alternating rounds (profiles/r05_a)
    const bool xcd_auto = a.wave_merge == 2 && a.n_chunks > 1;
    a.xcd_group = (g_opt_split_xcd == 2 || (g_opt_split_xcd == 0 && xcd_auto)) && (a.n_chunks * Y * S) % 8 == 0 ? 1 : 0;
    if (a.n_chunks > 1 && a.wave_merge) {
        // [arrival counters][(m, l) per part][row-0 O per part]; parts = waves
        // (wave_merge 1) or workgroups (2)
        const size_t parts = (size_t)S * Y * a.n_chunks * (a.wave_merge == 1 ? nwv : 1);
        pl.cnt_bytes = (size_t)S * Y * kCntStride * sizeof(uint32_t);
        pl.ml_bytes = (parts * 2 * sizeof(float) + 255) / 256 * 256;
        pl.ws_bytes = pl.cnt_bytes + pl.ml_bytes + parts * pl.D * 4;
    } else if (a.n_chunks > 1) {
        // [arrival words, one 256-B line per tile][(m, l) pairs][O partials];
        // no zeroing needed: each launch epoch-stamps its arrival words
        pl.cnt_bytes = (size_t)S * Y * kCntStride * sizeof(uint32_t);
        pl.ml_bytes = ((size_t)S * Y * a.n_chunks * kRows * 2 * sizeof(float) + 255) / 256 * 256;
        pl.ws_bytes = pl.cnt_bytes + pl.ml_bytes + (size_t)S * Y * a.n_chunks * kRows * pl.D * 4;
    } else {
        pl.cnt_bytes = pl.ml_bytes = pl.ws_bytes = 0;
    }
    return FATTN_OK;
}

template <int NW, int RPW>
int mq_lds_bytes_r(int kt, int D) {
    if (kt == FATTN_TYPE_Q8_0)
        return D == 128 ? MQCfg<FATTN_TYPE_Q8_0, 128, NW, RPW>::ldsBytes : MQCfg<FATTN_TYPE_Q8_0, 64, NW, RPW>::ldsBytes;
    return D == 128 ? MQCfg<FATTN_TYPE_Q4_0, 128, NW, RPW>::ldsBytes : MQCfg<FATTN_TYPE_Q4_0, 64, NW, RPW>::ldsBytes;
}
int mq_lds_bytes(int kt, int D, int nw) {
    if (D == 256)  // 64-row workgroups only (256 rows' mask tiles do not fit beside the D = 256 images)
        return kt == FATTN_TYPE_Q8_0 ? MQCfg<FATTN_TYPE_Q8_0, 256, 4, 16>::ldsBytes
                                     : MQCfg<FATTN_TYPE_Q4_0, 256, 4, 16>::ldsBytes;
    return nw == 8 ? mq_lds_bytes_r<8, 32>(kt, D) : mq_lds_bytes_r<4, 16>(kt, D);
}

// Multi-query sizing: 64 or 256 packed rows per workgroup, KV split only when the
// (kv head x query tile x seq) workgroups cannot fill the chip (two per CU at
// 64 rows, one at 256).
int size_mq(Plan& pl, int kv_chunk, int64_t Y, int64_t S, int64_t N) {
    SplitArgs& a = pl.a;
    const int64_t tiles = N / kStep;  // N % kStep == 0 (16-B path)
    const int64_t base = Y * S;
    int64_t nch;
    if (kv_chunk > 0) {
        nch = (N + kv_chunk - 1) / kv_chunk;
    } else {
        const int64_t want = pl.nw == 8 ? pl.cus : 2 * pl.cus;
        nch = (want + base - 1) / base;
        nch = std::min<int64_t>(nch, std::max<int64_t>(1, tiles / 4));  // >= 4 tiles per workgroup
    }
    nch = std::max<int64_t>(1, std::min<int64_t>(nch, tiles));
    int64_t tpc = (tiles + nch - 1) / nch;
    // the chunk partials merge in a second launch (one wave per packed row,
    // at most 64 chunks: one (m, l) pair per lane); FATTN_OPT_SPLIT_MERGE = 1:
    // in the tile's last-arriving workgroup (at most 16 chunks per 16-row subtile)
    const bool fused = g_opt_split_fused_merge != 0;
    // the merge launch's grid.y is Y x the 16-row subtiles per tile: where that
    // would pass the 65535 grid limit the KV sequence is not split (so many
    // tiles fill the chip without it; a requested kv_chunk is a hint)
    if (!fused && Y * (pl.nw == 8 ? 16 : 4) > 65535) tpc = tiles;
    for (;;) {
        nch = (tiles + tpc - 1) / tpc;
        if (nch == 1 || (fused ? combine_ok(nch, kRows, pl.D) : nch <= kWaveMergeParts)) break;
        tpc++;
    }
    a.chunk_len = (int)(tpc * kStep);
    a.n_chunks = (int)nch;
    a.merge_launch = (nch > 1 && !fused) ? 1 : 0;
    // (f16 partials: the config-5 shape at D = 256 55.14 -> 50.82 us, profiles/r06_p)
    a.part_f16 = part_f16_ok(a.merge_launch, pl.D) ? 1 : 0;
    a.ncp = 1;
    while (a.ncp < a.n_chunks) a.ncp <<= 1;
    a.nbuf = 0;
    a.wave_bytes = 0;
    pl.lds = mq_lds_bytes(pl.kt, pl.D, pl.nw);
    pl.grid = dim3(a.n_chunks, (unsigned)Y, (unsigned)S);
    if (a.n_chunks > 1) {
        const size_t subs = (size_t)S * Y * (pl.nw == 8 ? 16 : 4);  // 16-row subtiles per tile
        pl.cnt_bytes = (size_t)S * Y * kCntStride * sizeof(uint32_t);
        pl.ml_bytes = (subs * a.n_chunks * kRows * 2 * sizeof(float) + 255) / 256 * 256;
        pl.ws_bytes = pl.cnt_bytes + pl.ml_bytes + subs * a.n_chunks * kRows * pl.D * 4;
    } else {
        pl.cnt_bytes = pl.ml_bytes = pl.ws_bytes = 0;
    }
    return FATTN_OK;
}

// Batched-decode sizing: one 8-wave workgroup (64 packed rows, 134 KiB of
// LDS) per CU; the KV sequence of each (kv head x 64-row tile) splits into
// chunks of whole 128-key tiles until the workgroups cover the CUs (at most
// 64 chunks: the merge launch takes one (m, l) pair per lane).
int size_bd(Plan& pl, int kv_chunk, int64_t Y, int64_t S, int64_t N) {
    SplitArgs& a = pl.a;
    const int64_t tiles = (N + kBdKeys - 1) / kBdKeys;
    const bool q8 = pl.kt == FATTN_TYPE_Q8_0;
    pl.lds = pl.bdp && pl.D == 64 ? (q8 ? BdpCfg<FATTN_TYPE_Q8_0, 64>::ldsBytes : BdpCfg<FATTN_TYPE_Q4_0, 64>::ldsBytes)
             : pl.bdp && pl.D == 96 ? (q8 ? BdpCfg<FATTN_TYPE_Q8_0, 96>::ldsBytes : BdpCfg<FATTN_TYPE_Q4_0, 96>::ldsBytes)
             : pl.bdp             ? (q8 ? BdpCfg<FATTN_TYPE_Q8_0, 128>::ldsBytes : BdpCfg<FATTN_TYPE_Q4_0, 128>::ldsBytes)
             : pl.kt == FATTN_TYPE_Q8_0 ? BdCfg<FATTN_TYPE_Q8_0, 128>::ldsBytes
             : pl.kt == FATTN_TYPE_Q4_0 ? BdCfg<FATTN_TYPE_Q4_0, 128>::ldsBytes
             : pl.D == 64               ? BdCfg<FATTN_TYPE_F16, 64>::ldsBytes
             : pl.D == 96               ? BdCfg<FATTN_TYPE_F16, 96>::ldsBytes
                                        : BdCfg<FATTN_TYPE_F16, 128>::ldsBytes;
    // workgroups per CU by LDS (the f16 D = 64 form fits two): the KV split
    // fills every resident slot, not one per CU
    const int64_t per_cu = std::max<int64_t>(1, kLdsPerCU / pl.lds);
    int64_t nch;
    if (kv_chunk > 0) {
        nch = (N + kv_chunk - 1) / kv_chunk;
    } else {
        nch = (pl.cus * per_cu + Y * S - 1) / (Y * S);
    }
    nch = std::max<int64_t>(1, std::min<int64_t>(nch, tiles));
    int64_t tpc = (tiles + nch - 1) / nch;
    nch = (tiles + tpc - 1) / tpc;
    while (nch > kWaveMergeParts) {
        tpc++;
        nch = (tiles + tpc - 1) / tpc;
    }
    a.chunk_len = (int)(tpc * kBdKeys);
    a.n_chunks = (int)nch;
    a.ncp = 1;
    while (a.ncp < a.n_chunks) a.ncp <<= 1;
    a.nbuf = 0;
    a.wave_bytes = 0;
    pl.grid = dim3(a.n_chunks, (unsigned)Y, (unsigned)S);
    // XCD-grouped workgroup order (bd_tile_coords): whole tiles per XCD, so a
    // tile's Q rows come from HBM once (config 5: 49.7 vs 53.4 MB per launch,
    // 24.8-24.9 vs 25.1-25.4 us kernel + merge; profiles/r04_f)
    a.xcd_group = g_opt_bd_xcd != 1 && (a.n_chunks * Y * S) % 8 == 0 ? 1 : 0;
    // the chunk partials merge inside the launch (bd_tile_merge: the tile's
    // workgroups wait for each other, so only when the whole grid is
    // co-resident -- one workgroup per CU by LDS) or in a second launch
    const bool resident = nch * Y * S <= (int64_t)pl.cus * per_cu;
    a.merge_launch = nch == 1 ? 0 : (resident && g_opt_merge_in_kernel) ? 2 : 1;
    // (f16 partials: config 5 22.81 -> 20.90 us, its 2-rank shard 19.78 -> 16.16
    // us, same box, profiles/r06_f)
    a.part_f16 = part_f16_ok(a.merge_launch, pl.D) ? 1 : 0;
    if (nch > 1) {
        // [arrival words, in-kernel merge only][(m, l) pairs][O partials]: [S][Y][chunks][64 rows]
        const size_t slots = (size_t)S * Y * nch * kBdRows;
        pl.cnt_bytes = a.merge_launch == 2 ? (size_t)S * Y * kCntStride * sizeof(uint32_t) : 0;
        pl.ml_bytes = (slots * 2 * sizeof(float) + 255) / 256 * 256;
        pl.ws_bytes = pl.cnt_bytes + pl.ml_bytes + slots * pl.D * 4;
    } else {
        pl.cnt_bytes = pl.ml_bytes = pl.ws_bytes = 0;
    }
    return FATTN_OK;
}

// Validate and build the launch plan.  Returns FATTN_OK or an error.
int make_plan(const fattn_params* p, Plan& pl) {
    if (!p || !p->q.data || !p->k.data || !p->v.data || !p->dst) return FATTN_ERR_INVALID_ARG;
    pl.cus = device_cus();
    pl.merge_plain = g_opt_merge_plain == 2;
    const fattn_tensor &q = p->q, &k = p->k, &v = p->v, &mk = p->mask;
    if (q.type != FATTN_TYPE_F32 || q.nb[0] != 4) return FATTN_ERR_UNSUPPORTED_TYPE;
    const int64_t D = q.ne[0];
    if (D != 64 && D != 80 && D != 96 && D != 128 && D != 256) return FATTN_ERR_UNSUPPORTED_HEAD_DIM;
    if (D % QK && (k.type != FATTN_TYPE_F16 || v.type != FATTN_TYPE_F16)) return FATTN_ERR_UNSUPPORTED_HEAD_DIM;
    if (k.ne[0] != D || v.ne[0] != D) return FATTN_ERR_INVALID_ARG;
    const int64_t NQ = q.ne[1], H = q.ne[2], S = q.ne[3];
    const int64_t N = k.ne[1], Hkv = k.ne[2], Skv = k.ne[3];
    if (NQ <= 0 || H <= 0 || S <= 0 || N <= 0 || Hkv <= 0 || Skv <= 0) return FATTN_ERR_INVALID_ARG;
    if (v.ne[1] != N || v.ne[2] != Hkv || v.ne[3] != Skv) return FATTN_ERR_INVALID_ARG;
    if (H % Hkv || S % Skv) return FATTN_ERR_INVALID_ARG;
    if (N > (int64_t)1 << 30 || NQ * H * S > (int64_t)1 << 31) return FATTN_ERR_INVALID_ARG;
    if (k.type != FATTN_TYPE_F16 && !is_quant(k.type)) return FATTN_ERR_UNSUPPORTED_TYPE;
    if (v.type != FATTN_TYPE_F16 && !is_quant(v.type)) return FATTN_ERR_UNSUPPORTED_TYPE;
    // mixed K/V types (llama.cpp's separate cache types, e.g. K Q8_0 with V F16):
    // the split kernel, head dims 64 / 128 / 256
    const bool mixed = k.type != v.type;
    if (mixed && D != 64 && D != 128 && D != 256) return FATTN_ERR_UNSUPPORTED_TYPE;
    if ((uintptr_t)q.data % 16 || q.nb[1] % 16 || q.nb[2] % 16 || q.nb[3] % 16) return FATTN_ERR_ALIGNMENT;

    const size_t rowK = fattn_row_size(k.type, D), rowV = fattn_row_size(v.type, D);
    // K rows must be contiguous (nb[0] = element size / block granular)
    if (k.type == FATTN_TYPE_F16 && k.nb[0] != 2) return FATTN_ERR_BAD_STRIDE;
    if (is_quant(k.type) && k.nb[0] != (int64_t)fattn_row_size(k.type, 32)) return FATTN_ERR_BAD_STRIDE;
    bool v_trans = false;
    if (v.type == FATTN_TYPE_F16 && v.nb[0] != 2) {
        if (v.nb[1] != 2) return FATTN_ERR_BAD_STRIDE;
        v_trans = true;
        if (N % kStep || v.nb[0] % 16 || (uintptr_t)v.data % 16) return FATTN_ERR_BAD_STRIDE;
        // the transposed-V kernels exist for f16 K only (flash_row_float.h's layout)
        if (k.type != FATTN_TYPE_F16) return FATTN_ERR_UNSUPPORTED_TYPE;
    }
    if (is_quant(v.type) && v.nb[0] != (int64_t)fattn_row_size(v.type, 32)) return FATTN_ERR_BAD_STRIDE;
    if (k.nb[1] % 2 || k.nb[2] % 4 || k.nb[3] % 4 || (uintptr_t)k.data % 4) return FATTN_ERR_ALIGNMENT;
    if (v.nb[1] % 2 || v.nb[2] % 4 || v.nb[3] % 4 || (uintptr_t)v.data % 4) return FATTN_ERR_ALIGNMENT;

    const bool has_mask = mk.data != nullptr;
    if (has_mask) {
        // rows padded to an even length (ggml pads to GGML_KQ_MASK_PAD), dword aligned
        if (mk.type != FATTN_TYPE_F16 || mk.ne[0] < N + (N & 1) || mk.ne[1] < NQ) return FATTN_ERR_INVALID_ARG;
        if ((uintptr_t)mk.data % 4 || mk.nb[1] % 4) return FATTN_ERR_ALIGNMENT;
    }

    // fast path: 16-B pieces.  Quantised rows: contiguous per head (a step of
    // 32 rows is one run of bytes); f16 rows: 16-B aligned
    auto rows16 = [&](const fattn_tensor& t, size_t row) {
        const bool base = (uintptr_t)t.data % 16 == 0 && t.nb[2] % 16 == 0 && t.nb[3] % 16 == 0;
        return is_quant(t.type) ? base && t.nb[1] == (int64_t)row && N % kStep == 0 : base && t.nb[1] % 16 == 0;
    };
    bool g16 = rows16(k, rowK);
    if (!v_trans)
        g16 = g16 && rows16(v, rowV);
    else
        g16 = g16 && v.nb[2] % 16 == 0 && v.nb[3] % 16 == 0;
    if (has_mask) g16 = g16 && (uintptr_t)mk.data % 16 == 0 && mk.nb[1] % 16 == 0 && N % kStep == 0;
    if (!g16 && v_trans) return FATTN_ERR_BAD_STRIDE;
    // the dword-granular path needs dword rows (D = 96 Q8_0 / Q4_0 rows are 102 / 54 B:
    // contiguous 16-B-aligned caches only)
    if (!g16 && (k.nb[1] % 4 || (!v_trans && v.nb[1] % 4))) return FATTN_ERR_ALIGNMENT;

    SplitArgs& a = pl.a;
    std::memset(&a, 0, sizeof(a));
    a.q = (const uint8_t*)q.data;
    a.k = (const uint8_t*)k.data;
    a.v = (const uint8_t*)v.data;
    a.mask = (const uint8_t*)mk.data;
    a.dst = p->dst;
    a.q_nb1 = q.nb[1]; a.q_nb2 = q.nb[2]; a.q_nb3 = q.nb[3];
    a.k_nb1 = k.nb[1]; a.k_nb2 = k.nb[2]; a.k_nb3 = k.nb[3];
    a.v_nb0 = v.nb[0]; a.v_nb1 = v.nb[1]; a.v_nb2 = v.nb[2]; a.v_nb3 = v.nb[3];
    a.m_nb1 = has_mask ? mk.nb[1] : 0;
    a.NQ = (int)NQ; a.H = (int)H; a.S = (int)S; a.N = (int)N;
    a.rk2 = (int)(H / Hkv);
    a.rk3 = (int)(S / Skv);
    a.R = std::min(a.rk2, kRows);
    a.QPT = kRows / a.R;
    a.R_inv = 1.0f / (float)a.R;
    a.n_hsub = (a.rk2 + a.R - 1) / a.R;
    a.n_qt = (int)((NQ + a.QPT - 1) / a.QPT);
    a.has_mask = has_mask ? 1 : 0;
    a.scale_log2 = p->scale * 1.4426950408889634f;
    a.scale = p->scale;

    // byte spans addressed through the 32-bit buffer descriptors
    const int64_t k_span = (N - 1) * k.nb[1] + (int64_t)rowK;
    const int64_t v_span = v_trans ? (D - 1) * v.nb[0] + N * 2 : (N - 1) * v.nb[1] + (int64_t)rowV;
    const int64_t m_span = has_mask ? (NQ - 1) * mk.nb[1] + mk.ne[0] * 2 : 0;
    const int64_t q_span = (NQ - 1) * q.nb[1] + (H - 1) * q.nb[2] + D * 4;
    const int64_t span_max = (int64_t)0xFFFFFFF0;
    if (k_span > span_max || v_span > span_max || m_span > span_max || q_span > span_max) return FATTN_ERR_BAD_STRIDE;
    a.k_span = (uint32_t)k_span;
    a.v_span = (uint32_t)v_span;
    a.m_span = (uint32_t)m_span;
    a.q_span = (uint32_t)q_span;

    pl.kt = k.type;
    pl.vt = v_trans ? VT_F16T : v.type;
    pl.D = (int)D;
    pl.gran = g16 ? 16 : 4;
    // many query rows per kv head (batched decode, prefill): the multi-query
    // kernel dequantises each K/V tile once for 64 rows.  Whole head groups
    // are packed (R = rk2, a power of two <= 64).
    // (below 256 packed rows per kv head the split kernel measures faster:
    // config 5, 64 rows, 15.5 vs 37.6 us at 4 heads; FATTN_OPT_MQ_MIN_ROWS)
    // (any rk2 <= 64: with R = rk2 not a power of two a tile packs
    // floor(rows / R) whole head groups and its last rows stay empty)
    const bool heads_ok = NQ * a.rk2 >= 32 && a.rk2 <= 64;
    const bool quant_ok = !g_opt_mq_disable && !mixed && is_quant(k.type) && g16 && heads_ok;
    const bool mq_ok = quant_ok && (D == 64 || D == 128 || D == 256);
    // the same packing for f16 K/V rows (not transposed V): the prefill and
    // batched-decode kernels fill their f16 images by LDS-DMA straight from the rows
    const bool f16_ok = !g_opt_mq_disable && !mixed && k.type == FATTN_TYPE_F16 && !v_trans && g16 && heads_ok;
    // Both 64-row-tile kernels (multi-query, batched decode) need every KV
    // chunk to hold at least two 128-key tiles: a workgroup with one tile is all
    // prologue and epilogue (config-5 shard, 4 heads x 64 rows: split kernel
    // 9.4 + 4.3 us merge, multi-query 11.0 + 4.3, batched decode 10.9 + 4.4)
    const int64_t qpt64 = (quant_ok || f16_ok) ? 64 / a.rk2 : 1;  // query rows per 64-row tile (rk2 <= 64)
    const int64_t y64 = Hkv * ((NQ + qpt64 - 1) / qpt64);
    const bool wide = N * y64 * S >= (int64_t)2 * kBdKeys * pl.cus;
    pl.mq = mq_ok && NQ * a.rk2 >= g_opt_mq_min_rows &&
            (wide || NQ * a.rk2 >= 256 || g_opt_mq_min_rows_set);  // (an explicit threshold wins)
    if (pl.mq) {
        // 256 rows per workgroup once that still gives one workgroup per CU
        const int64_t wg256 = Hkv * S * ((NQ * a.rk2 + 255) / 256);
        pl.nw = g_opt_mq_rpw ? (g_opt_mq_rpw == 32 ? 8 : 4) : wg256 >= pl.cus ? 8 : 4;
        if (D == 256) pl.nw = 4;  // (mq_lds_bytes)
    }
    if (pl.mq) {
        a.R = a.rk2;
        a.QPT = (pl.nw == 8 ? 256 : 64) / a.R;
        a.R_inv = 1.0f / (float)a.R;
        a.n_hsub = 1;
        a.n_qt = (int)((NQ + a.QPT - 1) / a.QPT);
    }
    // prefill shapes: 256-row workgroups over 64-key tiles, no KV split, when
    // the (kv head x query tile x seq) workgroups alone fill the chip
    // (f16 K/V rows, not transposed V: the same kernel, images filled by DMA)
    pl.pf = false;
    // (D = 80: f16 only, its images padded to 96 dims)
    // (D = 80's padding dims are DMA'd from 0x80000000 past the row offset,
    // outside the descriptor only while the spans stay within 2 GiB: fattn_pf.h)
    const bool d80_ok = f16_ok && k_span <= (int64_t)0x80000000 && v_span <= (int64_t)0x80000000;
    if ((quant_ok || f16_ok) && g_opt_pf != 1 && (D == 64 || D == 96 || D == 128 || (D == 80 && d80_ok)) &&
        p->kv_chunk <= 0 &&
        N % kPfKeys == 0 &&
        p->scale > 0.0f && (g_opt_pf == 2 || Hkv * S * ((NQ * a.rk2 + kPfRows - 1) / kPfRows) >= pl.cus)) {
        pl.pf = true;
        pl.mq = false;
        a.R = a.rk2;
        a.R_inv = 1.0f / (float)a.R;
        a.n_hsub = 1;
        a.QPT = kPfRows / a.R;
        a.n_qt = (int)((NQ + a.QPT - 1) / a.QPT);
    }
    // batched decode (config 5: 64 query rows per kv head): 64-row workgroups
    // over 128-key tiles, the KV split over workgroups to fill the chip, the
    // chunk partials merged in a second launch; Q8_0 / Q4_0 and f16 K/V
    // (from 64 rows, when the chunks hold two tiles or more: `wide` above)
    // Q8_0 / Q4_0 take the compute / build-role form (fattn_bdp.h) unless
    // FATTN_OPT_BD = 2 asks for the all-waves form; head dims 64 and 96 (Q8_0 /
    // Q4_0) have the role form only (config-5 shape at D = 64: 19.2 us against
    // 21.3 for the multi-query kernel, profiles/r04_e)
    pl.bd = pl.bdp = false;
    const bool bd_dim = (D == 128 && (mq_ok || f16_ok)) || ((D == 64 || D == 96) && quant_ok && g_opt_bd != 2) ||
                        ((D == 64 || D == 96) && f16_ok);
    if (!pl.pf && g_opt_bd != 1 && bd_dim && N % kStep == 0 &&
        (g_opt_bd >= 2 || (NQ * a.rk2 >= kBdRows && wide))) {
        pl.bd = true;
        pl.bdp = quant_ok && g_opt_bd != 2;
        pl.mq = false;
        a.R = a.rk2;
        a.R_inv = 1.0f / (float)a.R;
        a.n_hsub = 1;
        a.QPT = kBdRows / a.R;
        a.n_qt = (int)((NQ + a.QPT - 1) / a.QPT);
    }
    // GQA decode of one query row (config 4): one q head per split tile instead
    // of the kv head's R heads packed -- one-row tiles, so the in-launch row
    // merge (wg_row_merge) replaces the merge launch; each K/V byte is read
    // by the R tiles of its kv head (the first from HBM, the rest mostly from
    // the caches) (FATTN_OPT_GQA_UNPACK)
    if (!pl.mq && !pl.pf && !pl.bd && NQ == 1 && a.rk2 > 1 && g_opt_gqa_unpack == 2) {
        a.R = 1;
        a.R_inv = 1.0f;
        a.QPT = kRows;
        a.n_hsub = a.rk2;
        a.n_qt = 1;
    }
    const int64_t Y = (int64_t)Hkv * a.n_hsub * a.n_qt;
    if (Y > 65535 || S > 65535) return FATTN_ERR_INVALID_ARG;
    if (pl.bd) return size_bd(pl, p->kv_chunk, Y, S, N);
    if (pl.pf) {
        a.chunk_len = (int)N;
        a.pf_stagger = g_opt_pf_stagger;
        a.n_chunks = 1;
        a.ncp = 1;
        pl.cnt_bytes = pl.ml_bytes = pl.ws_bytes = 0;
        // Q8_0 / Q4_0: staged to f16 rows in the workspace, then the f16 kernel
        // (each K/V tile is otherwise dequantised once per 256-row query tile)
        // (only while the f16 rows stay addressable by the kernels' 32-bit
        // descriptors and tile offsets, N * D * 2 bytes per (kv head, seq): a
        // longer cache keeps the in-kernel dequantisation rather than wrap)
        pl.pf_stage = is_quant(pl.kt) && g_opt_pf_stage != 1 && (int64_t)N * D * 2 <= (int64_t)0xFFFFFFF0;
        if (pl.pf_stage) {
            pl.stage_kt = pl.kt;
            pl.kt = pl.vt = FATTN_TYPE_F16;
            pl.stage_k = (const uint8_t*)k.data;
            pl.stage_v = (const uint8_t*)v.data;
            pl.stage_k_nb2 = k.nb[2]; pl.stage_k_nb3 = k.nb[3];
            pl.stage_v_nb2 = v.nb[2]; pl.stage_v_nb3 = v.nb[3];
            pl.stage_hkv = (int)Hkv;
            pl.stage_skv = (int)Skv;
            pl.stage_bytes = (size_t)Skv * Hkv * N * D * 2;
            // the staged rows: [Skv][Hkv][N][D] f16, contiguous
            a.k_nb1 = a.v_nb1 = D * 2;
            a.k_nb2 = a.v_nb2 = N * D * 2;
            a.k_nb3 = a.v_nb3 = Hkv * N * D * 2;
            a.k_span = a.v_span = (uint32_t)(N * D * 2);
        }
        auto pf_lds = [&](auto d) {
            constexpr int DD = decltype(d)::value;
            return pl.kt == FATTN_TYPE_F16    ? PfCfg<FATTN_TYPE_F16, DD>::ldsBytes
                   : pl.kt == FATTN_TYPE_Q8_0 ? PfCfg<FATTN_TYPE_Q8_0, DD>::ldsBytes
                                              : PfCfg<FATTN_TYPE_Q4_0, DD>::ldsBytes;
        };
        pl.lds = D == 64   ? pf_lds(std::integral_constant<int, 64>())
                 : D == 80 ? PfCfg<FATTN_TYPE_F16, 80>::ldsBytes
                 : D == 96 ? pf_lds(std::integral_constant<int, 96>())
                           : pf_lds(std::integral_constant<int, 128>());
        // f16 rows (native or staged) at D = 128: the one-wave-per-SIMD body
        // (auto: the lean balanced schedule, form 6 -- the balanced form 5 was
        // 0-4 % faster than the 8-wave body on f16 rows, 12-21 % on staged Q8_0
        // with the zero mask and 1-3 % faster than the pipelined form 4
        // (profiles/r05_h, r05_p); the lean form's chains started from -m / c
        // take 1.5 % (f16) to 3.6 % (Q8_0 zero mask) off it, profiles/r06_c;
        // form 1 keeps the 8-wave body)
        const int form = g_opt_pf_form == 0 ? 6 : (int)g_opt_pf_form;
        pl.pf4 = pl.kt == FATTN_TYPE_F16 && D == 128 && form >= 4;
        pl.pf4_sched = form - 2;  // 4: pipelined (SCHED 2), 5: balanced (SCHED 3), 6: lean (SCHED 4)
        if (pl.pf4) pl.lds = Pf4Cfg<128>::ldsBytes;
        pl.grid = dim3(1, (unsigned)Y, (unsigned)S);
        // workspace: live-block flags, n_qt x N/64 bytes (masked prefill).  They
        // share the front of the workspace with the split-KV arrival words; a
        // later decode supersedes whatever the flags left there (its epoch
        // stamp, arrival_begin in fattn_split.h), so nothing is re-zeroed.
        pl.pf_flags = has_mask && !g_opt_pf_no_skip;
        if (pl.pf_flags) pl.cnt_bytes = ((size_t)a.n_qt * (N / kPfKeys) + 255) / 256 * 256;
        pl.ws_bytes = pl.cnt_bytes;
        if (pl.pf_stage) {
            pl.stage_off = pl.cnt_bytes;
            pl.ws_bytes = pl.stage_off + 2 * pl.stage_bytes;
        }
        return FATTN_OK;
    }
    pl.nwv = 4;
    return pl.mq ? size_mq(pl, p->kv_chunk, Y, S, N) : size_split(pl, p->kv_chunk, Y, S, N, NQ);
}

}  // namespace

extern "C" {

#ifdef FATTN_STAMPS
// diagnostic build only: where the split kernel writes its phase stamps
int fattn_debug_set_stamps_d64(void*);
int fattn_debug_set_stamps_d80(void*);
int fattn_debug_set_stamps_d96(void*);
int fattn_debug_set_stamps_d128(void*);
int fattn_debug_set_stamps_d256(void*);
int fattn_debug_set_stamps(void* dev_ptr) {
    return fattn_debug_set_stamps_d64(dev_ptr) | fattn_debug_set_stamps_d80(dev_ptr) | fattn_debug_set_stamps_d96(dev_ptr) |
           fattn_debug_set_stamps_d128(dev_ptr) | fattn_debug_set_stamps_d256(dev_ptr);
}
// grid of the plan: out[0..2] = chunks, Y, S
int fattn_debug_plan(const fattn_params* p, int* out) {
    Plan pl;
    const int rc = make_plan(p, pl);
    if (rc) return rc;
    out[0] = (int)pl.grid.x;
    out[1] = (int)pl.grid.y;
    out[2] = (int)pl.grid.z;
    return 0;
}
#endif

int fattn_set_option(int option, int value) {
    switch (option) {
        case FATTN_OPT_MQ_ROWS_PER_WAVE:
            if (value != 0 && value != 16 && value != 32) return FATTN_ERR_INVALID_ARG;
            g_opt_mq_rpw = value;
            return FATTN_OK;
        case FATTN_OPT_MQ_DISABLE:
            g_opt_mq_disable = value ? 1 : 0;
            return FATTN_OK;
        case FATTN_OPT_PF:
            if (value < 0 || value > 2) return FATTN_ERR_INVALID_ARG;
            g_opt_pf = value;
            return FATTN_OK;
        case FATTN_OPT_PF_STAGGER:
            if (value < 0 || value > 7 || (value & 1)) return FATTN_ERR_INVALID_ARG;  // (bit 0: removed)
            g_opt_pf_stagger = value;
            return FATTN_OK;
        case FATTN_OPT_MQ_MIN_ROWS:
            if (value != 0 && value < 32) return FATTN_ERR_INVALID_ARG;
            g_opt_mq_min_rows = value ? value : kMqMinRowsDefault;
            g_opt_mq_min_rows_set = value ? 1 : 0;
            return FATTN_OK;
        case FATTN_OPT_PF_SKIP:
            if (value < 0 || value > 1) return FATTN_ERR_INVALID_ARG;
            g_opt_pf_no_skip = value;
            return FATTN_OK;
        case FATTN_OPT_SPLIT_PRIO:
            if (value < 0 || value > 2) return FATTN_ERR_INVALID_ARG;
            g_opt_split_prio = value;
            return FATTN_OK;
        case FATTN_OPT_SPLIT_WAVE_MERGE:
            if (value < 0 || value > 1) return FATTN_ERR_INVALID_ARG;
            g_opt_no_wave_merge = value;
            return FATTN_OK;
        case FATTN_OPT_SPLIT_MERGE:
            if (value < 0 || value > 1) return FATTN_ERR_INVALID_ARG;
            g_opt_split_fused_merge = value;
            return FATTN_OK;
        case FATTN_OPT_SPLIT_STEPS:
            if (value < 0 || value > 64) return FATTN_ERR_INVALID_ARG;
            g_opt_split_spw = value;
            return FATTN_OK;
        case FATTN_OPT_SPLIT_SKIP:
            if (value < 0 || value > 1) return FATTN_ERR_INVALID_ARG;
            g_opt_split_no_skip = value;
            return FATTN_OK;
        case FATTN_OPT_SPLIT_WAVES:
            if (value != 0 && value != 4 && value != 8 && value != 16) return FATTN_ERR_INVALID_ARG;
            g_opt_split_waves = value;
            return FATTN_OK;
        case FATTN_OPT_BD:
            if (value < 0 || value > 3) return FATTN_ERR_INVALID_ARG;
            g_opt_bd = value;
            return FATTN_OK;
        case FATTN_OPT_MERGE_IN_KERNEL:
            if (value < 0 || value > 1) return FATTN_ERR_INVALID_ARG;
            g_opt_merge_in_kernel = value;
            return FATTN_OK;
        case FATTN_OPT_BD_XCD:
            if (value < 0 || value > 2) return FATTN_ERR_INVALID_ARG;
            g_opt_bd_xcd = value;
            return FATTN_OK;
        case FATTN_OPT_GQA_UNPACK:
            if (value < 0 || value > 2) return FATTN_ERR_INVALID_ARG;
            g_opt_gqa_unpack = value;
            return FATTN_OK;
        case FATTN_OPT_PART_F16:
            if (value < 0 || value > 2) return FATTN_ERR_INVALID_ARG;
            g_opt_part_f16 = value;
            return FATTN_OK;
        case FATTN_OPT_MERGE_PLAIN:
            if (value < 0 || value > 2) return FATTN_ERR_INVALID_ARG;
            g_opt_merge_plain = value;
            return FATTN_OK;
        case FATTN_OPT_SPLIT_LOADERS:
            if (value < 0 || value > 2) return FATTN_ERR_INVALID_ARG;
            g_opt_split_loaders = value;
            return FATTN_OK;
        case FATTN_OPT_SPLIT_XCD:
            if (value < 0 || value > 2) return FATTN_ERR_INVALID_ARG;
            g_opt_split_xcd = value;
            return FATTN_OK;
        case FATTN_OPT_PF_FORM:
            // 2, 3: round 5's unpipelined one-wave-per-SIMD forms, removed (slower)
            if (value < 0 || value > 6 || value == 2 || value == 3) return FATTN_ERR_INVALID_ARG;
            g_opt_pf_form = value;
            return FATTN_OK;
        case FATTN_OPT_PF_STAGE:
            if (value < 0 || value > 2) return FATTN_ERR_INVALID_ARG;
            g_opt_pf_stage = value;
            return FATTN_OK;
        case FATTN_OPT_SPLIT_INFLIGHT:
            if (value < 0 || value > 4) return FATTN_ERR_INVALID_ARG;
            g_opt_split_nbuf = value;
            return FATTN_OK;
        default: return FATTN_ERR_INVALID_ARG;
    }
}

const char* fattn_version(void) { return "fattn-gfx950 0.1"; }

const char* fattn_strerror(int s) {
    switch (s) {
        case FATTN_OK: return "ok";
        case FATTN_ERR_INVALID_ARG: return "invalid argument";
        case FATTN_ERR_UNSUPPORTED_TYPE: return "unsupported tensor type";
        case FATTN_ERR_UNSUPPORTED_HEAD_DIM: return "unsupported head dim (64, 80 (f16 K/V), 96, 128, 256)";
        case FATTN_ERR_BAD_STRIDE: return "unsupported strides / layout";
        case FATTN_ERR_WORKSPACE: return "workspace too small";
        case FATTN_ERR_LAUNCH: return "HIP launch failed";
        case FATTN_ERR_ALIGNMENT: return "misaligned pointer or stride";
        default: return "unknown error";
    }
}

size_t fattn_row_size(int type, int64_t k) {
    switch (type) {
        case FATTN_TYPE_F32: return (size_t)k * 4;
        case FATTN_TYPE_F16: return (size_t)k * 2;
        case FATTN_TYPE_Q8_0: return k % QK ? 0 : (size_t)(k / QK) * kQ8Bytes;
        case FATTN_TYPE_Q4_0: return k % QK ? 0 : (size_t)(k / QK) * kQ4Bytes;
        default: return 0;
    }
}

int fattn_workspace_init(void* workspace, size_t workspace_bytes, void* stream) {
    if (!workspace && workspace_bytes) return FATTN_ERR_INVALID_ARG;
    if (!workspace_bytes) return FATTN_OK;
    return hipMemsetAsync(workspace, 0, workspace_bytes, (hipStream_t)stream) == hipSuccess ? FATTN_OK
                                                                                          : FATTN_ERR_LAUNCH;
}

size_t fattn_workspace_size(const fattn_params* p) {
    Plan pl;
    if (make_plan(p, pl) != FATTN_OK) return 0;
    return pl.ws_bytes;
}

int fattn_describe(const fattn_params* p, char* out, size_t cap) {
    Plan pl;
    const int rc = make_plan(p, pl);
    if (rc != FATTN_OK) return rc;
    auto tn = [](int t) {
        return t == FATTN_TYPE_Q8_0 ? "q8_0" : t == FATTN_TYPE_Q4_0 ? "q4_0" : t == VT_F16T ? "f16T" : "f16";
    };
    char kern[160];
    const char* hm = pl.a.has_mask ? "mask" : "nomask";
    if (pl.pf)  // (the pre-pass: one launch, pf_prepass_kernel)
        std::snprintf(kern, sizeof kern, "%s%s%s%s%s%s<%s,D%d,%s>", (pl.pf_stage || pl.pf_flags) ? "pf_prepass[" : "",
                      pl.pf_stage ? (pl.stage_kt == FATTN_TYPE_Q8_0 ? "kv_stage_f16<q8_0>" : "kv_stage_f16<q4_0>") : "",
                      pl.pf_stage && pl.pf_flags ? " + " : "", pl.pf_flags ? "pf_mask_flags" : "",
                      (pl.pf_stage || pl.pf_flags) ? "] + " : "",
                      pl.pf4 ? (pl.pf4_sched == 4 ? "fattn_pf4_kernel(lean)" : pl.pf4_sched == 3 ? "fattn_pf4_kernel(balanced)" : "fattn_pf4_kernel(pipelined)") : "fattn_pf_kernel",
                      tn(pl.kt), pl.D, hm);
    else if (pl.bd)
        std::snprintf(kern, sizeof kern, "%s<%s,D%d,%s>%s%s", pl.bdp ? "fattn_bdp_kernel" : "fattn_bd_kernel", tn(pl.kt), pl.D,
                      hm, pl.a.xcd_group ? " (xcd order)" : "",
                      pl.a.merge_launch == 1 ? (pl.a.part_f16 ? " + fattn_bd_merge_kernel(f16 partials)" : pl.merge_plain ? " + fattn_bd_merge_kernel(plain)" : " + fattn_bd_merge_kernel") : pl.a.merge_launch == 2 ? " (in-kernel merge)" : "");
    else if (pl.mq)
        std::snprintf(kern, sizeof kern, "fattn_mq_kernel<%s,D%d,%dwaves,%s>%s", tn(pl.kt), pl.D, pl.nw, hm,
                      pl.a.merge_launch ? (pl.a.part_f16 ? " + fattn_mq_merge_kernel(f16 partials)" : " + fattn_mq_merge_kernel") : "");
    else
        std::snprintf(kern, sizeof kern, "%s<%s,%s,D%d,gran%d,%s,%dwaves%s>%s%s",
                      pl.nld ? "fattn_split_ld_kernel" : "fattn_split_kernel", tn(pl.kt), tn(pl.vt),
                      pl.D, pl.gran, hm, pl.nwv, pl.nld ? "+4loaders" : "", pl.a.xcd_group ? " (xcd order)" : "",
                      pl.a.merge_launch == 1 ? (pl.a.part_f16 ? " + fattn_merge_kernel(f16 partials)" : pl.merge_plain ? " + fattn_merge_kernel(plain)" : " + fattn_merge_kernel") : pl.a.merge_launch == 2 ? " (in-kernel merge)" : "");
    const int n = std::snprintf(out, cap, "%s grid(%u,%u,%u) lds %d chunk %d steps/slots %d ws %zu", kern, pl.grid.x,
                                pl.grid.y, pl.grid.z, pl.lds, pl.a.chunk_len, pl.a.nbuf, pl.ws_bytes);
    return n < 0 || (size_t)n >= cap ? FATTN_ERR_INVALID_ARG : FATTN_OK;
}

int fattn_ext(const fattn_params* p, void* stream) { return fattn_ext_events(p, stream, nullptr, nullptr); }

int fattn_ext_events(const fattn_params* p, void* stream, void* ev_begin, void* ev_end) {
    Plan pl;
    const int rc = make_plan(p, pl);
    if (rc != FATTN_OK) return rc;
    if (pl.ws_bytes) {
        if (!p->workspace || p->workspace_bytes < pl.ws_bytes || (uintptr_t)p->workspace % 16) return FATTN_ERR_WORKSPACE;
        uint8_t* w = (uint8_t*)p->workspace;
        pl.a.ws_cnt = (uint32_t*)w;
        uint32_t e = g_epoch.fetch_add(1, std::memory_order_relaxed) + 1;
        if (e == 0) e = g_epoch.fetch_add(1, std::memory_order_relaxed) + 1;
        pl.a.arrival_stamp = kArrivalTag | (uint64_t)e << kArrivalEpochShift;
        pl.a.ws_ml = (float*)(w + pl.cnt_bytes);
        pl.a.ws_o = (float*)(w + pl.cnt_bytes + pl.ml_bytes);  // (prefill pre-pass: the f16 rows)
        if (pl.pf && pl.pf_flags) pl.a.pf_flags = w;
        if (pl.pf_stage) {
            pl.a.k = w + pl.stage_off;
            pl.a.v = w + pl.stage_off + pl.stage_bytes;
        }
    }
    hipStream_t st = (hipStream_t)stream;
    Events ev;
    ev.begin = (hipEvent_t)ev_begin;
    ev.end = (hipEvent_t)ev_end;
    switch (pl.D) {
        case 64: return launch_types<64>(pl, st, ev);
        case 80: return launch_types<80>(pl, st, ev);
        case 96: return launch_types<96>(pl, st, ev);
        case 128: return launch_types<128>(pl, st, ev);
        default: return launch_types<256>(pl, st, ev);
    }
}

int fattn_ext_f16_launch(const void* q, const void* k, const void* v, const void* mask, float* dst, float scale,
                         int ne00, int ne01, int ne02, int ne03, int ne10, int ne11, int ne12, int ne13, int ne31,
                         int nb31, int nb01, int nb02, int nb03, int nb11, int nb12, int nb13, int ne0, int ne1,
                         int ne2, int ne3, int k_type, int v_type, void* workspace, size_t workspace_bytes,
                         void* stream) {
    // flash-llama.h:120-125: V shares K's shape and strides -- so one row size:
    // mixed K / V types need the struct form (fattn_ext) with V's own strides
    (void)ne0; (void)ne1; (void)ne2; (void)ne3;
    if (k_type != v_type) return FATTN_ERR_INVALID_ARG;
    fattn_params p;
    std::memset(&p, 0, sizeof(p));
    p.q = {q, FATTN_TYPE_F32, 0, {ne00, ne01, ne02, ne03}, {4, nb01, nb02, nb03}};
    const int64_t kb0 = k_type == FATTN_TYPE_F16 ? 2 : (int64_t)fattn_row_size(k_type, 32);
    const int64_t vb0 = v_type == FATTN_TYPE_F16 ? 2 : (int64_t)fattn_row_size(v_type, 32);
    p.k = {k, k_type, 0, {ne10, ne11, ne12, ne13}, {kb0, nb11, nb12, nb13}};
    p.v = {v, v_type, 0, {ne10, ne11, ne12, ne13}, {vb0, nb11, nb12, nb13}};
    // mask rows hold nb31 / 2 halves: ggml pads them (GGML_KQ_MASK_PAD) past ne11,
    // which an odd ne11 needs (the kernels read rows in dword pieces)
    if (mask)
        p.mask = {mask, FATTN_TYPE_F16, 0, {nb31 / 2, ne31, 1, 1}, {2, nb31, (int64_t)nb31 * ne31, (int64_t)nb31 * ne31}};
    p.dst = dst;
    p.scale = scale;
    p.workspace = workspace;
    p.workspace_bytes = workspace_bytes;
    return fattn_ext(&p, stream);
}

static void fill_row_params(fattn_params& p, const float* query, const void* key, const void* value, const void* mask,
                            float* qkv, int head_dim, int kv_size, int num_heads, float scale, int head_stride,
                            int r_kv_heads) {
    std::memset(&p, 0, sizeof(p));
    const int64_t D = head_dim, N = kv_size, H = num_heads, Hkv = num_heads / r_kv_heads;
    p.q = {query, FATTN_TYPE_F32, 0, {D, 1, H, 1}, {4, D * H * 4, D * 4, D * H * 4}};
    // key [Hkv][N][D] f16 (flash_row_float.h:19,58): kv head offset head_stride elements
    p.k = {key, FATTN_TYPE_F16, 0, {D, N, Hkv, 1}, {2, D * 2, (int64_t)head_stride * 2, (int64_t)head_stride * 2 * Hkv}};
    // value f16 transposed [Hkv][D][N] (flash_row_float.h:177)
    p.v = {value, FATTN_TYPE_F16, 0, {D, N, Hkv, 1}, {N * 2, 2, (int64_t)head_stride * 2, (int64_t)head_stride * 2 * Hkv}};
    if (mask) p.mask = {mask, FATTN_TYPE_F16, 0, {N, 1, 1, 1}, {2, N * 2, N * 2, N * 2}};
    p.dst = qkv;  // [1][H][D] == qkv[h*D + d] (flash_row_float.h:469)
    p.scale = scale;
}

// The ABI (kernel_test.h:155's inline sizing) does not name r_kv_heads, and
// the plan -- rows per tile, chunks, merge layout -- depends on it: size for
// the largest plan over every r that divides num_heads, with and without a mask.
size_t fattn_row_workspace_size(int head_dim, int kv_size, int num_heads) {
    if (num_heads <= 0) return 0;
    size_t best = 0;
    static const float dummy_f[4] = {0, 0, 0, 0};
    for (int r = 1; r <= num_heads; r++) {
        if (num_heads % r) continue;
        for (int m = 0; m < 2; m++) {
            fattn_params p;
            fill_row_params(p, dummy_f, dummy_f, dummy_f, m ? dummy_f : nullptr, (float*)dummy_f, head_dim, kv_size,
                            num_heads, 1.0f, head_dim * kv_size, r);
            p.q.data = (const void*)(uintptr_t)16;  // alignment-only placeholders
            p.k.data = p.v.data = (const void*)(uintptr_t)16;
            if (m) p.mask.data = (const void*)(uintptr_t)16;
            Plan pl;
            if (make_plan(&p, pl) == FATTN_OK) best = std::max(best, pl.ws_bytes);
        }
    }
    return best;
}

int fattn_row(const float* query, const void* key, const void* value, const void* mask, void* tmp, size_t tmp_bytes,
              float* qkv, int head_dim, int kv_size, int num_heads, float scale, int head_stride, int r_kv_heads,
              void* stream) {
    if (r_kv_heads <= 0 || num_heads % r_kv_heads) return FATTN_ERR_INVALID_ARG;
    fattn_params p;
    fill_row_params(p, query, key, value, mask, qkv, head_dim, kv_size, num_heads, scale, head_stride, r_kv_heads);
    p.workspace = tmp;
    p.workspace_bytes = tmp_bytes;
    return fattn_ext(&p, stream);
}

int fattn_dequantize(int type, const void* src, float* dst, int64_t k, int64_t n_rows, void* stream) {
    if (!src || !dst || k <= 0 || n_rows <= 0) return FATTN_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    const int64_t n = k * n_rows;
    if (type == FATTN_TYPE_F16) {
        hipLaunchKernelGGL(dequant_f16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                           (const uint16_t*)src, dst, n);
    } else if (type == FATTN_TYPE_Q8_0 || type == FATTN_TYPE_Q4_0) {
        if (k % QK) return FATTN_ERR_INVALID_ARG;
        const int64_t nb = n / QK;
        if (type == FATTN_TYPE_Q8_0)
            hipLaunchKernelGGL(dequant_q8_0_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, st,
                               (const uint8_t*)src, dst, nb);
        else
            hipLaunchKernelGGL(dequant_q4_0_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, st,
                               (const uint8_t*)src, dst, nb);
    } else {
        return FATTN_ERR_UNSUPPORTED_TYPE;
    }
    return hipGetLastError() == hipSuccess ? FATTN_OK : FATTN_ERR_LAUNCH;
}

int fattn_quantize(int type, const float* src, void* dst, int64_t k, int64_t n_rows, void* stream) {
    if (!src || !dst || k <= 0 || n_rows <= 0) return FATTN_ERR_INVALID_ARG;
    if (k % QK) return FATTN_ERR_INVALID_ARG;
    if ((uintptr_t)src % 16) return FATTN_ERR_ALIGNMENT;
    hipStream_t st = (hipStream_t)stream;
    const int64_t nb = k * n_rows / QK;
    if (type == FATTN_TYPE_Q8_0)
        hipLaunchKernelGGL(quant_kernel<FATTN_TYPE_Q8_0>, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, st, src,
                           (uint8_t*)dst, nb);
    else if (type == FATTN_TYPE_Q4_0)
        hipLaunchKernelGGL(quant_kernel<FATTN_TYPE_Q4_0>, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, st, src,
                           (uint8_t*)dst, nb);
    else
        return FATTN_ERR_UNSUPPORTED_TYPE;
    return hipGetLastError() == hipSuccess ? FATTN_OK : FATTN_ERR_LAUNCH;
}

int fattn_cpy(const fattn_tensor* src, const fattn_tensor* dst, void* stream) {
    if (!src || !dst || !src->data || !dst->data) return FATTN_ERR_INVALID_ARG;
    if (src->type != FATTN_TYPE_F32 || src->nb[0] != 4) return FATTN_ERR_UNSUPPORTED_TYPE;
    const int t = dst->type;
    if (t != FATTN_TYPE_F16 && t != FATTN_TYPE_Q8_0 && t != FATTN_TYPE_Q4_0) return FATTN_ERR_UNSUPPORTED_TYPE;
    for (int i = 0; i < 4; i++)
        if (src->ne[i] != dst->ne[i] || src->ne[i] <= 0) return FATTN_ERR_INVALID_ARG;
    const int64_t ue = t == FATTN_TYPE_F16 ? 1 : QK;
    if (src->ne[0] % ue) return FATTN_ERR_INVALID_ARG;
    if (dst->nb[0] != (int64_t)fattn_row_size(t, ue)) return FATTN_ERR_BAD_STRIDE;
    if ((uintptr_t)src->data % 4 || src->nb[1] % 4 || src->nb[2] % 4 || src->nb[3] % 4) return FATTN_ERR_ALIGNMENT;
    if ((uintptr_t)dst->data % 2 || dst->nb[1] % 2 || dst->nb[2] % 2 || dst->nb[3] % 2) return FATTN_ERR_ALIGNMENT;
    CpyArgs a;
    a.src = (const uint8_t*)src->data;
    a.dst = (uint8_t*)dst->data;
    a.ne0 = src->ne[0]; a.ne1 = src->ne[1]; a.ne2 = src->ne[2]; a.ne3 = src->ne[3];
    a.snb1 = src->nb[1]; a.snb2 = src->nb[2]; a.snb3 = src->nb[3];
    a.dnb1 = dst->nb[1]; a.dnb2 = dst->nb[2]; a.dnb3 = dst->nb[3];
    const int64_t units = a.ne0 / ue * a.ne1 * a.ne2 * a.ne3;
    const dim3 grid((unsigned)((units + 255) / 256));
    hipStream_t st = (hipStream_t)stream;
    (void)hipGetLastError();
    if (t == FATTN_TYPE_F16) hipLaunchKernelGGL(cpy_f32_kernel<FATTN_TYPE_F16>, grid, dim3(256), 0, st, a, units);
    else if (t == FATTN_TYPE_Q8_0) hipLaunchKernelGGL(cpy_f32_kernel<FATTN_TYPE_Q8_0>, grid, dim3(256), 0, st, a, units);
    else hipLaunchKernelGGL(cpy_f32_kernel<FATTN_TYPE_Q4_0>, grid, dim3(256), 0, st, a, units);
    return hipGetLastError() == hipSuccess ? FATTN_OK : FATTN_ERR_LAUNCH;
}

}  // extern "C"
