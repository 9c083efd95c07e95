/*
 * fattn_debug.h -- diagnostics of the fattn C ABI (include/fattn.h): planner
 * overrides for tests, sweeps and A/B runs, the plan fattn_ext would launch as
 * text, and fattn_ext with HIP events around its kernels (bench.py's roofline).
 * Exported by the same library (libfattn.so).  None of this is needed to use
 * the drop-in path: every override defaults to the planner's choice, and a
 * production caller never sets one.
 */
#ifndef FATTN_DEBUG_H
#define FATTN_DEBUG_H

#include "fattn.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Same as fattn_ext, additionally recording the hipEvent_t `ev_begin` / `ev_end`
 * on `stream` immediately before the first and after the last kernel of the
 * plan -- the attention kernel, plus the chunk-merge kernel when the plan
 * merges its split-KV partials in a second launch (fattn_describe names both),
 * plus the prefill mask-flags pass before it -- so a caller can time the whole
 * attention op on the device with hipEventElapsedTime.  Either event may be NULL. */
int fattn_ext_events(const fattn_params* p, void* stream, void* ev_begin, void* ev_end);

/* Planner overrides (tests, benchmarks).  They are PROCESS-WIDE: one call changes
 * the plans of every later fattn_ext / fattn_describe / fattn_workspace_size on
 * every host thread (stored in atomics, so never torn, but a thread that sets an
 * option while another plans races with it).  Set them before launching, or from
 * one thread.  Option ids of removed experiments are not reused.  Returns
 * FATTN_OK or FATTN_ERR_INVALID_ARG. */
enum {
    FATTN_OPT_MQ_ROWS_PER_WAVE = 1, /* multi-query kernel: 0 = auto, 16 (4 waves x 16 rows), 32 (8 waves x 32 rows) */
    FATTN_OPT_MQ_DISABLE = 2,       /* 1 = never pick the multi-query kernel (split-KV kernel only) */
    FATTN_OPT_SPLIT_STEPS = 3,      /* split kernel: 32-position steps per wave (0 = auto, 1..64) */
    FATTN_OPT_SPLIT_INFLIGHT = 4,   /* split kernel: steps in flight per wave (0 = auto, 1..4; LDS permitting) */
    FATTN_OPT_PF = 5,               /* prefill kernel: 0 = auto, 1 = never, 2 = whenever eligible (even if the
                                       workgroups do not fill the chip) */
    FATTN_OPT_PF_STAGGER = 6,       /* prefill kernel, bit 1 (default on): waves 4-7 at s_setprio 1; bit 2:
                                       XCD-grouped workgroup order (the query tiles of a kv head on one XCD);
                                       bit 0 (a phase stagger of SIMD partners) was removed and is rejected */
    FATTN_OPT_SPLIT_WAVE_MERGE = 10 /* split kernel, one-row tiles with <= 32 wave partials: 0 = every wave
                                       publishes and the last-arriving wave merges (default), 1 = the
                                       workgroup-level merge used for all other tiles */,
    FATTN_OPT_SPLIT_PRIO = 11       /* split kernel wave priorities: 0 = staggered 3/2/1/0 (default), 1 = none,
                                       2 = staggered only while the first steps are issued */,
    FATTN_OPT_PF_SKIP = 12          /* masked prefill: 0 = a pre-pass flags the blocks with any key above -inf
                                       and the kernel walks only the live KV range, longest query tiles
                                       first (default; the workspace holds n_qt * N/64 flag bytes),
                                       1 = no pre-pass (every tile fetched; all -inf wave blocks still skipped) */,
    FATTN_OPT_MQ_MIN_ROWS = 13,     /* multi-query kernel only from this many packed (query x head) rows per kv
                                       head (0 = the default, 64; minimum 32); fewer rows take the split-KV kernel.
                                       An explicit value (64 included) also lifts the default's rule that every
                                       KV chunk hold two 128-key tiles */
    FATTN_OPT_SPLIT_WAVES = 19,     /* split kernel waves per workgroup: 0 = auto, 4, 8 or 16 (16-B row path;
                                       16 needs the Q8_0/Q4_0 register budget, else clamped to 8) */
    FATTN_OPT_SPLIT_SKIP = 20       /* split kernel, masked: 0 = steps whose mask is -inf for every key and row
                                       of the tile are neither loaded nor computed (default; the mask words are
                                       read beside Q), 1 = every step loaded and computed */,
    FATTN_OPT_SPLIT_MERGE = 21,     /* split kernel, tiles of several packed rows: 0 = with 4+ chunks the partials
                                       merge one wave per (tile, row), in a second launch or in-kernel
                                       (FATTN_OPT_MERGE_IN_KERNEL) (default), 1 = the last-arriving workgroup merges
                                       the whole tile (combine_tile) */
    FATTN_OPT_BD = 22               /* batched-decode kernels (64-row workgroups, 16-B rows): the compute /
                                       build-role form fattn_bdp_kernel for Q8_0 / Q4_0 K/V at D = 64, 96, 128;
                                       the all-waves form fattn_bd_kernel for Q8_0 / Q4_0 at D = 128 (value 2
                                       only) and for f16 K/V at D = 64, 96, 128 (always: f16 has no role form).
                                       0 = auto (from 64 packed rows per kv head, below the prefill shapes),
                                       1 = never, 2 = the all-waves form whenever eligible (quantised D = 64 / 96:
                                       the multi-query kernel instead), 3 = the role form whenever eligible --
                                       on f16 K/V 3 runs the all-waves form */,
    /* 23: a removed experiment (one-row partials as data-tagged granules), rejected */
    FATTN_OPT_MERGE_IN_KERNEL = 24  /* chunk partials of multi-row tiles (split kernel with 4+ chunks, batched-
                                       decode kernel): 0 = merged in a second launch (default); 1 = inside the
                                       launch when the whole grid is co-resident -- the tile's workgroups wait
                                       for each other, then each merges a share of the rows (0.6-1.5 us slower).
                                       Co-residency is judged from CU count, LDS and launch bounds only: on a
                                       device shared with other streams or processes (or CU-masked) a waiting
                                       workgroup's bounded poll can give up, and it then writes NaN rows while
                                       fattn_ext has returned FATTN_OK.  Diagnostics only; keep 0 in production */,
    FATTN_OPT_BD_XCD = 25           /* batched-decode kernels: workgroup order. 0 = auto (XCD-grouped), 1 = plain
                                       (chunk fastest), 2 = XCD-grouped: each of the 8 XCDs takes whole (kv head x
                                       row tile)s, so a tile's Q rows come from HBM once, not once per chunk
                                       (needs a grid of a multiple of 8 workgroups; otherwise plain) */,
    FATTN_OPT_SPLIT_XCD = 26        /* split kernel: workgroup order. 0 = auto (XCD-grouped for one-row tiles merged
                                       in the launch, e.g. config 3; plain otherwise), 1 = plain, 2 = XCD-grouped:
                                       a tile's chunk workgroups on one XCD (grid a multiple of 8 workgroups) */,
    /* 27: a removed experiment (speculative granule merge of one-row tiles: slower), rejected */
    FATTN_OPT_PF_STAGE = 28         /* prefill kernel over Q8_0 / Q4_0 K/V: 0 = auto (staged), 1 = dequantised in
                                       the kernel, tile by tile, once per 256-row query tile; 2 = staged: the rows
                                       converted once to f16 in the workspace (kv_stage_f16, + 2 * Skv * Hkv * N *
                                       D * 2 bytes of fattn_workspace_size), then the f16 prefill kernel */,
    FATTN_OPT_SPLIT_LOADERS = 30,   /* split kernel, one-row tiles on 8 waves whose whole KV chunk fits the LDS (16-B
                                       rows, D = 64 / 128, one K / V type): 0 = auto, 1 = off (every wave issues its
                                       own steps), 2 = 4 loader waves issue every step up front and hand each over
                                       to its compute wave by LDS flags (fattn_split_ld_kernel) */
    FATTN_OPT_GQA_UNPACK = 33,      /* GQA decode of one query row (config 4): 0 = auto (packed), 1 = the kv head's
                                       R q heads packed in one split tile (second-launch merge), 2 = one q head
                                       per tile (one-row tiles, merged in the launch; K/V read R times) */
    FATTN_OPT_PART_F16 = 32,        /* chunk partials of the second-launch merges (multi-row split tiles, batched
                                       decode, multi-query; D != 64): 0 = auto (f16 for batched decode, multi-query
                                       and split tiles of 8+ rows), 1 = f32 (O unnormalised), 2 = f16 (O / l in
                                       f16 beside (m, l) in f32: half the partial bytes) */
    FATTN_OPT_MERGE_PLAIN = 31,     /* second-launch merges of multi-row split / batched-decode plans
                                       (fattn_merge_kernel, fattn_bd_merge_kernel): 0 = auto (sc1 loads), 1 = sc1
                                       loads, 2 = plain loads (the kernel boundary already orders the partials) */
    FATTN_OPT_PF_FORM = 29          /* prefill body over f16 rows (native or staged) at D = 128: 0 = auto (6), 1 =
                                       the 8-wave form (fattn_pf_kernel), 4 = one wave per SIMD, pipelined (two
                                       32-MFMA phases per tile, P.V one tile behind S), 5 = pipelined and balanced
                                       (each phase carries one row block's exponentials and the other's scores /
                                       max, interleaved over its 32 steps), 6 = "lean": the balanced form with each
                                       S^T chain started from the row's -m / c, so the accumulator times c is the
                                       exponent argument (bodies without mask values; not bit-identical to 1 / 4
                                       / 5).  2, 3: round 5's unpipelined
                                       one-wave-per-SIMD forms, removed (slower), rejected */
};
int fattn_set_option(int option, int value);

/* Diagnostic: the kernel(s) fattn_ext would launch for `p` and the plan's
 * grid / LDS / chunk / workspace, as text (NUL-terminated, at most cap bytes).
 * Returns FATTN_OK or the error fattn_ext would return. */
int fattn_describe(const fattn_params* p, char* out, size_t cap);


#ifdef __cplusplus
}
#endif
#endif /* FATTN_DEBUG_H */
