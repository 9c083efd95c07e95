// fattn_launch.h -- the launch plan and the kernel launchers, shared by the
// planner / C ABI (fattn_api.hip) and the per-head-dim translation units
// (fattn_launch_d*.hip: each instantiates launch_types<D>, so the kernels of
// the head dims compile in parallel).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>

#include "fattn_quant.h"
#include "fattn_mq.h"
#include "fattn_pf.h"
#include "fattn_pf4.h"
#include "fattn_bd.h"
#include "fattn_bdp.h"
#include "fattn_split.h"

namespace fattn {

constexpr int kMaxDevices = 64;

struct Plan {
    SplitArgs a;
    int kt, vt;  // vt may be VT_F16T
    int D;
    int gran;
    dim3 grid;
    int lds;
    size_t ws_bytes, cnt_bytes, ml_bytes;
    int cus;  // compute units of the device the plan is for
    int nwv;  // split kernel: waves per workgroup (4, 8, 16)
    int nld = 0;
    bool merge_plain = false;  // second-launch merges (split, batched decode): plain loads (FATTN_OPT_MERGE_PLAIN)  // split kernel: loader waves beside the nwv compute waves (fattn_split_ld_kernel), 0 = none
    bool mq;  // multi-query kernel (fattn_mq.h)
    bool pf;  // prefill kernel (fattn_pf.h)
    bool bd;  // batched-decode kernel (fattn_bd.h)
    bool bdp; // ... in its compute / build-role form (fattn_bdp.h; Q8_0 / Q4_0)
    bool pf_flags = false;  // masked prefill: live-block flags pre-pass (tile-range skipping)
    // prefill over Q8_0 / Q4_0: the rows staged to f16 in the workspace first
    // (kv_stage_f16_kernel), then the f16 prefill kernel (kt = vt = F16 then)
    bool pf4 = false;       // the prefill's one-wave-per-SIMD body (fattn_pf4.h; f16 rows, D = 128)
    int pf4_sched = 0;      // ... its schedule (fattn_pf4_kernel's SCHED)
    bool pf_stage = false;
    int stage_kt = 0;                                  // the cache's type
    const uint8_t *stage_k = nullptr, *stage_v = nullptr;  // the cache's K / V
    int64_t stage_k_nb2 = 0, stage_k_nb3 = 0, stage_v_nb2 = 0, stage_v_nb3 = 0;
    int stage_hkv = 0, stage_skv = 0;
    size_t stage_off = 0, stage_bytes = 0;             // per K (or V): Skv * Hkv * N * D * 2
    int nw;   // mq kernel: waves per workgroup: 4 (16 rows each) or 8 (32 rows each)
};

struct Events {
    hipEvent_t begin = nullptr, end = nullptr;
};

// Launch with errors attributed to this launch only: a pending error left on
// the thread by other code is cleared first; FATTN_DEBUG=1 names a failure.
template <typename F>
int launch_kernel(const void* kern, const Plan& pl, hipStream_t st, const Events& ev, F&& go) {
    (void)hipGetLastError();
    // large dynamic LDS must be allowed per kernel and per device: cached per
    // (launch site = F's instantiation, device); a lost race only repeats the call
    static std::atomic<int> lds_set[kMaxDevices];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = 0;
    if (pl.lds > 65536 && pl.lds > lds_set[dev].load(std::memory_order_relaxed)) {
        // the query loads the code object (HIP loads kernels lazily; setting an
        // attribute of a kernel whose module is not loaded yet fails)
        hipFuncAttributes fa;
        (void)hipFuncGetAttributes(&fa, kern);
        if (hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, pl.lds) == hipSuccess) {
            lds_set[dev].store(pl.lds, std::memory_order_relaxed);
        } else if (std::getenv("FATTN_DEBUG")) {
            std::fprintf(stderr, "fattn: hipFuncSetAttribute(%d B LDS) failed; launching anyway\n", pl.lds);
        }
        (void)hipGetLastError();
    }
    if (ev.begin) (void)hipEventRecord(ev.begin, st);
    go();
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        if (std::getenv("FATTN_DEBUG"))
            std::fprintf(stderr, "fattn: launch grid (%u,%u,%u) lds %d failed: %s\n", pl.grid.x, pl.grid.y, pl.grid.z,
                         pl.lds, hipGetErrorString(e));
        return FATTN_ERR_LAUNCH;
    }
    if (ev.end) (void)hipEventRecord(ev.end, st);
    return FATTN_OK;
}

template <int KT, int VT, int D, int GRAN, bool HM, int NWV, int EPI>
int launch_split_e(const Plan& pl, hipStream_t st, const Events& ev) {
    if constexpr (GRAN == 16 && NWV == 8 && EPI == 2 && KT == VT && (D == 64 || D == 128)) {
        if (pl.nld == kSplitLoaders) {
            auto lk = fattn_split_ld_kernel<KT, VT, D, HM, NWV, kSplitLoaders>;
            return launch_kernel((const void*)lk, pl, st, ev, [&] {
                hipLaunchKernelGGL(lk, pl.grid, dim3((NWV + kSplitLoaders) * kWave), pl.lds, st, pl.a);
            });
        }
    }
    if (pl.nld) return FATTN_ERR_INVALID_ARG;
    auto kern = fattn_split_kernel<KT, VT, D, GRAN, HM, NWV, EPI>;
    return launch_kernel((const void*)kern, pl, st, ev, [&] {
        hipLaunchKernelGGL(kern, pl.grid, dim3(NWV * kWave), pl.lds, st, pl.a);
        if constexpr (EPI == 0) {
            // multi-row tiles: the chunk partials merge in a second launch, with
            // as few load slots per lane as the chunk count allows (the slots
            // past it still cost issue cycles) -- unless they merge in-kernel (2)
            if (pl.a.merge_launch == 1) {
                // one wave per packed row a tile can hold: R heads x the query
                // rows it really has (config 4's 4-row GQA tiles, QPT 4 but one
                // query row: one workgroup per tile, not four)
                const int qrows = pl.a.QPT < pl.a.NQ ? pl.a.QPT : pl.a.NQ;
                const int rows = qrows * pl.a.R < kRows ? qrows * pl.a.R : kRows;
                const dim3 g((unsigned)((rows + 3) / 4), pl.grid.y, pl.grid.z);
                const int need = (pl.a.n_chunks + merge_ppr<D>() - 1) / merge_ppr<D>();
                auto go = [&](auto kit, auto plain, auto f16) {
                    hipLaunchKernelGGL((fattn_merge_kernel<D, decltype(kit)::value, decltype(plain)::value, decltype(f16)::value>),
                                       g, dim3(256), 0, st, pl.a);
                };
                auto pick = [&](int nd, auto plain, auto f16) {
                    if (nd <= 2) go(std::integral_constant<int, 2>(), plain, f16);
                    else if (nd <= 4) go(std::integral_constant<int, 4>(), plain, f16);
                    else if (nd <= 8) go(std::integral_constant<int, 8>(), plain, f16);
                    else go(std::integral_constant<int, 16>(), plain, f16);
                };
                if constexpr (D != 64) {
                    if (pl.a.part_f16) {  // (f16 partials: 16-B loads of 8 dims, merge_ppr_h parts per lane row)
                        pick((pl.a.n_chunks + merge_ppr_h<D>() - 1) / merge_ppr_h<D>(), std::false_type(), std::true_type());
                        return;
                    }
                }
                if (pl.merge_plain) pick(need, std::true_type(), std::false_type());
                else pick(need, std::false_type(), std::false_type());
            }
        }
    });
}

// the plan's epilogue (a.wave_merge): 1 only for 4 waves at D = 128
template <int KT, int VT, int D, int GRAN, bool HM, int NWV>
int launch_split_w(const Plan& pl, hipStream_t st, const Events& ev) {
    if constexpr (NWV == 4 && D == 128) {
        if (pl.a.wave_merge == 1) return launch_split_e<KT, VT, D, GRAN, HM, NWV, 1>(pl, st, ev);
    }
    if (pl.a.wave_merge == 2) return launch_split_e<KT, VT, D, GRAN, HM, NWV, 2>(pl, st, ev);
    if (pl.a.wave_merge != 0) return FATTN_ERR_INVALID_ARG;
    return launch_split_e<KT, VT, D, GRAN, HM, NWV, 0>(pl, st, ev);
}

// 8 / 16 waves per workgroup: the 16-B path only; 16 needs the 4-waves-per-SIMD
// register budget (split_waves_per_simd); the planner never asks otherwise
template <int KT, int VT, int D, int GRAN, bool HM>
int launch_split_hm(const Plan& pl, hipStream_t st, const Events& ev) {
    if constexpr (GRAN == 16) {
        if (pl.nwv == 8) return launch_split_w<KT, VT, D, GRAN, HM, 8>(pl, st, ev);
        if constexpr (split_waves_per_simd<KT, D, GRAN>() == 4) {
            if (pl.nwv == 16) return launch_split_w<KT, VT, D, GRAN, HM, 16>(pl, st, ev);
        }
    }
    if (pl.nwv != 4) return FATTN_ERR_INVALID_ARG;
    return launch_split_w<KT, VT, D, GRAN, HM, 4>(pl, st, ev);
}

template <int KT, int VT, int D, int GRAN>
int launch_split(const Plan& pl, hipStream_t st, const Events& ev) {
    return pl.a.has_mask ? launch_split_hm<KT, VT, D, GRAN, true>(pl, st, ev)
                         : launch_split_hm<KT, VT, D, GRAN, false>(pl, st, ev);
}

template <int KT, int VT, int D>
int launch_gran(const Plan& pl, hipStream_t st, const Events& ev) {
    if constexpr (VT == VT_F16T) {
        return launch_split<KT, VT, D, 16>(pl, st, ev);
    } else {
        return pl.gran == 16 ? launch_split<KT, VT, D, 16>(pl, st, ev) : launch_split<KT, VT, D, 4>(pl, st, ev);
    }
}

template <int KT, int D, int NW, bool HM>
int launch_mq_hm(const Plan& pl, hipStream_t st, const Events& ev) {
    auto kern = fattn_mq_kernel<KT, D, NW, HM>;
    return launch_kernel((const void*)kern, pl, st, ev, [&] {
        hipLaunchKernelGGL(kern, pl.grid, dim3(NW * kWave), pl.lds, st, pl.a);
        if (pl.a.merge_launch) {
            // the chunk partials of every 16-row subtile (4 per 64-row tile,
            // 16 per 256-row tile) merge in a second launch
            constexpr int SUBS = NW == 8 ? 16 : 4;
            const dim3 g(kRows / 4, pl.grid.y * SUBS, pl.grid.z);
            const int need = (pl.a.n_chunks + merge_ppr<D>() - 1) / merge_ppr<D>();
            auto go = [&](auto kit, auto f16) {
                hipLaunchKernelGGL((fattn_mq_merge_kernel<D, decltype(kit)::value, SUBS, decltype(f16)::value>), g,
                                   dim3(256), 0, st, pl.a);
            };
            auto pick = [&](int nd, auto f16) {
                if (nd <= 2) go(std::integral_constant<int, 2>(), f16);
                else if (nd <= 4) go(std::integral_constant<int, 4>(), f16);
                else if (nd <= 8) go(std::integral_constant<int, 8>(), f16);
                else go(std::integral_constant<int, 16>(), f16);
            };
            if constexpr (D != 64) {
                if (pl.a.part_f16) {
                    pick((pl.a.n_chunks + merge_ppr_h<D>() - 1) / merge_ppr_h<D>(), std::true_type());
                    return;
                }
            }
            pick(need, std::false_type());
        }
    });
}

template <int KT, int D>
int launch_mq(const Plan& pl, hipStream_t st, const Events& ev) {
    if constexpr (D != 256) {  // D = 256: 64-row workgroups only (LDS)
        if (pl.nw == 8)
            return pl.a.has_mask ? launch_mq_hm<KT, D, 8, true>(pl, st, ev) : launch_mq_hm<KT, D, 8, false>(pl, st, ev);
    }
    return pl.a.has_mask ? launch_mq_hm<KT, D, 4, true>(pl, st, ev) : launch_mq_hm<KT, D, 4, false>(pl, st, ev);
}

template <int KT, int D, bool HM>
int launch_pf_hm(const Plan& pl, hipStream_t st, const Events& ev) {
    auto kern = fattn_pf_kernel<KT, D, HM>;
    const void* main_kern = (const void*)kern;
    if constexpr (KT == FATTN_TYPE_F16 && D == 128) {
        if (pl.pf4)
            main_kern = pl.pf4_sched == 4   ? (const void*)fattn_pf4_kernel<D, HM, 4>
                        : pl.pf4_sched == 3 ? (const void*)fattn_pf4_kernel<D, HM, 3>
                                            : (const void*)fattn_pf4_kernel<D, HM, 2>;
    }
    return launch_kernel(main_kern, pl, st, ev, [&] {
        // the pre-pass, one launch: the quantised cache's rows -> f16 rows in the
        // workspace (K and V), and the mask's live / +-0 block flags
        bool staged = false;
        if constexpr (KT == FATTN_TYPE_F16 && D % QK == 0) staged = pl.pf_stage;
        const bool flags = HM && pl.a.pf_flags;
        if (staged || flags) {
            PfPrepassArgs pa{};
            pa.nblk = (int64_t)pl.a.N * D / QK;
            pa.per_head = staged ? (int)((4 * pa.nblk + 255) / 256) : 0;
            pa.hkv = pl.stage_hkv, pa.skv = pl.stage_skv;
            pa.k = pl.stage_k, pa.v = pl.stage_v;
            pa.k_nb2 = pl.stage_k_nb2, pa.k_nb3 = pl.stage_k_nb3, pa.v_nb2 = pl.stage_v_nb2, pa.v_nb3 = pl.stage_v_nb3;
            pa.k16 = (uint16_t*)pl.a.k, pa.v16 = (uint16_t*)pl.a.v;
            pa.mask = pl.a.mask, pa.m_nb1 = pl.a.m_nb1, pa.NQ = pl.a.NQ, pa.QPT = pl.a.QPT;
            pa.ntiles = pl.a.N / kPfKeys, pa.flags = (uint8_t*)pl.a.pf_flags;
            const int64_t nfl = flags ? (int64_t)pa.ntiles * pl.a.n_qt : 0;
            const int64_t nst = staged ? 2 * (int64_t)pa.per_head * pa.hkv * pa.skv : 0;
            const dim3 g((unsigned)(nst + nfl));
            if (!staged) hipLaunchKernelGGL(pf_prepass_kernel<0>, g, dim3(256), 0, st, pa);
            else if (pl.stage_kt == FATTN_TYPE_Q8_0) hipLaunchKernelGGL(pf_prepass_kernel<FATTN_TYPE_Q8_0>, g, dim3(256), 0, st, pa);
            else hipLaunchKernelGGL(pf_prepass_kernel<FATTN_TYPE_Q4_0>, g, dim3(256), 0, st, pa);
        }
        if constexpr (KT == FATTN_TYPE_F16 && D == 128) {
            if (pl.pf4) {
                if (pl.pf4_sched == 4)
                    hipLaunchKernelGGL((fattn_pf4_kernel<D, HM, 4>), pl.grid, dim3(kPf4Waves * kWave), pl.lds, st, pl.a);
                else if (pl.pf4_sched == 3)
                    hipLaunchKernelGGL((fattn_pf4_kernel<D, HM, 3>), pl.grid, dim3(kPf4Waves * kWave), pl.lds, st, pl.a);
                else
                    hipLaunchKernelGGL((fattn_pf4_kernel<D, HM, 2>), pl.grid, dim3(kPf4Waves * kWave), pl.lds, st, pl.a);
                return;
            }
        }
        hipLaunchKernelGGL(kern, pl.grid, dim3(kPfWaves * kWave), pl.lds, st, pl.a);
    });
}

// D = 128: the all-waves form, or the role form for quantised K/V (pl.bdp);
// D = 64 / 96: the role form for quantised K/V (the planner sets pl.bdp), the
// all-waves form's f16 image ring for f16
template <int KT, int D, bool HM>
int launch_bd_hm(const Plan& pl, hipStream_t st, const Events& ev) {
    void (*kern)(SplitArgs) = nullptr;
    if constexpr (D == 128 || KT == FATTN_TYPE_F16) kern = fattn_bd_kernel<KT, D, HM>;
    if constexpr (KT != FATTN_TYPE_F16) {
        if (pl.bdp) kern = fattn_bdp_kernel<KT, D, HM>;
    }
    if (kern == nullptr || (D != 128 && KT != FATTN_TYPE_F16 && !pl.bdp)) return FATTN_ERR_UNSUPPORTED_TYPE;
    return launch_kernel((const void*)kern, pl, st, ev, [&] {
        hipLaunchKernelGGL(kern, pl.grid, dim3(kBdWaves * kWave), pl.lds, st, pl.a);
        if (pl.a.merge_launch == 1) {
            const dim3 g(kBdRows / 4, pl.grid.y, pl.grid.z);
            const int need = (pl.a.n_chunks + merge_ppr<D>() - 1) / merge_ppr<D>();
            auto go = [&](auto kit, auto plain, auto f16) {
                hipLaunchKernelGGL((fattn_bd_merge_kernel<D, decltype(kit)::value, decltype(plain)::value, decltype(f16)::value>),
                                   g, dim3(256), 0, st, pl.a);
            };
            auto pick = [&](int nd, auto plain, auto f16) {
                if (nd <= 2) go(std::integral_constant<int, 2>(), plain, f16);
                else if (nd <= 4) go(std::integral_constant<int, 4>(), plain, f16);
                else if (nd <= 8) go(std::integral_constant<int, 8>(), plain, f16);
                else go(std::integral_constant<int, 16>(), plain, f16);
            };
            if constexpr (D != 64) {
                if (pl.a.part_f16) {  // (f16 partials: 16-B loads of 8 dims, merge_ppr_h parts per lane row)
                    pick((pl.a.n_chunks + merge_ppr_h<D>() - 1) / merge_ppr_h<D>(), std::false_type(), std::true_type());
                    return;
                }
            }
            if (pl.merge_plain) pick(need, std::true_type(), std::false_type());
            else pick(need, std::false_type(), std::false_type());
        }
    });
}

template <int KT, int D>
int launch_bd(const Plan& pl, hipStream_t st, const Events& ev) {
    return pl.a.has_mask ? launch_bd_hm<KT, D, true>(pl, st, ev) : launch_bd_hm<KT, D, false>(pl, st, ev);
}

template <int KT, int D>
int launch_pf(const Plan& pl, hipStream_t st, const Events& ev) {
    return pl.a.has_mask ? launch_pf_hm<KT, D, true>(pl, st, ev) : launch_pf_hm<KT, D, false>(pl, st, ev);
}

// split kernel over mixed K / V cache types (instantiated once per D in
// fattn_launch_mixed_d<D>.hip; D = 64, 128, 256)
template <int D>
int launch_mixed(const Plan& pl, hipStream_t st, const Events& ev) {
    constexpr int F16 = FATTN_TYPE_F16, Q8 = FATTN_TYPE_Q8_0, Q4 = FATTN_TYPE_Q4_0;
    if (pl.kt == Q8 && pl.vt == F16) return launch_gran<Q8, F16, D>(pl, st, ev);
    if (pl.kt == Q4 && pl.vt == F16) return launch_gran<Q4, F16, D>(pl, st, ev);
    if (pl.kt == F16 && pl.vt == Q8) return launch_gran<F16, Q8, D>(pl, st, ev);
    if (pl.kt == F16 && pl.vt == Q4) return launch_gran<F16, Q4, D>(pl, st, ev);
    if (pl.kt == Q8 && pl.vt == Q4) return launch_gran<Q8, Q4, D>(pl, st, ev);
    if (pl.kt == Q4 && pl.vt == Q8) return launch_gran<Q4, Q8, D>(pl, st, ev);
    return FATTN_ERR_UNSUPPORTED_TYPE;
}
extern template int launch_mixed<64>(const Plan&, hipStream_t, const Events&);
extern template int launch_mixed<128>(const Plan&, hipStream_t, const Events&);
extern template int launch_mixed<256>(const Plan&, hipStream_t, const Events&);

// every kernel of head dim D (defined here, instantiated once per D in
// fattn_launch_d<D>.hip)
template <int D>
int launch_types(const Plan& pl, hipStream_t st, const Events& ev) {
    if constexpr (D == 64 || D == 128 || D == 256) {
        if (pl.kt != pl.vt && pl.vt != VT_F16T) return launch_mixed<D>(pl, st, ev);
    }
    if constexpr (D == 64 || D == 80 || D == 96 || D == 128) {
        if (pl.pf) {
            if (pl.kt == FATTN_TYPE_F16 && pl.vt == FATTN_TYPE_F16) return launch_pf<FATTN_TYPE_F16, D>(pl, st, ev);
            if constexpr (D != 80) {  // (80 is not a whole number of ggml blocks)
                if (pl.kt == FATTN_TYPE_Q8_0 && pl.vt == FATTN_TYPE_Q8_0) return launch_pf<FATTN_TYPE_Q8_0, D>(pl, st, ev);
                if (pl.kt == FATTN_TYPE_Q4_0 && pl.vt == FATTN_TYPE_Q4_0) return launch_pf<FATTN_TYPE_Q4_0, D>(pl, st, ev);
            }
            return FATTN_ERR_UNSUPPORTED_TYPE;
        }
    }
    if constexpr (D == 64 || D == 96 || D == 128) {
        if (pl.bd) {
            if (pl.kt == FATTN_TYPE_Q8_0 && pl.vt == FATTN_TYPE_Q8_0) return launch_bd<FATTN_TYPE_Q8_0, D>(pl, st, ev);
            if (pl.kt == FATTN_TYPE_Q4_0 && pl.vt == FATTN_TYPE_Q4_0) return launch_bd<FATTN_TYPE_Q4_0, D>(pl, st, ev);
            if (pl.kt == FATTN_TYPE_F16 && pl.vt == FATTN_TYPE_F16) return launch_bd<FATTN_TYPE_F16, D>(pl, st, ev);
            return FATTN_ERR_UNSUPPORTED_TYPE;
        }
    }
    if constexpr (D == 64 || D == 128 || D == 256) {
        if (pl.mq) {
            if (pl.kt == FATTN_TYPE_Q8_0 && pl.vt == FATTN_TYPE_Q8_0) return launch_mq<FATTN_TYPE_Q8_0, D>(pl, st, ev);
            if (pl.kt == FATTN_TYPE_Q4_0 && pl.vt == FATTN_TYPE_Q4_0) return launch_mq<FATTN_TYPE_Q4_0, D>(pl, st, ev);
            return FATTN_ERR_UNSUPPORTED_TYPE;
        }
    }
    if (pl.pf || pl.mq || pl.bd) return FATTN_ERR_UNSUPPORTED_HEAD_DIM;
    if constexpr (D % QK == 0) {
        if (pl.kt == FATTN_TYPE_Q8_0 && pl.vt == FATTN_TYPE_Q8_0)
            return launch_gran<FATTN_TYPE_Q8_0, FATTN_TYPE_Q8_0, D>(pl, st, ev);
        if (pl.kt == FATTN_TYPE_Q4_0 && pl.vt == FATTN_TYPE_Q4_0)
            return launch_gran<FATTN_TYPE_Q4_0, FATTN_TYPE_Q4_0, D>(pl, st, ev);
    }
    if (pl.kt == FATTN_TYPE_F16 && pl.vt == FATTN_TYPE_F16) return launch_gran<FATTN_TYPE_F16, FATTN_TYPE_F16, D>(pl, st, ev);
    if (pl.kt == FATTN_TYPE_F16 && pl.vt == VT_F16T) return launch_gran<FATTN_TYPE_F16, VT_F16T, D>(pl, st, ev);
    return FATTN_ERR_UNSUPPORTED_TYPE;
}

extern template int launch_types<64>(const Plan&, hipStream_t, const Events&);
extern template int launch_types<80>(const Plan&, hipStream_t, const Events&);
extern template int launch_types<96>(const Plan&, hipStream_t, const Events&);
extern template int launch_types<128>(const Plan&, hipStream_t, const Events&);
extern template int launch_types<256>(const Plan&, hipStream_t, const Events&);

}  // namespace fattn
