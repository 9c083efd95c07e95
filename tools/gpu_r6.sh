#!/bin/bash
# Round 6's GPU passes, one function per pass: bash tools/gpu_r6.sh <pass>
source tools/gpu_round.sh
export TMPDIR=/tmp

# First pass: the one-shot read ceiling of config 3's launch shape, the default
# bench line of the round-5 tree, the world-1 RCCL bench lines (graph, eager).
pass_a() {
  run oneshot 300 python -u tools/oneshot.py
  run bench 500 python -u bench.py
  run dist_graph 300 python -u bench.py --dist --no-side-line
  run dist_eager 300 python -u bench.py --dist --no-side-line --eager-gather
}



# Second pass: config 3's timeline from the LDS-stamps build (auto plan, then
# both steps in flight, 16 waves).
pass_b() {
  run stamps_auto 200 python -u tools/stamps.py
  run stamps_inflight2 200 python -u tools/stamps.py --inflight 2
  run stamps_w16 200 python -u tools/stamps.py --waves 16
  run stamps_w4 200 python -u tools/stamps.py --waves 4
}

# Third pass: the loader-wave split kernel -- parity, same-box A/B on configs
# 3 and 2, its stamps timeline.
pass_c() {
  run t_ld 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "loader_waves or config3 or config2"
  run ab_ld_c3 300 python -u tools/ab_decode.py --workload config3 --rounds 6 --variant base: --variant ld:SPLIT_LOADERS=2
  run ab_ld_c2 300 python -u tools/ab_decode.py --workload config2 --rounds 4 --variant base: --variant ld:SPLIT_LOADERS=2
  run stamps_ld 200 python -u tools/stamps.py --loaders 2
}

# Fourth pass: loader waves v2 (compute waves issue step 0) -- parity, A/B,
# stamps; the lean prefill body (form 6) -- parity, A/B against the balanced
# body (form 5) on the bench's prefill shapes.
pass_d() {
  run t_d 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "loader_waves or pf4 or pf_sweep or pf_staged or zero_mask_bench"
  run ab_ld2_c3 300 python -u tools/ab_decode.py --workload config3 --rounds 6 --variant base: --variant ld:SPLIT_LOADERS=2
  run ab_ld2_c2 300 python -u tools/ab_decode.py --workload config2 --rounds 4 --variant base: --variant ld:SPLIT_LOADERS=2
  run stamps_ld2 200 python -u tools/stamps.py --loaders 2
  run ab_lean_q8z 400 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 3 --variant bal:PF_FORM=5 --variant lean:PF_FORM=6
  run ab_lean_f16 300 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 3 --variant bal:PF_FORM=5 --variant lean:PF_FORM=6
  run ab_lean_q8r 300 python -u tools/ab_prefill.py --kv q8_0 --mask random --rounds 2 --variant bal:PF_FORM=5 --variant lean:PF_FORM=6
}

# Fifth pass: the lean prefill body (exact Q, chains from -m / c; masked bodies
# balanced) -- parity, then a longer same-box A/B against the balanced body.
pass_e() {
  run t_e 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "pf4 or pf_sweep or pf_staged or zero_mask_bench"
  run ab_lean2_q8z 500 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 6 --variant bal:PF_FORM=5 --variant lean:PF_FORM=6
  run ab_lean2_f16 400 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 5 --variant bal:PF_FORM=5 --variant lean:PF_FORM=6
  run ab_lean2_q8r 300 python -u tools/ab_prefill.py --kv q8_0 --mask random --rounds 3 --variant bal:PF_FORM=5 --variant lean:PF_FORM=6
}

# Sixth pass: the harness's new flags on the GPU, the merge-grid change's
# parity (config 4, shards), and the default bench line with the lean prefill.
pass_f() {
  run t_harness 600 python -u -m pytest tests/test_harness.py -x -q --timeout 300 --timeout-method thread -m gpu
  run t_merge 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -x -q --timeout 300 --timeout-method thread -m gpu -k "config4 or merge or shard or workspace or config5"
  run ab_c4 300 python -u tools/ab_decode.py --workload config4 --rounds 5 --variant base:
  run bench 500 python -u bench.py
}

# Seventh pass: the one-launch prefill pre-pass -- prefill parity, harness,
# the bench line.
pass_g() {
  run t_g 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py tests/test_harness.py -x -q --timeout 300 --timeout-method thread -m gpu -k "pf or prefill or harness or flags"
  run bench 500 python -u bench.py
}

# Eighth pass: rocprofv3 kernel stats of config 4, the 8-rank config-5 shard
# and the prefill plan (the pre-pass launch vs the body), to size the merge
# launch and the pre-pass.
pass_h() {
  local Q="--no-prefill --no-scale-ref --no-cpu-baseline --no-copy-peak --steps 100 --warmup 10"
  run kt_c4 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6h_c4 -o run -- python3 -u bench.py $Q --kv-type q4_0 --heads 32 --kv-heads 8 --kv-len 8192
  run kt_s8 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6h_s8 -o run -- python3 -u bench.py $Q --workload config5 --heads 4 --kv-heads 4
  run kt_pf 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6h_pf -o run -- python3 -u bench.py --prefill-only
}
# Ninth pass: plain-load second-launch merges (parity, same-box A/B on config
# 4, config 5 and its 8-rank shard), the batched mask-flags loads (prefill
# parity), the prefill workgroup timeline (stamps build).
pass_i() {
  run t_i 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -x -q --timeout 300 --timeout-method thread -m gpu -k "merge_forms or pf or prefill or flags or config4 or config5"
  run ab_plain_c4 300 python -u tools/ab_decode.py --workload config4 --rounds 6 --variant base: --variant plain:MERGE_PLAIN=2
  run ab_plain_c5 300 python -u tools/ab_decode.py --workload config5 --rounds 6 --variant base: --variant plain:MERGE_PLAIN=2
  run ab_plain_s8 300 python -u tools/ab_decode.py --workload config5_s8 --rounds 6 --variant base: --variant plain:MERGE_PLAIN=2
  run st_pf_zm 200 python -u tools/pf_stamps.py --kv-type q8_0 --mask-zero
  run st_pf_f16 200 python -u tools/pf_stamps.py --kv-type f16 --no-mask
  run ab_pf_q8z 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 5 --variant base:
}
# Tenth pass: the DMA helper's M0 operand (every kernel's LDS-DMA issue: 2
# scalar instructions fewer per DMA) -- the whole GPU suite, then same-box A/B
# against the round-5 save / restore form (lib/libfattn_m0save.so), processes
# alternating.
pass_j() {
  run t_j 900 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu
  for r in 1 2; do
    for L in libfattn.so libfattn_m0save.so; do
      FATTN_LIB=$L run ab_m0_pf_${L%.so}_$r 200 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 2 --variant $L:
      FATTN_LIB=$L run ab_m0_c3_${L%.so}_$r 200 python -u tools/ab_decode.py --workload config3 --rounds 2 --variant $L:
      FATTN_LIB=$L run ab_m0_c5_${L%.so}_$r 200 python -u tools/ab_decode.py --workload config5 --rounds 2 --variant $L:
    done
  done
}
# Eleventh pass: f16 chunk partials for the second-launch merges -- the merge
# and batched-decode tests, then same-box A/B against f32 partials on config
# 4, config 5 and its 8- / 4-rank shards; the prefill line's new median.
pass_k() {
  run t_k 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -q --timeout 300 --timeout-method thread -m gpu -k "merge or bd or config4 or config5 or shard or multirow or workspace or masked or nan"
  run ab_p16_c5 300 python -u tools/ab_decode.py --workload config5 --rounds 6 --variant f16: --variant f32:PART_F16=1
  run ab_p16_s8 300 python -u tools/ab_decode.py --workload config5_s8 --rounds 6 --variant f16: --variant f32:PART_F16=1
  run ab_p16_s4 300 python -u tools/ab_decode.py --workload config5_s4 --rounds 6 --variant f16: --variant f32:PART_F16=1
  run ab_p16_c4 300 python -u tools/ab_decode.py --workload config4 --rounds 6 --variant f16: --variant f32:PART_F16=1
  run ab_p16_s2 300 python -u tools/ab_decode.py --workload config5_s2 --rounds 4 --variant f16: --variant f32:PART_F16=1
}
# Twelfth pass: the GQA one-row decode with one q head per tile (config 4) --
# parity, same-box A/B against the packed plan; the merge tests after the
# f16-partial policy change.
pass_l() {
  run t_l 900 python -u -m pytest tests/test_gpu_extra.py tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -m gpu -k "gqa_unpacked or merge_forms or config4 or shard"
  run ab_unpack_c4 300 python -u tools/ab_decode.py --workload config4 --rounds 6 --variant packed: --variant unpack:GQA_UNPACK=2 --variant unpack_s2:GQA_UNPACK=2,SPLIT_STEPS=2 --variant unpack_w4:GQA_UNPACK=2,SPLIT_WAVES=4
}
# Thirteenth pass: config 5's 64-sequence reading (bench side line) -- parity
# at a reduced cache, the bench line on the final kernels.
pass_m() {
  run t_m 300 python -u -m pytest tests/test_gpu_extra.py -q --timeout 300 --timeout-method thread -m gpu -k "seq64 or gqa_unpacked"
  run bench 600 python -u bench.py
}
# Fourteenth pass: with f16 partials, does the batched-decode role form now
# beat the split kernel on the 4- and 8-rank config-5 shards?
pass_n() {
  run ab_bd_s8 300 python -u tools/ab_decode.py --workload config5_s8 --rounds 6 --variant auto: --variant bdp:BD=3 --variant bd:BD=2
  run ab_bd_s4 300 python -u tools/ab_decode.py --workload config5_s4 --rounds 6 --variant auto: --variant bdp:BD=3 --variant bd:BD=2
}
# Fifteenth pass: config 5 (bdp) variants around the f16-partial plan: the
# in-kernel merge (f32 sc1 partials), plain workgroup order.
pass_o() {
  run ab_c5_var 400 python -u tools/ab_decode.py --workload config5 --rounds 6 --variant auto: --variant inkernel:MERGE_IN_KERNEL=1 --variant plainxcd:BD_XCD=1 --variant f32:PART_F16=1
}
# Sixteenth pass: config 5's bdp timeline on the f16-partial tree (stamps build).
pass_p() {
  run st_bdp_c5 200 python -u tools/stamps_bd.py --form bdp --heads 32 --kv-len 4096 --n-q 64
}
# Seventeenth pass: the lean loop's ring slots carried (no mod-3 divisions)
# and its K / V DMA opened by s_nop 0 (loop-invariant descriptors, audited) --
# prefill parity, then processes alternating libfattn.so and the previous
# tree's libfattn_prev.so.
pass_q() {
  run t_q 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -q --timeout 300 --timeout-method thread -m gpu -k "pf or prefill"
  for r in 1 2 3; do
    for L in libfattn.so libfattn_prev.so; do
      FATTN_LIB=$L run ab_q_z_${L%.so}_$r 200 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 2 --variant $L:
      FATTN_LIB=$L run ab_q_f_${L%.so}_$r 200 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 2 --variant $L:
    done
  done
}
# Eighteenth pass (reverted change): bdp's prologue issuing raw 0 and 1 only
# before raw 0's dequantisation -- batched-decode parity, then processes
# alternating libfattn.so and the previous tree's libfattn_prev.so.
pass_r() {
  run t_r 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -q --timeout 300 --timeout-method thread -m gpu -k "bd or config5 or batched or shard"
  for r in 1 2 3; do
    for L in libfattn.so libfattn_prev.so; do
      FATTN_LIB=$L run ab_r_c5_${L%.so}_$r 200 python -u tools/ab_decode.py --workload config5 --rounds 2 --variant $L:
      FATTN_LIB=$L run ab_r_s2_${L%.so}_$r 200 python -u tools/ab_decode.py --workload config5_s2 --rounds 2 --variant $L:
    done
  done
}
# Nineteenth pass: how much of the oracle bar the f16 chunk partials use.
pass_s() {
  run err_part 300 python -u tools/err_part.py
}
# Twentieth pass (reverted change): lean2 (PF_FORM 7: chains from 0, row sums
# by MFMA) -- the prefill parity suite (every form), then same-box A/B against
# lean (6).
pass_t() {
  run t_t 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -q --timeout 300 --timeout-method thread -m gpu -k "pf or prefill"
  run ab_l2_q8z 400 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 6 --variant lean:PF_FORM=6 --variant lean2:PF_FORM=7
  run ab_l2_f16 400 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 6 --variant lean:PF_FORM=6 --variant lean2:PF_FORM=7
}
# Twenty-first pass: f16 partials for the multi-query merge (D = 256) --
# parity, then same-box A/B on the config-5 shape at D = 256.
pass_u() {
  run t_u 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -m gpu -k "mq"
  run ab_mq16 300 python -u tools/ab_decode.py --workload config5_d256 --rounds 6 --variant f32: --variant f16:PART_F16=2
}
# Twenty-second pass: the merge forms at D = 64 / 80 / 96 (f16 partial paths).
pass_v() {
  run t_v 600 python -u -m pytest tests/test_gpu_extra.py -q --timeout 300 --timeout-method thread -m gpu -k "merge_forms"
}
# Twenty-third pass (reverted change): the prefill bodies without mask values issuing K 0-2
# before Q's loads -- prefill parity, then processes alternating libfattn.so
# and the previous tree's libfattn_prev.so.
pass_w() {
  run t_w 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -q --timeout 300 --timeout-method thread -m gpu -k "pf or prefill"
  for r in 1 2 3; do
    for L in libfattn.so libfattn_prev.so; do
      FATTN_LIB=$L run ab_w_z_${L%.so}_$r 200 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 2 --variant $L:
      FATTN_LIB=$L run ab_w_f_${L%.so}_$r 200 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 2 --variant $L:
    done
  done
}
# Twenty-fourth pass: the lean body's S^T chains as asm MFMAs into VGPRs with
# Q^T's operands in AGPRs (no accumulator reads) -- prefill parity, then
# processes alternating libfattn.so and the previous tree's libfattn_prev.so.
pass_x() {
  run t_x 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -q --timeout 300 --timeout-method thread -m gpu -k "pf or prefill"
  for r in 1 2 3; do
    for L in libfattn.so libfattn_prev.so; do
      FATTN_LIB=$L run ab_x_z_${L%.so}_$r 200 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 2 --variant $L:
      FATTN_LIB=$L run ab_x_f_${L%.so}_$r 200 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 2 --variant $L:
    done
  done
}
# Twenty-fifth pass: the same change in the stamps build (cycles per tile,
# both lean bodies), new form against FATTN_PF4_SAGPR (the committed one).
pass_y() {
  for r in 1 2; do
    for L in libfattn_stnew.so libfattn_stold.so; do
      FATTN_LIB=$L run st_y_z_${L%.so}_$r 200 python -u tools/pf_stamps.py --kv-type q8_0 --mask-zero
      FATTN_LIB=$L run st_y_f_${L%.so}_$r 200 python -u tools/pf_stamps.py --kv-type f16 --no-mask
    done
  done
}
# Twenty-sixth pass: the masked prefill body's S^T chains in VGPRs too (its
# accumulator reads gone) -- prefill parity, then stamps (libfattn_stnew.so /
# libfattn_stold.so, the tree before) and processes alternating libfattn.so /
# libfattn_prev.so on the random mask.
pass_z() {
  run t_z 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -q --timeout 300 --timeout-method thread -m gpu -k "pf or prefill"
  for L in libfattn_stnew.so libfattn_stold.so; do
    FATTN_LIB=$L run st_z_r_${L%.so} 200 python -u tools/pf_stamps.py --kv-type q8_0
  done
  for r in 1 2 3; do
    for L in libfattn.so libfattn_prev.so; do
      FATTN_LIB=$L run ab_z_r_${L%.so}_$r 200 python -u tools/ab_prefill.py --kv q8_0 --mask random --rounds 2 --variant $L:
    done
  done
}
"$@"
