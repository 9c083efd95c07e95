#!/bin/bash
# Round 5's one-off GPU passes, one function per pass (formerly
# tools/gpu_r5_<pass>.sh): bash tools/gpu_r5.sh <pass>
source tools/gpu_round.sh
export TMPDIR=/tmp

# Round 5, first GPU pass: the GPU suite (KAT through the kernels, the world-1
# RCCL bench path, speculative merge / XCD order, prefill staging and the
# one-wave-per-SIMD body), then same-box A/Bs (config 3 options; prefill forms).
pass_a() {
  run tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
  run ab_cfg3 300 python -u tools/ab_decode.py --workload config3 --rounds 6 \
      --variant base: --variant spec:SPLIT_SPEC=2 --variant xcd:SPLIT_XCD=2 --variant spec_xcd:SPLIT_SPEC=2,SPLIT_XCD=2
  run ab_pf_zero 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 2 \
      --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2 --variant inkernel:PF_STAGE=1,PF_FORM=1
}

# Round 5, second GPU pass: the one-wave-per-SIMD prefill body after the
# branch-free / immediate-offset rework, the XCD-order default, then a
# same-box prefill A/B.
pass_b() {
  run tests_sel 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      -k "pf or xcd or row_merge or workspace_not_zeroed or kat or nccl"
  run ab_pf_zero 400 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 3 \
      --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2 --variant inkernel:PF_STAGE=1,PF_FORM=1
  run ab_pf_random 300 python -u tools/ab_prefill.py --kv q8_0 --mask random --rounds 2 \
      --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2
}

# Round 5, third GPU pass: fattn_pf4_kernel row-level diagnostic, then the
# default bench line of the current tree.
pass_c() {
  run dbg_pf4 200 python -u tools/dbg_pf4.py
  run bench 500 python -u bench.py
}

# Round 5, fourth GPU pass: fattn_pf4_kernel row-level diagnostic over
# diagnostic builds (lib/libfattn_d*.so: plain adds, no scheduling groups, no
# opaque bases, shuffle reductions, all four) to localise its parity failure.
pass_d() {
  for v in dadd dsgb dopq dshf dall; do
    FATTN_LIB=libfattn_$v.so run dbg_$v 120 python -u tools/dbg_pf4.py
  done
}

# Round 5, fifth GPU pass: fattn_pf4_kernel with plain row-sum adds -- its
# parity tests (bit-identical to the 8-wave form, oracle), then the prefill A/B
# of the three bodies (Q8_0 staged zero mask, f16 no mask).
pass_e() {
  run pf_tests 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pf4 or pf_sweep or pf_staged or pf_prefill"
  run ab_pf_q8 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2 --variant pf4s1:PF_FORM=3
  run ab_pf_f16 300 python -u tools/ab_prefill.py --kv f16 --mask none --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2 --variant pf4s1:PF_FORM=3
}

# Round 5, sixth GPU pass: pf4 parity after the contraction fix; same-box A/B of
# the multi-row split merges (second launch vs last-arriving workgroup, XCD
# order, chunk size) on config 4 and the config-5 4- and 8-rank shards.
pass_f() {
  run pf4_tests 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pf4"
  V="--variant base: --variant fused:SPLIT_MERGE=1 --variant xcd:SPLIT_XCD=2 --variant fx:SPLIT_MERGE=1,SPLIT_XCD=2"
  run ab_cfg4 300 python -u tools/ab_decode.py --workload config4 --rounds 5 $V \
      --variant fx512:SPLIT_MERGE=1,SPLIT_XCD=2,kv_chunk=512 --variant fx1024:SPLIT_MERGE=1,SPLIT_XCD=2,kv_chunk=1024
  run ab_s8 300 python -u tools/ab_decode.py --workload config5_s8 --rounds 5 $V \
      --variant fx512:SPLIT_MERGE=1,SPLIT_XCD=2,kv_chunk=512
  run ab_s4 300 python -u tools/ab_decode.py --workload config5_s4 --rounds 5 $V \
      --variant fx512:SPLIT_MERGE=1,SPLIT_XCD=2,kv_chunk=512
  # bdp image swizzles (round 5): parity, then config 5 new vs old swizzles (two libraries, alternating processes)
  run bdp_tests 300 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu -k "bdp"
  FATTN_LIB=libfattn_raw64.so run bdp_tests_raw64 300 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu -k "bdp"
  for i in 1 2; do
    run ab_c5_new_$i 200 python -u tools/ab_decode.py --workload config5 --rounds 3 --variant new:
    run ab_c5_old_$i 200 python -u tools/ab_decode.py --workload config5 --rounds 3 --variant old: --lib libfattn_oldswz.so
    run ab_c5_raw64_$i 200 python -u tools/ab_decode.py --workload config5 --rounds 3 --variant raw64: --lib libfattn_raw64.so
  done
  run nccl_world1 400 python -u -m pytest tests/test_rehearsal.py -x -q --timeout 300 --timeout-method thread -m gpu -k "nccl"
  # D = 256 (verdict r04 missing 2): batched decode (config-5 shape) multi-query vs split kernel; prefill
  run ab_d256_dec 300 python -u tools/ab_decode.py --workload config5 --D 256 --rounds 3 --variant mq: --variant split:MQ_DISABLE=1
  run ab_d256_pf 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --D 256 --H 16 --rounds 2 --variant auto:
  run ab_d256_pf16 300 python -u tools/ab_prefill.py --kv f16 --mask none --D 256 --H 16 --rounds 2 --variant auto:
}

# Round 5: kernel stats of the staged prefill (stage + flags + f16 body), then
# the instruction-mix / LDS counters of the prefill body and of the role-form
# batched decode (config 5, new image swizzles) -- the round-4 counter sets.
pass_g() {
  F=gpurun_out/r5g
  mkdir -p $F
  run pfstats 200 timeout -s KILL 190 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g_prof/pf -o pf -- python3 bench.py --prefill-only
  A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"
  P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
  run pfA 200 timeout -s KILL 190 rocprofv3 --output-format csv --pmc $A -d gpurun_out/r5g_pmc/pfA -o a -- python3 bench.py --prefill-only
  run pfB 200 timeout -s KILL 190 rocprofv3 --output-format csv --pmc $P -d gpurun_out/r5g_pmc/pfB -o b -- python3 bench.py --prefill-only
  B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 20 --warmup 5 --workload config5"
  run c5A 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc $A -d gpurun_out/r5g_pmc/c5A -o a -- python3 bench.py $B
  run c5B 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc $P -d gpurun_out/r5g_pmc/c5B -o b -- python3 bench.py $B
  python tools/pmc_summary.py --kernel fattn_pf_kernel --mfma $(find gpurun_out/r5g_pmc/pfA gpurun_out/r5g_pmc/pfB -name "*counter_collection.csv") > $F/counters_prefill.txt 2>&1
  python tools/pmc_summary.py --kernel fattn_bdp_kernel --mfma $(find gpurun_out/r5g_pmc/c5A gpurun_out/r5g_pmc/c5B -name "*counter_collection.csv") > $F/counters_cfg5_bdp.txt 2>&1
  python tools/kstats.py $(find gpurun_out/r5g_prof/pf -name "*kernel_stats.csv") > $F/prefill_kernel_stats.txt 2>&1 || true
  cat $F/counters_prefill.txt $F/counters_cfg5_bdp.txt $F/prefill_kernel_stats.txt
  # per-phase cycles of the 8-wave f16 body (stamps build), no mask
  run pf_stamps_f16 200 python -u tools/pf_stamps.py --no-mask --kv-type f16
}

# Round 5: the pipelined one-wave-per-SIMD prefill schedule (FATTN_OPT_PF_FORM
# = 4): row diagnostic, parity (bit-identical to the 8-wave body), prefill A/B.
pass_h() {
  run dbg_pf4p 200 python -u tools/dbg_pf4.py
  run pf4p_tests 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pf4 or pf_sweep"
  run ab_pfp_f16 300 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4
  run ab_pfp_q8 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4
  run ab_pfp_q8r 300 python -u tools/ab_prefill.py --kv q8_0 --mask random --rounds 2 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4
}

# Round 5: per-phase cycle stamps of the pipelined prefill body (stamps build),
# f16 no mask and Q8_0 staged random mask, and of the 8-wave body beside it.
pass_i() {
  run st_pf4p_f16 200 python -u tools/pf_stamps.py --no-mask --kv-type f16
  run st_pf4p_q8 200 python -u tools/pf_stamps.py --kv-type q8_0
  run st_pf8_f16 200 python -u tools/pf_stamps.py --no-mask --kv-type f16 --form 1
}

# Round 5: pipelined prefill with its operand reads streamed inside the steps:
# parity, stamps, same-box A/B against the 8-wave body.
pass_j() {
  run pf4p_tests 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pf4 or pf_sweep or pf_prefill or pf_staged"
  run st_pf4p_f16 200 python -u tools/pf_stamps.py --no-mask --kv-type f16
  run st_pf4p_q8 200 python -u tools/pf_stamps.py --kv-type q8_0
  run ab_pfp_f16 300 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4
  run ab_pfp_q8 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4
}

# Round 5: pipelined prefill DMA / operand-read placement variants (libraries
# built by `make variant`): parity per library, then alternating same-box A/B.
#   base  V_j DMA in A's exponential steps 1-13, K_{j+1} first reads in B 28-31
#   vl    V_j DMA in A's max steps 17-29          (-DFATTN_PF4_VDMA_LATE)
#   ke    K_{j+1} first reads in B steps 5-8      (-DFATTN_PF4_KREAD_EARLY)
#   vlke  both
pass_k() {
  K="pf4_bit_identical or pf_staged"
  run t_base 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "$K"
  for v in vl ke vlke; do
    FATTN_LIB=libfattn_$v.so run t_$v 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "$K"
  done
  for i in 1 2; do
    for v in base vl ke vlke; do
      L=libfattn_$v.so; [ $v = base ] && L=libfattn.so
      FATTN_LIB=$L run ab_f16_${v}_$i 200 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 3 --variant $v:PF_FORM=4
      FATTN_LIB=$L run ab_q8_${v}_$i 200 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 3 --variant $v:PF_FORM=4
    done
  done
  grep -h "median" gpurun_out/ab_f16_*.log gpurun_out/ab_q8_*.log
}

# config-5 shards (4 / 8 heads per rank): kernel families and chunk sizes
pass_l() {
  V="--variant base: --variant bdp:BD=3 --variant bd:BD=2 --variant mq:MQ_MIN_ROWS=64 --variant c128:kv_chunk=128 --variant w8:SPLIT_WAVES=8"
  run ab_s8_fam 300 python -u tools/ab_decode.py --workload config5_s8 --rounds 3 $V
  run ab_s4_fam 300 python -u tools/ab_decode.py --workload config5_s4 --rounds 3 $V
}

# config-5 shards: split-kernel waves / chunk / steps, and where the time goes
pass_m() {
  V="--variant base: --variant w8:SPLIT_WAVES=8 --variant w8c256:SPLIT_WAVES=8,kv_chunk=256 --variant w8c1024:SPLIT_WAVES=8,kv_chunk=1024 --variant w16:SPLIT_WAVES=16 --variant w8i2:SPLIT_WAVES=8,SPLIT_INFLIGHT=2"
  for w in config5_s8 config5_s4 config5_s2; do
    run ab_${w}_w 300 python -u tools/ab_decode.py --workload $w --rounds 3 $V
  done
  run kt_s8 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5m_kt8 -o kt -- python3 tools/ab_decode.py --workload config5_s8 --rounds 1 --variant base:
  python tools/kstats.py $(find gpurun_out/r5m_kt8 -name "*kernel_stats.csv") > gpurun_out/kt_s8_summary.txt 2>&1 || true
  cat gpurun_out/kt_s8_summary.txt
}

# the planner's 8-wave rule for multi-row split tiles from 16 steps per CU:
# parity of the split paths, then auto vs forced 4 waves
pass_n() {
  run t_split 600 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu -k "split or shard or sweep or config4 or config2"
  for w in config5_s8 config5_s4 config5_s2 config4 config2; do
    run ab_${w}_n 300 python -u tools/ab_decode.py --workload $w --rounds 3 --variant auto: --variant w4:SPLIT_WAVES=4
  done
}

# config 3 (the headline decode) re-swept on the round-5 kernel: chunk, waves, in flight
pass_o() {
  V="--variant auto: --variant c256:kv_chunk=256 --variant c1024:kv_chunk=1024 --variant w4:SPLIT_WAVES=4 --variant w16:SPLIT_WAVES=16 --variant i2:SPLIT_INFLIGHT=2 --variant plain:SPLIT_XCD=1 --variant wm1:SPLIT_WAVE_MERGE=1"
  run ab_config3_o 300 python -u tools/ab_decode.py --workload config3 --rounds 5 $V
}

# the balanced pipelined prefill (FATTN_OPT_PF_FORM = 5): row diagnostic,
# parity, stamps, same-box A/B against the pipelined (4) and 8-wave (1) bodies
pass_p() {
  run dbg_bal 200 python -u tools/dbg_pf4.py
  run t_bal 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pf4 or pf_sweep or pf_prefill or pf_staged"
  run st_bal_f16 200 python -u tools/pf_stamps.py --no-mask --kv-type f16 --form 5
  run st_bal_q8 200 python -u tools/pf_stamps.py --kv-type q8_0 --form 5
  run ab_bal_f16 300 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4 --variant bal:PF_FORM=5
  run ab_bal_q8 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4 --variant bal:PF_FORM=5
}

# where the balanced body's phase time goes: stamps of diagnostic builds
# without the vector pieces (snv), without the in-loop DMA (snd), without both
# (snb); outputs wrong, cycles only (make variant VAR=snv VFLAGS="-DFATTN_STAMPS
# -DFATTN_PF4_DIAG_NO_VALU", ...)
pass_q() {
  run st_q_full 200 python -u tools/pf_stamps.py --no-mask --kv-type f16 --form 5
  for v in snv snd snb; do
    FATTN_LIB=libfattn_$v.so run st_q_$v 200 python -u tools/pf_stamps.py --no-mask --kv-type f16 --form 5
  done
}

# a second box for the prefill body choice (forms 1 / 4 / 5, 5 rounds), and
# where the 4-rank shard's step goes on the new plan (rocprofv3)
pass_r() {
  run ab_r_f16 300 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 5 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4 --variant bal:PF_FORM=5
  run ab_r_q8 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 5 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4 --variant bal:PF_FORM=5
  run ab_r_q8r 300 python -u tools/ab_prefill.py --kv q8_0 --mask random --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4 --variant bal:PF_FORM=5
  run kt_s4 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5r_kt4 -o kt -- python3 tools/ab_decode.py --workload config5_s4 --rounds 1 --variant auto:
  python tools/kstats.py $(find gpurun_out/r5r_kt4 -name "*kernel_stats.csv") > gpurun_out/kt_s4_summary.txt 2>&1 || true
  cat gpurun_out/kt_s4_summary.txt
}

# would a pre-transposed V image pay?  a diagnostic build reading each V^T
# operand with ONE ds_read_b128 (outputs wrong; lib/libfattn_vb128.so from
# -DFATTN_PF4_DIAG_VB128, kept out of the tree) against the shipped body
pass_s() {
  for i in 1 2 3; do
    run ab_s_base_$i 200 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 3 --variant bal:PF_FORM=5
    FATTN_LIB=libfattn_vb128.so run ab_s_vb128_$i 200 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 3 --variant vb128:PF_FORM=5
  done
  grep -h median gpurun_out/ab_s_*.log
}

# config 3: wave priorities and the masked-step skip, re-measured on the round-5 kernel
pass_t() {
  run ab_config3_t 300 python -u tools/ab_decode.py --workload config3 --rounds 7 --variant auto: --variant prio_none:SPLIT_PRIO=1 --variant prio_issue:SPLIT_PRIO=2 --variant noskip:SPLIT_SKIP=1
}

# config 4 (Q4_0, GQA 32/8, N 8192): chunk / waves around the auto plan, merge launch kept
pass_u() {
  run ab_config4_u 300 python -u tools/ab_decode.py --workload config4 --rounds 5 --variant auto: --variant c512:kv_chunk=512 --variant w8:SPLIT_WAVES=8 --variant w8c512:SPLIT_WAVES=8,kv_chunk=512 --variant c128:kv_chunk=128 --variant xcd:SPLIT_XCD=2
}

# D = 256 on the multi-query kernel: rows per wave and chunk around the auto plan
pass_v() {
  run ab_d256_pf_v 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --D 256 --H 16 --rounds 2 --variant auto: --variant r16:MQ_ROWS_PER_WAVE=16 --variant r32:MQ_ROWS_PER_WAVE=32
  run ab_d256_dec_v 300 python -u tools/ab_decode.py --workload config5 --D 256 --rounds 3 --variant auto: --variant r16:MQ_ROWS_PER_WAVE=16 --variant r32:MQ_ROWS_PER_WAVE=32 --variant c256:kv_chunk=256 --variant c1024:kv_chunk=1024
}

case "$1" in
  a|b|c|d|e|f|g|h|i|j|k|l|m|n|o|p|q|r|s|t|u|v) pass_$1 ;;
  *) echo "usage: bash tools/gpu_r5.sh {a|b|c|d|e|f|g|h|i|j|k|l|m|n|o|p|q|r|s|t|u|v}"; exit 2 ;;
esac
