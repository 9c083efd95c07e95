"""CPU: the C-ABI library loads, exports every symbol include/fattn.h declares,
and validates arguments without touching a GPU (no compute calls here)."""
import ctypes as C
import os
import re

import pytest

import fattn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols(names=("fattn.h", "fattn_debug.h")):
    """The functions include/fattn.h (the drop-in ABI) and include/fattn_debug.h
    (its diagnostics) declare."""
    syms = set()
    for n in names:
        src = open(os.path.join(ROOT, "include", n)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        syms |= set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(fattn_\w+)\s*\(", src, flags=re.M))
    return sorted(syms)


def test_drop_in_header_lists_no_diagnostics():
    """include/fattn.h holds the drop-in entry points only: the planner
    overrides, fattn_describe and fattn_ext_events live in fattn_debug.h."""
    main = header_symbols(("fattn.h",))
    assert "fattn_ext" in main and "fattn_row" in main and "fattn_cpy" in main
    for s in ("fattn_set_option", "fattn_describe", "fattn_ext_events"):
        assert s not in main and s in header_symbols(("fattn_debug.h",))
    assert "FATTN_OPT_" not in open(os.path.join(ROOT, "include", "fattn.h")).read()


def test_header_symbols_parsed():
    syms = header_symbols()
    assert "fattn_ext" in syms and "fattn_quantize" in syms and len(syms) == len(fattn.EXPORTS)
    assert set(syms) == set(fattn.EXPORTS)


def test_library_exports_every_header_symbol():
    L = fattn.lib()
    for s in header_symbols():
        assert hasattr(L, s), s


def test_nm_exports():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", fattn.LIB_PATH], capture_output=True, text=True).stdout
    for s in header_symbols():
        assert re.search(rf"\bT {s}$", out, flags=re.M), s


def test_strerror_and_sizes():
    assert fattn.strerror(0) == "ok"
    assert "stride" in fattn.strerror(-4)
    assert fattn.row_size(fattn.TYPE_Q8_0, 128) == 136
    assert fattn.row_size(fattn.TYPE_Q4_0, 128) == 72
    assert fattn.row_size(fattn.TYPE_F16, 128) == 256
    assert fattn.row_size(fattn.TYPE_Q8_0, 100) == 0
    assert fattn.lib().fattn_version().startswith(b"fattn-gfx950")


def _params(D=128, NQ=1, H=32, Hkv=32, N=4096, kt=fattn.TYPE_Q8_0, kv_chunk=0, ptr=1 << 20, mask=True, vt=None):
    def view(t):
        rb = fattn.row_size(t, D)
        eb = 2 if t == fattn.TYPE_F16 else fattn.BLOCK_BYTES.get(t, 4)
        return fattn.View(ptr, t, (D, N, Hkv, 1), (eb, rb, rb * N, rb * N * Hkv))
    q = fattn.View(ptr, fattn.TYPE_F32, (D, NQ, H, 1), (4, H * D * 4, D * 4, NQ * H * D * 4))
    m = fattn.View(ptr, fattn.TYPE_F16, (N, NQ, 1, 1), (2, N * 2, N * 2 * NQ, N * 2 * NQ)) if mask else None
    return fattn.ext_params(q, view(kt), view(kt if vt is None else vt), m, ptr, 0.088, kv_chunk=kv_chunk)


def test_workspace_size_config3():
    p = _params()
    ws = fattn.workspace_size(p)
    # one-row tiles: 32 heads x n_chunks (>= 2) rows of D floats + (m, l) pairs
    # + one 256-B arrival counter per head
    assert ws > 0 and ws >= 32 * 2 * (128 * 4 + 8) + 32 * 256


@pytest.mark.parametrize("kw,want", [
    (dict(), ["8waves>", "grid(8,32,1)", "steps/slots 1"]),                                 # config 3
    (dict(N=2048, kt=fattn.TYPE_F16), ["f16,f16", "8waves>", "grid(8,32,1)"]),              # config 2
    (dict(H=32, Hkv=8, N=8192, kt=fattn.TYPE_Q4_0), ["4waves> + fattn_merge_kernel", "grid(32,8,1)"]),  # config 4
    (dict(NQ=64), ["fattn_bdp_kernel<q8_0", "+ fattn_bd_merge_kernel", "grid(8,32,1)"]),   # config 5, one GPU
    (dict(NQ=64, H=4, Hkv=4), ["fattn_split_kernel", "4waves> + fattn_merge_kernel"]),     # config 5, 8-rank shard
    (dict(NQ=64, H=8, Hkv=8), ["fattn_split_kernel", "8waves> + fattn_merge_kernel", "grid(8,32,1)"]),  # 4-rank shard
    (dict(NQ=64, H=16, Hkv=16), ["fattn_bdp_kernel", "+ fattn_bd_merge_kernel", "grid(16,16,1)"]),  # config 5, 2-rank shard
    (dict(NQ=256), ["fattn_bdp_kernel", "grid(2,128,1)"]),                                  # batched: 4 row tiles
    (dict(NQ=64, kt=fattn.TYPE_F16), ["fattn_bd_kernel<f16,D128", "+ fattn_bd_merge_kernel"]),  # config 5 shape, f16
    (dict(D=64, NQ=64, kt=fattn.TYPE_F16), ["fattn_bd_kernel<f16,D64"]),                    # f16 at D = 64 / 96
    (dict(D=96, NQ=64, kt=fattn.TYPE_F16), ["fattn_bd_kernel<f16,D96"]),
    (dict(NQ=64, H=24, Hkv=4), ["fattn_bdp_kernel<q8_0", "grid(8,28,1)"]),                  # GQA 6: 7 tiles of 10 queries
    (dict(NQ=64, H=4, Hkv=4, kt=fattn.TYPE_F16), ["fattn_split_kernel<f16,f16"]),           # f16, 8-rank shard
    (dict(NQ=8, H=32, Hkv=8), ["fattn_split_kernel", "+ fattn_merge_kernel"]),              # < 64 rows per kv head
    (dict(D=64, NQ=4096, H=32, Hkv=32), ["kv_stage_f16<q8_0> +", "fattn_pf_kernel<f16,D64"]),  # D = 64 prefill (staged)
    (dict(D=96, NQ=4096, H=32, Hkv=32), ["kv_stage_f16<q8_0> +", "fattn_pf_kernel<f16,D96"]),  # D = 96 prefill
    (dict(D=96, NQ=4096, H=32, Hkv=32, kt=fattn.TYPE_F16), ["fattn_pf_kernel<f16,D96"]),
    (dict(D=80, NQ=4096, H=32, Hkv=32, kt=fattn.TYPE_F16), ["fattn_pf_kernel<f16,D80"]),      # D = 80 prefill (f16)
    (dict(D=256, NQ=4096, H=16, Hkv=16), ["fattn_mq_kernel<q8_0,D256,4waves"]),              # D = 256 prefill
], ids=["config3", "config2", "config4", "config5", "config5_shard", "config5_shard4", "config5_shard2", "mq_nq256", "bd_f16", "bd_f16_d64", "bd_f16_d96",
        "bd_gqa6", "bd_f16_shard", "split_nq8_gqa", "pf_d64", "pf_d96", "pf_d96_f16", "pf_d80_f16", "mq_d256"])
def test_planner_picks(kw, want):
    """The plans the round-2 measurements chose, at 256 CUs:
    one-row tiles take 8 waves with the fused row merge; multi-row split tiles
    with 4+ chunks and batched-decode tiles merge in a second launch; long
    multi-row slices take twice the chunks; multi-row split tiles take 8 waves
    from 16 steps per CU (round 5: the 4-rank config-5 shard)."""
    d = fattn.describe(_params(**kw))
    for w in want:
        assert w in d, d


def test_bd_option_forms():
    """FATTN_OPT_BD: 2 = the all-waves form, 3 = the compute / build-role form
    (quantised K/V only; f16 keeps the all-waves form's image ring)."""
    with fattn.options({fattn.OPT_BD: 2}):
        assert fattn.describe(_params(NQ=64)).startswith("fattn_bd_kernel<q8_0")
    with fattn.options({fattn.OPT_BD: 3}):
        assert fattn.describe(_params(NQ=64, kt=fattn.TYPE_Q4_0)).startswith("fattn_bdp_kernel<q4_0")
        assert fattn.describe(_params(NQ=64, kt=fattn.TYPE_F16)).startswith("fattn_bd_kernel<f16")
        # head dim 64: the role form (quantised; f16 keeps the image ring)
        assert fattn.describe(_params(D=64, NQ=64)).startswith("fattn_bdp_kernel<q8_0,D64")
        assert fattn.describe(_params(D=64, NQ=64, kt=fattn.TYPE_F16)).startswith("fattn_bd_kernel<f16,D64")
    assert fattn.describe(_params(D=64, NQ=64)).startswith("fattn_bdp_kernel<q8_0,D64")  # (auto too)
    assert fattn.describe(_params(D=96, NQ=64, kt=fattn.TYPE_Q4_0)).startswith("fattn_bdp_kernel<q4_0,D96")
    with fattn.options({fattn.OPT_BD: 2}):  # (the all-waves form is D = 128 only: the multi-query kernel)
        assert fattn.describe(_params(D=64, NQ=64)).startswith("fattn_mq_kernel")
    with pytest.raises(Exception):
        fattn.set_option(fattn.OPT_BD, 4)


def test_bd_xcd_option():
    """FATTN_OPT_BD_XCD: 2 = XCD-grouped workgroup order for the batched-decode
    kernels when the grid is a multiple of 8 workgroups; other plans unchanged."""
    with fattn.options({fattn.OPT_BD_XCD: 2}):
        assert "(xcd order)" in fattn.describe(_params(NQ=64))                   # grid(8,32,1)
        assert "(xcd order)" in fattn.describe(_params())                        # config 3: split kernel (FATTN_OPT_SPLIT_XCD auto)
        d5 = fattn.describe(_params(NQ=64, H=5, Hkv=5, N=32768))             # grid(52,5,1): not a multiple of 8
        assert d5.startswith("fattn_bdp_kernel") and "(xcd order)" not in d5, d5
    with fattn.options({fattn.OPT_BD_XCD: 1}):
        assert "(xcd order)" not in fattn.describe(_params(NQ=64))
    assert "(xcd order)" in fattn.describe(_params(NQ=64))  # (the default)
    with pytest.raises(Exception):
        fattn.set_option(fattn.OPT_BD_XCD, 3)


def test_split_xcd_option():
    """FATTN_OPT_SPLIT_XCD: one-row tiles merged in the launch (config 3) take
    the XCD-grouped order by default; multi-row tiles (merge launch) stay
    plain unless forced; 1 = plain everywhere."""
    assert "(xcd order)" in fattn.describe(_params())                                   # config 3
    assert "(xcd order)" not in fattn.describe(_params(H=32, Hkv=8, N=8192, kt=fattn.TYPE_Q4_0))  # config 4
    with fattn.options({fattn.OPT_SPLIT_XCD: 1}):
        assert "(xcd order)" not in fattn.describe(_params())
    with fattn.options({fattn.OPT_SPLIT_XCD: 2}):
        assert "(xcd order)" in fattn.describe(_params(H=32, Hkv=8, N=8192, kt=fattn.TYPE_Q4_0))
    with pytest.raises(Exception):
        fattn.set_option(27, 2)  # the removed speculative-merge option


def test_merge_in_kernel_option():
    fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 1)
    try:
        d = fattn.describe(_params(NQ=64))
        assert "(in-kernel merge)" in d, d
        d4 = fattn.describe(_params(H=32, Hkv=8, N=8192, kt=fattn.TYPE_Q4_0))
        assert "4waves> (in-kernel merge)" in d4, d4
        ws1 = fattn.workspace_size(_params(NQ=64))
    finally:
        fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 0)
    ws0 = fattn.workspace_size(_params(NQ=64))
    assert ws1 == ws0 + 32 * 256  # one 256-B arrival line per tile for the in-kernel merge
    with pytest.raises(Exception):
        fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 2)  # rejected (FATTN_ERR_INVALID_ARG)


def test_split_merge_option_restores_fused_merge():
    fattn.set_option(fattn.OPT_SPLIT_MERGE, 1)
    try:
        d2 = fattn.describe(_params(NQ=8, H=4, Hkv=1))
    finally:
        fattn.set_option(fattn.OPT_SPLIT_MERGE, 0)
    assert "merge_kernel" not in d2, d2   # split kernel, 32 rows per kv head: fused merge


def test_pf_stagger_option_range():
    """FATTN_OPT_PF_STAGGER: bits 1-2 settable, the removed bit 0 and values
    past 7 rejected (include/fattn.h)."""
    for v in (0, 2, 4, 6):
        fattn.set_option(fattn.OPT_PF_STAGGER, v)
    fattn.set_option(fattn.OPT_PF_STAGGER, 2)
    for v in (1, 3, 8, -1):
        with pytest.raises(Exception):
            fattn.set_option(fattn.OPT_PF_STAGGER, v)


@pytest.mark.parametrize("kt,vt", [(fattn.TYPE_Q8_0, fattn.TYPE_F16), (fattn.TYPE_F16, fattn.TYPE_Q4_0),
                                   (fattn.TYPE_Q4_0, fattn.TYPE_Q8_0)])
@pytest.mark.parametrize("D,NQ", [(128, 1), (64, 64), (256, 4096)])
def test_mixed_kv_types_take_the_split_kernel(kt, vt, D, NQ):
    """Separate K and V cache types: the split kernel instantiated for the pair
    (never the single-type batched-decode, multi-query or prefill kernels)."""
    d = fattn.describe(_params(D=D, NQ=NQ, H=8, Hkv=8, N=2048, kt=kt, vt=vt))
    names = {fattn.TYPE_F16: "f16", fattn.TYPE_Q8_0: "q8_0", fattn.TYPE_Q4_0: "q4_0"}
    assert d.startswith(f"fattn_split_kernel<{names[kt]},{names[vt]},D{D},"), d


def test_mixed_kv_types_other_head_dims_rejected():
    p = _params(D=96, kt=fattn.TYPE_Q8_0, vt=fattn.TYPE_F16)
    assert fattn.workspace_size(p) == 0


@pytest.mark.parametrize("kt", [fattn.TYPE_Q8_0, fattn.TYPE_Q4_0])
def test_quant_k_with_transposed_f16_v_rejected(kt):
    """The transposed-V (flash_row_float.h) kernels exist for f16 K only: the
    planner refuses the pair instead of planning a launch that cannot run."""
    D, N, H = 128, 2048, 8
    p = _params(D=D, N=N, H=H, Hkv=H, kt=kt)
    # V f16 [Hkv][D][N]: nb0 = N * 2 (along D), nb1 = 2 (along N)
    vt = fattn.View(1 << 20, fattn.TYPE_F16, (D, N, H, 1), (N * 2, 2, D * N * 2, D * N * 2 * H))
    p.v = vt.c()
    assert fattn.workspace_size(p) == 0
    with pytest.raises(fattn.FattnError) as e:
        fattn.describe(p)
    assert e.value.code == -2  # FATTN_ERR_UNSUPPORTED_TYPE


def test_mq_min_rows_explicit_default_lifts_the_wide_gate():
    """An explicit FATTN_OPT_MQ_MIN_ROWS = 64 (the default's value) bypasses the
    rule that every chunk hold two 128-key tiles, as the header says."""
    p = _params(NQ=64, H=4, Hkv=4)  # config-5 8-rank shard: the split kernel by default
    assert fattn.describe(p).startswith("fattn_split_kernel"), fattn.describe(p)
    with fattn.options({fattn.OPT_MQ_MIN_ROWS: 64, fattn.OPT_BD: 1}):
        d = fattn.describe(p)
    assert d.startswith("fattn_mq_kernel"), d
    assert fattn.describe(p).startswith("fattn_split_kernel")  # restored


def test_merge_plain_option():
    """FATTN_OPT_MERGE_PLAIN (f32 partials, FATTN_OPT_PART_F16 = 1): 0 (auto)
    and 1 keep the second-launch merges' sc1 loads, 2 names the plain-load
    kernels in the plan; out of range is rejected."""
    p = _params(NQ=1, H=32, Hkv=8, N=8192, kt=fattn.TYPE_Q4_0)  # config 4: 4-row tiles, second-launch merge
    with fattn.options({fattn.OPT_PART_F16: 1}):
        assert "fattn_merge_kernel" in fattn.describe(p) and "(plain)" not in fattn.describe(p)
        with fattn.options({fattn.OPT_MERGE_PLAIN: 2}):
            assert "fattn_merge_kernel(plain)" in fattn.describe(p)
        with fattn.options({fattn.OPT_MERGE_PLAIN: 1}):
            assert "(plain)" not in fattn.describe(p)
    for bad in (-1, 3):
        with pytest.raises(Exception):
            fattn.set_option(fattn.OPT_MERGE_PLAIN, bad)


def test_part_f16_option():
    """FATTN_OPT_PART_F16: the second-launch merges take f16 partials by
    default for batched decode and for split tiles of 8+ rows (config 4's
    4-row tiles keep f32: measured slower), never at D = 64 or with the
    in-kernel merge; 1 forces f32, 2 f16; out of range is rejected."""
    c4 = _params(NQ=1, H=32, Hkv=8, N=8192, kt=fattn.TYPE_Q4_0)
    c5 = _params(NQ=64, H=32, Hkv=32, N=4096, kt=fattn.TYPE_Q8_0)
    s8 = _params(NQ=64, H=4, Hkv=4, N=4096, kt=fattn.TYPE_Q8_0)
    assert "f16 partials" not in fattn.describe(c4), fattn.describe(c4)
    with fattn.options({fattn.OPT_PART_F16: 2}):
        assert "fattn_merge_kernel(f16 partials)" in fattn.describe(c4)
    for p, kern in ((s8, "fattn_merge_kernel(f16 partials)"), (c5, "fattn_bd_merge_kernel(f16 partials)")):
        assert kern in fattn.describe(p), fattn.describe(p)
        with fattn.options({fattn.OPT_PART_F16: 1}):
            assert "f16 partials" not in fattn.describe(p)
        with fattn.options({fattn.OPT_PART_F16: 2}):
            assert kern in fattn.describe(p)
    assert "f16 partials" not in fattn.describe(_params(D=64, NQ=1, H=32, Hkv=8, N=8192, kt=fattn.TYPE_Q4_0))
    for bad in (-1, 3):
        with pytest.raises(Exception):
            fattn.set_option(fattn.OPT_PART_F16, bad)


def test_pf_form_option():
    """The prefill body over f16 rows at D = 128: the lean balanced
    one-wave-per-SIMD body (chains started from -m / c) by default and with
    FATTN_OPT_PF_FORM = 6, the 8-wave body with 1, the pipelined one with 4,
    the balanced one with 5; 2 and 3 (round 5's
    unpipelined one-wave-per-SIMD forms) were removed and are rejected; other
    head dims keep the 8-wave body."""
    p = _params(NQ=4096, kt=fattn.TYPE_F16)
    assert "fattn_pf4_kernel(lean)<f16,D128" in fattn.describe(p)
    want = {1: "fattn_pf_kernel<f16,D128", 4: "fattn_pf4_kernel(pipelined)<f16,D128",
            5: "fattn_pf4_kernel(balanced)<f16,D128", 6: "fattn_pf4_kernel(lean)<f16,D128"}
    for form, name in want.items():
        with fattn.options({fattn.OPT_PF_FORM: form}):
            assert name in fattn.describe(p), (form, fattn.describe(p))
    assert "fattn_pf_kernel<f16,D64" in fattn.describe(_params(NQ=4096, D=64, kt=fattn.TYPE_F16))
    for bad in (2, 3, 7):
        with pytest.raises(Exception):
            with fattn.options({fattn.OPT_PF_FORM: bad}):
                pass


def test_pf_stage_option_and_workspace():
    """Prefill over Q8_0 / Q4_0: staged to f16 rows in the workspace by default
    (2 x Hkv x N x D x 2 bytes more), dequantised in the kernel with
    FATTN_OPT_PF_STAGE = 1; f16 caches are never staged."""
    p = _params(NQ=4096)
    d = fattn.describe(p)
    assert d.startswith("pf_prepass[kv_stage_f16<q8_0> + pf_mask_flags] + fattn_pf4_kernel(lean)<f16,D128"), d
    ws = fattn.workspace_size(p)
    with fattn.options({fattn.OPT_PF_STAGE: 1}):
        d1 = fattn.describe(p)
        ws1 = fattn.workspace_size(p)
    assert d1.startswith("pf_prepass[pf_mask_flags] + fattn_pf_kernel<q8_0,D128"), d1
    assert ws == ws1 + 2 * 32 * 4096 * 128 * 2
    with fattn.options({fattn.OPT_PF_STAGE: 2}):
        assert "kv_stage_f16<q4_0>" in fattn.describe(_params(NQ=4096, kt=fattn.TYPE_Q4_0))
        assert "kv_stage" not in fattn.describe(_params(NQ=4096, kt=fattn.TYPE_F16))
    with pytest.raises(Exception):
        fattn.set_option(fattn.OPT_PF_STAGE, 3)


def test_mq_merge_launch_grid_limit():
    """A forced small KV chunk with many 64-row query tiles: the merge launch's
    grid.y (tiles x 4 subtiles) would pass 65535, so the plan does not split
    the KV sequence (one chunk, no merge launch, no workspace) instead of
    refusing; below the limit the requested chunk stands."""
    p = _params(NQ=64 * 20000, H=1, Hkv=1, N=1024, kv_chunk=256)
    with fattn.options({fattn.OPT_PF: 1, fattn.OPT_BD: 1}):
        d = fattn.describe(p)
        assert d.startswith("fattn_mq_kernel") and "merge" not in d, d
        assert "grid(1,5000,1)" in d, d  # (256-row tiles: 5000 x 16 subtiles)
        assert fattn.workspace_size(p) == 0
        small = _params(NQ=64 * 100, H=1, Hkv=1, N=1024, kv_chunk=256)
        d2 = fattn.describe(small)
        assert "fattn_mq_merge_kernel" in d2 and "grid(4,100,1)" in d2, d2


def test_pf_d80_needs_spans_within_2gib():
    """D = 80 prefill reads its padding dims from 2 GiB past the row offset:
    a cache whose head span passes 2 GiB takes the multi-query / split path."""
    ok = _params(D=80, NQ=4096, H=32, Hkv=32, kt=fattn.TYPE_F16)
    assert "fattn_pf_kernel<f16,D80" in fattn.describe(ok)
    big = _params(D=80, NQ=4096, H=32, Hkv=32, kt=fattn.TYPE_F16)
    nb1 = (1 << 19) + 256  # rows 512.25 KiB apart: the span passes 2 GiB
    big.k = fattn.View(1 << 20, fattn.TYPE_F16, (80, 4096, 32, 1), (2, nb1, 160, nb1 * 4096)).c()
    assert "fattn_pf_kernel" not in fattn.describe(big), fattn.describe(big)


def test_single_chunk_needs_no_workspace():
    assert fattn.workspace_size(_params(N=128)) == 0


@pytest.mark.parametrize("bad", [
    dict(D=80), dict(D=72, kt=fattn.TYPE_F16), dict(D=112, kt=fattn.TYPE_F16), dict(D=512), dict(H=30, Hkv=8),
    dict(N=0), dict(kt=fattn.TYPE_F32), dict(kt=5),
])
def test_rejects_invalid(bad):
    p = _params(**bad)
    assert fattn.workspace_size(p) == 0
    with pytest.raises(fattn.FattnError):
        fattn.flash_attn_ext(p, stream=0)


@pytest.mark.parametrize("ok", [dict(D=96), dict(D=96, kt=fattn.TYPE_Q4_0), dict(D=96, kt=fattn.TYPE_F16),
                                dict(D=80, kt=fattn.TYPE_F16)])
def test_accepts_head_dims_80_96(ok):
    """D = 96 for every K/V type, D = 80 for f16 K/V (80 is not
    a whole number of 32-element ggml blocks, so the Q8_0 row above is rejected)."""
    assert fattn.workspace_size(_params(**ok)) > 0


def test_d96_quant_needs_dword_rows():
    """D = 96 Q8_0 rows are 102 B: a [N][Hkv][row] cache (rows Hkv * 102 B apart,
    heads 102 B apart) cannot be moved in dwords -> FATTN_ERR_ALIGNMENT."""
    D, N, Hkv, ptr = 96, 256, 3, 1 << 20
    rb = fattn.row_size(fattn.TYPE_Q8_0, D)
    q = fattn.View(ptr, fattn.TYPE_F32, (D, 1, Hkv, 1), (4, Hkv * D * 4, D * 4, Hkv * D * 4))
    k = fattn.View(ptr, fattn.TYPE_Q8_0, (D, N, Hkv, 1), (34, rb * Hkv, rb, rb * Hkv * N))
    p = fattn.ext_params(q, k, k, None, ptr, 0.1)
    assert fattn.workspace_size(p) == 0
    with pytest.raises(fattn.FattnError) as e:
        fattn.flash_attn_ext(p, stream=0)
    assert e.value.code == -7


def test_rejects_missing_workspace():
    p = _params()
    with pytest.raises(fattn.FattnError) as e:
        fattn.flash_attn_ext(p, stream=0)
    assert e.value.code == -5


def test_rejects_misaligned_q():
    p = _params()
    p.q.data = (1 << 20) + 4
    assert fattn.lib().fattn_ext(C.byref(p), None) == -7


def test_rejects_null():
    p = _params()
    p.q.data = None
    assert fattn.lib().fattn_ext(C.byref(p), None) == -1
    assert fattn.lib().fattn_quantize(fattn.TYPE_Q8_0, None, None, 32, 1, None) == -1
    assert fattn.lib().fattn_dequantize(fattn.TYPE_Q8_0, None, None, 32, 1, None) == -1


def test_row_workspace_size():
    assert fattn.lib().fattn_row_workspace_size(128, 4096, 32) > 0
    assert fattn.lib().fattn_row_workspace_size(96, 4096, 32) > 0   # head dims 80 / 96 (f16 rows)
    assert fattn.lib().fattn_row_workspace_size(72, 4096, 32) == 0


def test_cpy_rejects_bad_views():
    """fattn_cpy validates before launching anything (no GPU needed)."""
    f32 = fattn.View(16, fattn.TYPE_F32, (128, 8, 1, 1), (4, 512, 4096, 4096))
    q8 = fattn.View(16, fattn.TYPE_Q8_0, (128, 8, 1, 1), (34, 136, 1088, 1088))
    L = fattn.lib()

    def rc(s, d):
        a, b = s.c(), d.c()
        return L.fattn_cpy(C.byref(a), C.byref(b), None)

    assert rc(q8, q8) == -2                                                            # src must be f32
    assert rc(f32, fattn.View(16, fattn.TYPE_Q8_0, (96, 8, 1, 1), (34, 136, 1088, 1088))) == -1  # ne differ
    assert rc(fattn.View(16, 0, (100, 8, 1, 1), (4, 400, 3200, 3200)),
              fattn.View(16, fattn.TYPE_Q8_0, (100, 8, 1, 1), (34, 136, 1088, 1088))) == -1  # not whole blocks
    assert rc(f32, fattn.View(16, fattn.TYPE_Q8_0, (128, 8, 1, 1), (18, 136, 1088, 1088))) == -4  # wrong nb0
    assert rc(fattn.View(18, fattn.TYPE_F32, (128, 8, 1, 1), (4, 512, 4096, 4096)), q8) == -7      # misaligned


def test_positional_launch_rejects_mixed_types():
    """fattn_ext_f16_launch shares K's row strides with V (src/flash-llama.h:123-125),
    so a mixed K / V type pair cannot be described there: rejected before any launch."""
    D, H, N, ptr = 128, 8, 256, 1 << 20
    rc = fattn.lib().fattn_ext_f16_launch(
        ptr, ptr, ptr, None, ptr, 0.088, D, 1, H, 1, D, N, H, 1, 1, N * 2, D * 4 * H, D * 4, D * H * 4,
        136, 136 * N, 136 * N * H, D, H, 1, 1, fattn.TYPE_Q8_0, fattn.TYPE_F16, None, 0, None)
    assert rc == -1


def test_pf_stage_falls_back_past_32bit_f16_span():
    """A Q8_0 cache whose staged f16 rows would pass the 32-bit descriptor span
    (N x D x 2 > 4 GiB per kv head, here 2^24 keys at D = 128: 4 GiB of f16,
    2.1 GiB of Q8_0) keeps the in-kernel dequantisation instead of wrapping its
    offsets; a shorter cache is staged."""
    big = _params(NQ=4096, H=32, Hkv=32, N=1 << 24, mask=False)
    d = fattn.describe(big)
    assert "kv_stage_f16" not in d and "fattn_pf_kernel<q8_0" in d, d
    small = _params(NQ=4096, H=32, Hkv=32, N=1 << 20, mask=False)
    assert fattn.describe(small).startswith("pf_prepass[kv_stage_f16<q8_0>"), fattn.describe(small)
