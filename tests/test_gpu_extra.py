"""GPU parity, round 2: the reference's own fixtures and call sites through the
HIP path, the head-sharded multi-GPU slices on one GPU, one workspace shared
by a prefill and a decode, fattn_row at the reference's default GQA shape,
and the split kernel at 4, 8 and 16 waves per workgroup on the BASELINE configs.

Bar as in test_gpu_parity.py: attention within 1e-3 normwise relative error
per output row against the oracle -- here mostly against outputs the
REFERENCE's src/utils.h produced (tests/golden/, oracle/gen_golden.py).
"""
import os
import zlib

import numpy as np
import pytest

import fattn
from fattn.shard import assemble_heads, head_views, shard_heads
from gpu_util import run_gpu, upload, views
from oracle import oracle as orc
from problems import attn_elem_err, attn_rel_err, make_problem

pytestmark = pytest.mark.gpu
RTOL = 1e-3
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _kernel_test_inputs(D, H, Hkv, N):
    """kernel_test.h:45-48: glibc rand() from seed 1, fill order Q, K, V, mask."""
    orc.srand(1)
    return orc.random(D * H), orc.random(D * N * Hkv), orc.random(D * N * Hkv), orc.random(N)


def _t(a, dev):
    import torch
    return torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else np.ascontiguousarray(a)).to(dev)


# ------------------------------------------------------------------ reference fixtures through the HIP path

def test_golden_kernel_test_default_row(dev):
    """tests/golden/kernel_test_default.npz (the reference's CPU output for
    kernel_test.h's defaults: 32 q / 8 kv heads, D=128, kv_size=512) against
    fattn_row -- the flash_attn_row + fa_reduce call of kernel_test.h:161-162
    (V transposed, -DFA_KV_BLOCK_256, kernel_test.h:96-105)."""
    import torch
    z = np.load(os.path.join(GOLDEN, "kernel_test_default.npz"))
    D, H, Hkv, N = (int(x) for x in z["meta"])
    q, k, v, m = _kernel_test_inputs(D, H, Hkv, N)
    assert np.array_equal(q[:16], z["q_head"]) and np.array_equal(m[:16], z["m_head"])
    vt = orc.f32_to_f16_bits(np.ascontiguousarray(v.reshape(Hkv, N, D).transpose(0, 2, 1)))
    qkv = torch.empty(H * D, dtype=torch.float32, device=dev)
    fattn.row(_t(q, dev), _t(orc.f32_to_f16_bits(k), dev), _t(vt, dev), _t(orc.f32_to_f16_bits(m), dev), qkv, D, N,
              H, 1.0 / np.sqrt(np.float32(D)), D * N, H // Hkv)
    torch.cuda.synchronize()
    assert attn_rel_err(qkv.cpu().numpy().reshape(H, D), z["out"].reshape(H, D)) <= RTOL


def _reference_ext_call(dev, q, k16, v16, m, D, H, Hkv, N, k_type=fattn.TYPE_F16):
    """kernel_test.h:191-198 byte for byte: the flash_attn_ext_f16 argument list
    with the 32-row padded mask (row 0 = the mask, rows 1..31 zeros,
    kernel_test.h:74-85), ne31 = 32, nb31 = kv_size*2, nb01 = nb02 =
    head_dim*4, V not transposed."""
    import torch
    padded = np.zeros((32, N), dtype=np.uint16)
    padded[0] = orc.f32_to_f16_bits(m)
    dq, dk, dv, dm = _t(q, dev), _t(k16, dev), _t(v16, dev), _t(padded, dev)
    dst = torch.full((H * D,), float("nan"), dtype=torch.float32, device=dev)
    ws = torch.zeros(1 << 22, dtype=torch.uint8, device=dev)
    rb = fattn.row_size(k_type, D)
    rc = fattn.lib().fattn_ext_f16_launch(
        dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), dm.data_ptr(), dst.data_ptr(), 1.0 / np.sqrt(np.float32(D)),
        D, 1, H, 1,
        D, N, Hkv, 1,
        32, N * 2,
        D * 4, D * 4, D * H * 4,
        rb, rb * N, rb * N * Hkv,
        D, H, 1, 1,
        k_type, k_type, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0, fattn.strerror(rc)
    torch.cuda.synchronize()
    return dst.cpu().numpy().reshape(H, D)


def test_golden_kernel_test_default_ext_call(dev):
    """The same fixture through kernel_test.h's --no-kv-parallel branch, called
    exactly as kernel_test.h:191-198 calls flash_attn_ext_f16."""
    z = np.load(os.path.join(GOLDEN, "kernel_test_default.npz"))
    D, H, Hkv, N = (int(x) for x in z["meta"])
    q, k, v, m = _kernel_test_inputs(D, H, Hkv, N)
    got = _reference_ext_call(dev, q, orc.f32_to_f16_bits(k), orc.f32_to_f16_bits(v), m, D, H, Hkv, N)
    assert attn_rel_err(got, z["out"].reshape(H, D)) <= RTOL


def test_golden_kernel_test_q8_0_ext_call(dev):
    """tests/golden/kernel_test_q8_0.npz: the reference's attention arithmetic on
    Q8_0-rounded K/V (H=4, D=128, N=256), against the HIP kernel reading the
    Q8_0 blocks, through the kernel_test.h:191-198 argument list."""
    z = np.load(os.path.join(GOLDEN, "kernel_test_q8_0.npz"))
    D, H, Hkv, N = (int(x) for x in z["meta"])
    q, k, v, m = _kernel_test_inputs(D, H, Hkv, N)
    kq = orc.quantize(k.reshape(-1, D), orc.TYPE_Q8_0).reshape(-1)
    vq = orc.quantize(v.reshape(-1, D), orc.TYPE_Q8_0).reshape(-1)
    got = _reference_ext_call(dev, q, kq, vq, m, D, H, Hkv, N, fattn.TYPE_Q8_0)
    assert attn_rel_err(got, z["out"].reshape(H, D)) <= RTOL


def test_golden_cfg1_row(dev):
    """BASELINE config 1's fixture (H=1, D=64, N=128; full inputs and the
    reference's output) through fattn_row on the GPU."""
    import torch
    z = np.load(os.path.join(GOLDEN, "kernel_test_cfg1.npz"))
    D, H, Hkv, N = (int(x) for x in z["meta"])
    vt = orc.f32_to_f16_bits(np.ascontiguousarray(z["value"].reshape(Hkv, N, D).transpose(0, 2, 1)))
    qkv = torch.empty(H * D, dtype=torch.float32, device=dev)
    fattn.row(_t(z["query"], dev), _t(orc.f32_to_f16_bits(z["key"]), dev), _t(vt, dev),
              _t(orc.f32_to_f16_bits(z["mask"]), dev), qkv, D, N, H, 1.0 / np.sqrt(np.float32(D)), D * N, 1)
    torch.cuda.synchronize()
    assert attn_rel_err(qkv.cpu().numpy().reshape(H, D), z["out"].reshape(H, D)) <= RTOL


# ------------------------------------------------------------------ call-site details

def test_row_gqa_full_size(dev):
    """fattn_row at N=4096 with the reference's default GQA 32/8
    (r_kv_heads = 4): fattn_row_workspace_size must cover the r = 4 plan."""
    import torch
    D, H, Hkv, N = 128, 32, 8, 4096
    rng = np.random.default_rng(7)
    q = (1 - 2 * rng.random(H * D, dtype=np.float32))
    k = (1 - 2 * rng.random(Hkv * N * D, dtype=np.float32))
    v = (1 - 2 * rng.random(Hkv * N * D, dtype=np.float32))
    m = (1 - 2 * rng.random(N, dtype=np.float32))
    ref = orc.kernel_test_cpu(q, k, v, m, N, D, H, Hkv, n_threads=8)
    vt = orc.f32_to_f16_bits(np.ascontiguousarray(v.reshape(Hkv, N, D).transpose(0, 2, 1)))
    qkv = torch.empty(H * D, dtype=torch.float32, device=dev)
    fattn.row(_t(q, dev), _t(orc.f32_to_f16_bits(k), dev), _t(vt, dev), _t(orc.f32_to_f16_bits(m), dev), qkv, D, N,
              H, 1.0 / np.sqrt(np.float32(D)), D * N, H // Hkv)
    torch.cuda.synchronize()
    assert attn_rel_err(qkv.cpu().numpy().reshape(H, D), ref.reshape(H, D)) <= RTOL


def test_positional_launch_odd_kv(dev):
    """flash-llama.h:7-32 argument list with an odd ne11: the mask row length
    comes from nb31 (ggml pads mask rows, GGML_KQ_MASK_PAD), not from ne11."""
    import torch
    D, H, Hkv, N = 128, 8, 8, 333
    p = make_problem(D=D, NQ=1, H=H, Hkv=Hkv, N=N, kv_type="f16", mask="random", seed=17, mask_pad=64)
    t = upload(p, dev)
    npad = p.mask_bits.shape[1]
    ws = torch.zeros(1 << 22, dtype=torch.uint8, device=dev)
    rc = fattn.lib().fattn_ext_f16_launch(
        t["q"].data_ptr(), t["k"].data_ptr(), t["v"].data_ptr(), t["mask"].data_ptr(), t["dst"].data_ptr(),
        p.scale, D, 1, H, 1, D, N, Hkv, 1, p.mask_bits.shape[0], npad * 2, D * 4 * H, D * 4, D * H * 4,
        D * 2, D * N * 2, D * N * Hkv * 2, D, H, 1, 1, fattn.TYPE_F16, fattn.TYPE_F16, ws.data_ptr(), ws.numel(),
        torch.cuda.current_stream().cuda_stream)
    assert rc == 0, fattn.strerror(rc)
    torch.cuda.synchronize()
    assert attn_rel_err(t["dst"].cpu().numpy(), p.oracle()) <= RTOL


def test_workspace_prefill_then_decode(dev):
    """One workspace for a masked (causal) prefill and then a multi-chunk
    decode, as llama.cpp reuses it: the prefill's live-block flags share the
    front of the workspace with the decode's arrival words, which the decode
    supersedes by its epoch stamp (nothing re-zeroes the flags)."""
    import torch
    pre = make_problem(D=128, NQ=512, H=8, Hkv=2, N=512, kv_type="q8_0", mask="causal", seed=61)
    dec = make_problem(D=128, NQ=1, H=32, Hkv=8, N=4096, kv_type="q8_0", mask="random", seed=62)
    tp, td = upload(pre, dev), upload(dec, dev)
    fattn.set_option(fattn.OPT_PF, 2)  # the prefill kernel on this small prefill too
    try:
        ap = fattn.Attention(*views(pre, tp), tp["dst"], pre.scale)
        ad = fattn.Attention(*views(dec, td), td["dst"], dec.scale)
        assert "pf_mask_flags" in ap.describe(), ap.describe()
        assert int(ad.describe().split("grid(")[1].split(",")[0]) > 1, ad.describe()  # several chunks
        need = max(fattn.workspace_size(ap.p), fattn.workspace_size(ad.p))
        ws = torch.zeros(need, dtype=torch.uint8, device=dev)
        for a in (ap, ad):
            a.p.workspace, a.p.workspace_bytes = ws.data_ptr(), ws.numel()
        ref_dec = dec.oracle()
        for _ in range(3):
            ap()
            ad()
            torch.cuda.synchronize()
            assert attn_rel_err(td["dst"].cpu().numpy(), ref_dec) <= RTOL
        assert attn_rel_err(tp["dst"].cpu().numpy(), pre.oracle()) <= RTOL
    finally:
        fattn.set_option(fattn.OPT_PF, 0)


@pytest.mark.parametrize("fill", ["bytes5a", "stale_count"])
@pytest.mark.parametrize("case", [
    dict(D=128, NQ=1, H=32, N=4096, kv_type="q8_0"),                  # config 3: workgroup-level row merge
    dict(D=128, NQ=1, H=32, N=4096, kv_type="q8_0", waves=4),         # wave partials (wave_merge 1)
    dict(D=128, NQ=16, H=4, N=4096, kv_type="q8_0", merge=1),         # multi-row tiles, fused: combine_tile
    dict(D=128, NQ=16, H=4, N=4096, kv_type="q8_0"),                  # multi-row tiles, second-launch merge
    dict(D=128, NQ=64, H=32, Hkv=8, N=2048, kv_type="q8_0", mq=1, merge=1),  # multi-query kernel, fused
    dict(D=128, NQ=64, H=4, N=4096, kv_type="q8_0"),                  # batched-decode kernel (merge launch)
    dict(D=128, NQ=1, H=32, N=4096, kv_type="q8_0", xcd=1),          # config 3, plain workgroup order
    dict(D=64, NQ=1, H=32, N=8192, kv_type="q4_0"),                   # D = 64, XCD order (auto)
], ids=["row_merge", "wave_merge", "combine", "merge_launch", "mq", "bd", "row_merge_plain", "row_merge_d64"])
def test_workspace_not_zeroed(dev, case, fill):
    # (the multi-row case merges in a second launch and never reads the words;
    # it checks that the garbage does not leak into the partials either)
    """The arrival words need no zeroing: each launch stamps them with its own
    epoch before counting (fattn_split.h arrival_begin), so a workspace full of
    garbage, or left mid-count by an aborted launch, gives the right result on
    the first launch and leaves the words re-armed for the next."""
    import torch
    case = dict(case)
    waves = case.pop("waves", 0)
    merge = case.pop("merge", 0)
    mq = case.pop("mq", 0)
    xcd = case.pop("xcd", 0)
    p = make_problem(seed=71, **case)
    t = upload(p, dev)
    fattn.set_option(fattn.OPT_SPLIT_WAVES, waves)
    fattn.set_option(fattn.OPT_SPLIT_MERGE, merge)
    fattn.set_option(fattn.OPT_SPLIT_XCD, xcd)
    if mq:
        fattn.set_option(fattn.OPT_BD, 1)
        fattn.set_option(fattn.OPT_MQ_MIN_ROWS, 32)
    try:
        att = fattn.Attention(*views(p, t), t["dst"], p.scale)
        assert int(att.describe().split("grid(")[1].split(",")[0]) > 1, att.describe()  # several chunks
        if xcd == 1:
            assert "(xcd order)" not in att.describe(), att.describe()
        ws = att.workspace
        if fill == "bytes5a":
            ws.fill_(0x5A)
        else:  # every 256-B counter line: tag | epoch 1 | generation 0 | 5 arrivals already counted
            words = ws[: ws.numel() // 8 * 8].view(torch.int64)
            words[::32] = (0xFF << 56 | 1 << 24 | 5) - (1 << 64)
        ref = p.oracle()
        for _ in range(2):
            t["dst"].zero_()
            att()
            torch.cuda.synchronize()
            assert attn_rel_err(t["dst"].cpu().numpy(), ref) <= RTOL
    finally:
        fattn.set_option(fattn.OPT_SPLIT_WAVES, 0)
        fattn.set_option(fattn.OPT_SPLIT_MERGE, 0)
        fattn.set_option(fattn.OPT_BD, 0)
        fattn.set_option(fattn.OPT_MQ_MIN_ROWS, 0)


# ------------------------------------------------------------------ multi-GPU head shard, one GPU

@pytest.mark.parametrize("world", [2, 4, 8])
def test_config5_head_shard_slices(dev, world):
    """BASELINE config 5 (n_q = 64, 32 heads, N = 4096, Q8_0) cut into the
    per-rank slices bench.py --gpus N runs (fattn.shard.shard_heads +
    head_views: zero-copy q / k / v views, the GQA map kept inside a slice),
    each slice run through the HIP kernel on this GPU, the slices assembled
    into the ggml dst layout exactly as gather_heads does after the RCCL
    all_gather -- against the oracle of the whole problem.  (World 4: the
    multi-row split kernel's 8-wave plan.)"""
    import torch
    p = make_problem(D=128, NQ=64, H=32, N=4096, kv_type="q8_0", seed=55)
    t = upload(p, dev)
    qv, kv, vv, mv = views(p, t)
    parts = []
    for rank in range(world):
        sh = shard_heads(p.H, p.Hkv, world, rank)
        qs, ks, vs = head_views(qv, kv, vv, sh)
        dst = torch.full((1, p.NQ, sh.n_heads, p.D), float("nan"), dtype=torch.float32, device=dev)
        att = fattn.Attention(qs, ks, vs, mv, dst, p.scale)
        if world == 4:
            assert "8waves> + fattn_merge_kernel" in att.describe(), att.describe()
        att()
        parts.append(dst)
    torch.cuda.synchronize()
    full = assemble_heads(torch.stack(parts)).cpu().numpy()
    assert attn_rel_err(full, p.oracle()) <= RTOL


def test_config4_gqa_head_shard_slices(dev):
    """Config 4 (Q4_0, GQA 32/8) on 8 ranks: one kv head and its 4 q heads each."""
    import torch
    p = make_problem(D=128, NQ=1, H=32, Hkv=8, N=8192, kv_type="q4_0", seed=56)
    t = upload(p, dev)
    qv, kv, vv, mv = views(p, t)
    parts = []
    for rank in range(8):
        sh = shard_heads(p.H, p.Hkv, 8, rank)
        assert (sh.n_kv, sh.n_heads) == (1, 4)
        qs, ks, vs = head_views(qv, kv, vv, sh)
        dst = torch.empty((1, 1, sh.n_heads, p.D), dtype=torch.float32, device=dev)
        fattn.Attention(qs, ks, vs, mv, dst, p.scale)()
        parts.append(dst)
    torch.cuda.synchronize()
    assert attn_rel_err(assemble_heads(torch.stack(parts)).cpu().numpy(), p.oracle()) <= RTOL


# ------------------------------------------------------------------ split kernel, 4 / 8 / 16 waves per workgroup

@pytest.fixture(params=[(4, 0), (8, 0), (16, 0), (4, 1), (8, 1)], ids=["4waves", "8waves", "16waves", "4waves-noskip",
                                                                       "8waves-noskip"])
def split_waves(request):
    waves, no_skip = request.param
    fattn.set_option(fattn.OPT_SPLIT_WAVES, waves)
    fattn.set_option(fattn.OPT_SPLIT_SKIP, no_skip)
    fattn.set_option(fattn.OPT_MQ_DISABLE, 1)  # the config-5 shard case exercises the split kernel
    yield request.param
    fattn.set_option(fattn.OPT_SPLIT_WAVES, 0)
    fattn.set_option(fattn.OPT_SPLIT_SKIP, 0)
    fattn.set_option(fattn.OPT_MQ_DISABLE, 0)


DEC_CASES = [
    dict(D=128, NQ=1, H=32, N=4096, kv_type="q8_0"),                 # config 3
    dict(D=128, NQ=1, H=32, N=2048, kv_type="f16"),                  # config 2
    dict(D=128, NQ=1, H=32, Hkv=8, N=8192, kv_type="q4_0"),          # config 4
    dict(D=128, NQ=1, H=8, N=32768, kv_type="q8_0"),                 # long KV: several steps per wave
    dict(D=128, NQ=64, H=4, N=4096, kv_type="q8_0"),                 # config 5, one GPU's shard
    dict(D=64, NQ=3, H=8, Hkv=2, N=1024, kv_type="q4_0", mask="causal"),
    dict(D=64, NQ=1, H=16, N=2048, kv_type="q8_0"),
    dict(D=256, NQ=1, H=4, N=1024, kv_type="q8_0"),
    dict(D=256, NQ=1, H=16, N=2048, kv_type="f16"),
    dict(D=128, NQ=1, H=4, N=512, kv_type="f16", v_trans=True),
    dict(D=128, NQ=2, H=4, N=96, kv_type="q8_0", mask="neginf_blocks", S=2),
    dict(D=128, NQ=1, H=8, N=1000, kv_type="q8_0", layout="pos"),    # generic-stride path: always 4 waves
    # padded caches: whole steps, slices and chunks -inf (step skipping, empty partials)
    dict(D=128, NQ=1, H=32, N=4096, kv_type="q8_0", mask="tail"),
    dict(D=128, NQ=1, H=32, Hkv=8, N=8192, kv_type="q4_0", mask="tail"),
    dict(D=128, NQ=64, H=4, N=4096, kv_type="q8_0", mask="tail"),
    dict(D=128, NQ=1, H=8, N=32768, kv_type="q8_0", mask="tail"),            # >= 4 steps per wave: K/V of
    dict(D=128, NQ=3, H=8, Hkv=2, N=16384, kv_type="q4_0", mask="tail"),     # -inf steps not fetched
]


@pytest.mark.parametrize("case", DEC_CASES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_split_waves(dev, split_waves, case):
    p = make_problem(seed=zlib.crc32(str(sorted(case.items())).encode()) % 1000, **case)
    t = upload(p, dev)
    att = fattn.Attention(*views(p, t), t["dst"], p.scale)
    assert "fattn_split_kernel" in att.describe(), att.describe()
    assert attn_rel_err(run_gpu(p), p.oracle()) <= RTOL


@pytest.mark.parametrize("case", [
    dict(D=128, NQ=1, H=8, N=32768, kv_type="q8_0", mask="tail"),
    dict(D=128, NQ=3, H=8, Hkv=2, N=16384, kv_type="q4_0", mask="tail"),
    dict(D=64, NQ=1, H=16, N=16384, kv_type="f16", mask="neginf_blocks"),
], ids=["q8_0_tail", "q4_0_gqa_tail", "f16_blocks"])
def test_step_skip_bitexact(dev, case):
    """Steps that are -inf for the whole tile are not fetched (K/V through
    empty descriptors); their compute then adds exactly 0, so the output is
    bit-identical to the run that fetches every step (FATTN_OPT_SPLIT_SKIP)."""
    import torch
    p = make_problem(seed=83, **case)
    t = upload(p, dev)
    att = fattn.Attention(*views(p, t), t["dst"], p.scale)
    outs = []
    try:
        for no_skip in (0, 1):
            fattn.set_option(fattn.OPT_SPLIT_SKIP, no_skip)
            t["dst"].zero_()
            att()
            torch.cuda.synchronize()
            outs.append(t["dst"].cpu().clone())
    finally:
        fattn.set_option(fattn.OPT_SPLIT_SKIP, 0)
    assert torch.equal(outs[0], outs[1])
    assert attn_rel_err(outs[0].numpy(), p.oracle()) <= RTOL


@pytest.mark.parametrize("fused", [0, 1], ids=["merge_launch", "fused"])
@pytest.mark.parametrize("case", [
    dict(D=128, NQ=64, H=4, N=4096, kv_type="q8_0"),                  # config 5 shard: 16-row tiles, 16 chunks
    dict(D=128, NQ=1, H=32, Hkv=8, N=8192, kv_type="q4_0"),           # config 4: 4-row tiles, 32 chunks
    dict(D=96, NQ=4, H=16, Hkv=4, N=4096, kv_type="q8_0", mask="tail"),
    dict(D=80, NQ=3, H=8, Hkv=2, N=4096, kv_type="f16"),
    dict(D=256, NQ=2, H=8, Hkv=4, N=4096, kv_type="f16", S=2),
    dict(D=64, NQ=9, H=8, Hkv=2, N=4096, kv_type="q4_0", mask="causal"),
], ids=["config5_shard", "config4", "d96_tail", "d80", "d256_s2", "d64_causal"])
def test_multirow_merge_paths(dev, case, fused):
    """Multi-row split tiles: the second-launch merge (one wave per tile row,
    fattn_merge_kernel) and the last-arriving-workgroup merge (combine_tile)
    both match the oracle."""
    p = make_problem(seed=zlib.crc32(str(sorted(case.items())).encode()) % 1000, **case)
    t = upload(p, dev)
    fattn.set_option(fattn.OPT_SPLIT_MERGE, fused)
    fattn.set_option(fattn.OPT_MQ_DISABLE, 1)  # config 5's shard would take the batched-decode kernel
    try:
        att = fattn.Attention(*views(p, t), t["dst"], p.scale)
        d = att.describe()
        assert "fattn_split_kernel" in d and int(d.split("grid(")[1].split(",")[0]) >= 4, d
        assert ("fattn_merge_kernel" in d) == (not fused), d
        assert attn_rel_err(run_gpu(p), p.oracle()) <= RTOL
    finally:
        fattn.set_option(fattn.OPT_SPLIT_MERGE, 0)
        fattn.set_option(fattn.OPT_MQ_DISABLE, 0)


# ------------------------------------------------------------------ quantize-on-write (fattn_cpy)

@pytest.mark.parametrize("kt", ["q8_0", "q4_0", "f16"])
@pytest.mark.parametrize("layout", ["head", "pos"])
@pytest.mark.parametrize("ntok", [1, 5])
def test_cpy_into_kv_cache_view(dev, kt, layout, ntok):
    """GGML_OP_CPY f32 -> cache type into the cache view of `ntok` new tokens at
    position p: every written row bit-exact with the oracle's ggml
    quantisation (or f16 RNE), every other byte of the cache untouched."""
    import torch
    from problems import TYPES, encode_rows
    typ = TYPES[kt]
    D, Hkv, N, p0 = 128, 8, 64, 37
    rb = fattn.row_size(typ, D)
    eb = 2 if typ == fattn.TYPE_F16 else fattn.BLOCK_BYTES[typ]
    rng = np.random.default_rng(ntok * 10 + len(layout))
    cache0 = rng.integers(0, 256, size=Hkv * N * rb, dtype=np.uint8)
    cur = (1 - 2 * rng.random((ntok, Hkv, D), dtype=np.float32)) * 3  # K_cur [tok][Hkv][D]
    cur[0, 1, :32] = 0.0                                                # an all-zero block (d = 0)
    cache = torch.from_numpy(cache0.copy()).to(dev)
    src = torch.from_numpy(cur).to(dev)
    sv = fattn.View(src.data_ptr(), fattn.TYPE_F32, (D, Hkv, ntok, 1), (4, D * 4, Hkv * D * 4, ntok * Hkv * D * 4))
    if layout == "head":  # [Hkv][N][row]: a token's rows are N rows apart
        dv = fattn.View(cache.data_ptr() + p0 * rb, typ, (D, Hkv, ntok, 1), (eb, N * rb, rb, N * Hkv * rb))
    else:                 # [N][Hkv][row]: llama.cpp's cache, a token's rows contiguous
        dv = fattn.View(cache.data_ptr() + p0 * Hkv * rb, typ, (D, Hkv, ntok, 1), (eb, rb, Hkv * rb, N * Hkv * rb))
    fattn.cpy(sv, dv)
    torch.cuda.synchronize()
    got = cache.cpu().numpy()
    want = cache0.copy()
    rows = encode_rows(cur, typ)  # [tok][Hkv][rb]
    w = want.reshape(Hkv, N, rb) if layout == "head" else want.reshape(N, Hkv, rb)
    for t in range(ntok):
        for h in range(Hkv):
            if layout == "head":
                w[h, p0 + t] = rows[t, h]
            else:
                w[p0 + t, h] = rows[t, h]
    assert np.array_equal(got, want)


# ------------------------------------------------------------------ chunk merges: one-row tiles, batched decode in-kernel

@pytest.mark.parametrize("case", [
    dict(D=128, H=32, N=4096, kv_type="q8_0"),                 # config 3 (8 waves, 8 chunks)
    dict(D=128, H=8, N=8192, kv_type="q4_0", mask="tail"),      # whole chunks -inf
    dict(D=64, H=16, N=4096, kv_type="q8_0"),
    dict(D=80, H=16, N=2048, kv_type="f16"),
    dict(D=96, H=16, N=4096, kv_type="q8_0"),
    dict(D=256, H=16, N=2048, kv_type="f16"),
], ids=["cfg3", "q4_tail", "d64", "d80", "d96", "d256"])
def test_row_merge_head_dims(dev, case):
    """One-row tiles over several KV chunks (workgroup merge + last-arriver
    row merge) at every head dim, with forced chunk counts, against the oracle."""
    import torch
    p = make_problem(seed=5 + case["D"], **case)
    ref = p.oracle()
    t = upload(p, dev)
    for chunk in (0, 256, 512):
        att = fattn.Attention(*views(p, t), t["dst"], p.scale, kv_chunk=chunk)
        t["dst"].fill_(float("nan"))
        att()
        torch.cuda.synchronize()
        assert attn_rel_err(t["dst"].cpu().numpy(), ref) <= RTOL, att.describe()


def _replay_new_inputs(dev, shape, n_iter=12):
    """Capture one launch, then replay it (same epoch every replay) over K/V/Q/
    mask rewritten in place between replays, under uneven load from a copy
    stream; every replay against the oracle of its own inputs."""
    import torch
    probs = [make_problem(seed=400 + i, **shape) for i in range(3)]
    refs = [p.oracle() for p in probs]
    t = upload(probs[0], dev)
    att = fattn.Attention(*views(probs[0], t), t["dst"], probs[0].scale)
    assert int(att.describe().split("grid(")[1].split(",")[0]) > 1, att.describe()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        att(s.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        att(s.cuda_stream)
    noise_src = torch.randn(1 << 25, device=dev)
    noise_dst = torch.empty_like(noise_src)
    side = torch.cuda.Stream()
    for it in range(n_iter):
        p = probs[it % 3]
        t["q"].copy_(torch.from_numpy(np.ascontiguousarray(p.q)))
        t["k"].copy_(torch.from_numpy(p.k_bytes))
        t["v"].copy_(torch.from_numpy(p.v_bytes))
        t["mask"].copy_(torch.from_numpy(np.ascontiguousarray(p.mask_bits).view(np.int16)))
        t["dst"].fill_(float("nan"))
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            for _ in range(it % 3):
                noise_dst.copy_(noise_src)
        g.replay()
        torch.cuda.synchronize()
        assert attn_rel_err(t["dst"].cpu().numpy(), refs[it % 3]) <= RTOL, f"replay {it}: {att.describe()}"
    return att.describe()


@pytest.mark.parametrize("xcd", [1, 0], ids=["plain", "xcd_auto"])
def test_row_merge_graph_replays_new_inputs(dev, xcd):
    """Config 3 (one-row tiles, last-arriver merge): a captured launch replays
    with one epoch; the arrival words re-arm (count 0, generation + 1) so every
    replay merges its own partials -- in the plain and the XCD-grouped
    workgroup order (the default for these tiles)."""
    with fattn.options({fattn.OPT_SPLIT_XCD: xcd}):
        desc = _replay_new_inputs(dev, dict(D=128, NQ=1, H=32, N=4096, kv_type="q8_0"))
    assert ("(xcd order)" in desc) == (xcd == 0), desc


@pytest.mark.parametrize("in_kernel", [1, 0, 2, 3], ids=["in_kernel", "second_launch", "second_launch_plain",
                                                       "second_launch_f32"])
@pytest.mark.parametrize("case", [
    dict(D=128, NQ=64, H=32, N=4096, kv_type="q8_0"),                 # config 5 (8 chunks per kv head)
    dict(D=128, NQ=64, H=16, N=4096, kv_type="q8_0"),                 # its 2-rank shard
    dict(D=128, NQ=40, H=32, Hkv=8, N=4096, kv_type="q4_0", mask="causal"),  # GQA, partial row tile, causal
    dict(D=128, NQ=64, H=8, N=8192, kv_type="q8_0", mask="tail"),     # whole chunks -inf
    dict(D=96, NQ=64, H=32, N=4096, kv_type="q8_0"),                  # role form at D = 96: 12 dims a thread (8-B f16 stores)
    dict(D=64, NQ=64, H=32, N=4096, kv_type="q4_0"),                  # D = 64: f32 partials always
], ids=["cfg5", "cfg5_h16", "gqa_causal", "tail", "d96", "d64"])
def test_bd_chunk_merge_forms(dev, in_kernel, case):
    """The batched-decode kernel over several KV chunks: the partials merge in
    the second launch (default) or inside the launch (FATTN_OPT_MERGE_IN_KERNEL:
    every workgroup co-resident, each waits for the tile's count, then merges
    its share of the rows); both against the oracle, forced chunk counts
    included.  The second launch with f16 partials (0, FATTN_OPT_PART_F16 =
    2; the default here), f32 partials with plain loads (2,
    FATTN_OPT_MERGE_PLAIN) or with sc1 loads (3)."""
    import torch
    p = make_problem(seed=90 + case["H"], **case)
    ref = p.oracle()
    t = upload(p, dev)
    fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 1 if in_kernel == 1 else 0)
    fattn.set_option(fattn.OPT_MERGE_PLAIN, 2 if in_kernel == 2 else 0)
    fattn.set_option(fattn.OPT_PART_F16, 1 if in_kernel >= 2 else 2 if in_kernel == 0 else 0)
    try:
        for chunk in (0, 1024):
            att = fattn.Attention(*views(p, t), t["dst"], p.scale, kv_chunk=chunk)
            desc = att.describe()
            assert desc.startswith(("fattn_bd_kernel", "fattn_bdp_kernel")), desc
            g = [int(x) for x in desc.split("grid(")[1].split(")")[0].split(",")]
            cus = torch.cuda.get_device_properties(dev).multi_processor_count
            lds = int(desc.split(" lds ")[1].split()[0])
            resident = g[0] * g[1] * g[2] <= cus * max(1, 163840 // lds)  # (the planner's rule: workgroups a CU's LDS holds)
            assert ("in-kernel" in desc) == (in_kernel == 1 and resident), desc
            assert ("merge_kernel(plain)" in desc) == (in_kernel == 2 and "merge_kernel" in desc), desc
            # (in_kernel 1 on a grid that is not co-resident: the second launch, auto = f16)
            assert ("merge_kernel(f16 partials)" in desc) == (in_kernel in (0, 1) and "merge_kernel" in desc
                                                               and case["D"] != 64), desc
            t["dst"].fill_(float("nan"))
            att()
            torch.cuda.synchronize()
            assert attn_rel_err(t["dst"].cpu().numpy(), ref) <= RTOL, desc
    finally:
        fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 0)
        fattn.set_option(fattn.OPT_MERGE_PLAIN, 0)
        fattn.set_option(fattn.OPT_PART_F16, 0)


def test_bd_in_kernel_merge_graph_replays_new_inputs(dev):
    """Config 5 through the batched-decode kernel with the in-kernel merge: the
    waiting workgroups watch the arrival word for a complete count or the last
    arriver's re-arm (generation + 1), which must hold replay after replay of
    one captured launch (one epoch)."""
    fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 1)
    try:
        desc = _replay_new_inputs(dev, dict(D=128, NQ=64, H=32, N=4096, kv_type="q8_0"), n_iter=9)
    finally:
        fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 0)
    assert "in-kernel" in desc, desc


@pytest.mark.parametrize("in_kernel", [1, 0, 2, 3], ids=["in_kernel", "second_launch", "second_launch_plain",
                                                       "second_launch_f32"])
@pytest.mark.parametrize("case", [
    dict(D=128, NQ=1, H=32, Hkv=8, N=8192, kv_type="q4_0"),           # config 4
    dict(D=128, NQ=64, H=4, N=4096, kv_type="q8_0"),                  # config 5, 8-rank shard
    dict(D=128, NQ=16, H=4, N=4096, kv_type="q8_0", mask="tail"),     # whole chunks -inf
    dict(D=64, NQ=8, H=16, Hkv=4, N=4096, kv_type="q8_0"),
    dict(D=96, NQ=4, H=16, Hkv=4, N=4096, kv_type="q8_0"),
    dict(D=256, NQ=4, H=8, Hkv=2, N=2048, kv_type="f16"),
    dict(D=80, NQ=4, H=16, Hkv=4, N=2048, kv_type="f16"),             # D = 80: 10 lanes a part (f16 merge)
], ids=["cfg4", "cfg5_shard", "tail", "d64", "d96", "d256", "d80"])
def test_split_multirow_merge_forms(dev, in_kernel, case):
    """Multi-row split tiles over 4+ KV chunks: the partials merge one wave per
    (tile, row), inside the launch (the tile's workgroups wait for each other)
    or in the second launch (0: f16 partials forced, FATTN_OPT_PART_F16 = 2,
    except at D = 64; 2: f32 partials with plain loads, FATTN_OPT_MERGE_PLAIN;
    3: f32 partials); all against the oracle at several head dims."""
    import torch
    p = make_problem(seed=70 + case["D"], **case)
    ref = p.oracle()
    t = upload(p, dev)
    fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 1 if in_kernel == 1 else 0)
    fattn.set_option(fattn.OPT_MERGE_PLAIN, 2 if in_kernel == 2 else 0)
    fattn.set_option(fattn.OPT_PART_F16, 1 if in_kernel >= 2 else 2 if in_kernel == 0 else 0)
    fattn.set_option(fattn.OPT_MQ_DISABLE, 1)
    try:
        for chunk in (0, 256):
            att = fattn.Attention(*views(p, t), t["dst"], p.scale, kv_chunk=chunk)
            desc = att.describe()
            assert ("merge_kernel(plain)" in desc) == (in_kernel == 2 and "merge_kernel" in desc), desc
            if in_kernel != 1:
                assert ("f16 partials" in desc) == (in_kernel == 0 and "merge_kernel" in desc and case["D"] != 64), desc
            t["dst"].fill_(float("nan"))
            att()
            torch.cuda.synchronize()
            assert attn_rel_err(t["dst"].cpu().numpy(), ref) <= RTOL, desc
    finally:
        fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 0)
        fattn.set_option(fattn.OPT_MERGE_PLAIN, 0)
        fattn.set_option(fattn.OPT_PART_F16, 0)
        fattn.set_option(fattn.OPT_MQ_DISABLE, 0)


def test_split_in_kernel_merge_graph_replays_new_inputs(dev):
    """Config 4 (multi-row split tiles, in-kernel merge) replayed from one
    captured launch over changing inputs: the waiting workgroups see each
    replay's own count / generation."""
    fattn.set_option(fattn.OPT_MQ_DISABLE, 1)
    fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 1)
    try:
        desc = _replay_new_inputs(dev, dict(D=128, NQ=1, H=32, Hkv=8, N=8192, kv_type="q4_0"), n_iter=9)
    finally:
        fattn.set_option(fattn.OPT_MQ_DISABLE, 0)
        fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, 0)
    assert "in-kernel" in desc, desc


@pytest.mark.parametrize("case", [
    dict(D=128, NQ=1, H=32, Hkv=8, N=8192, kv_type="q4_0"),                # config 4
    dict(D=128, NQ=1, H=32, Hkv=8, N=4096, kv_type="q8_0", mask="tail"),   # whole chunks -inf
    dict(D=128, NQ=1, H=16, Hkv=2, N=2048, kv_type="f16"),                 # R = 8, f16
    dict(D=128, NQ=1, H=12, Hkv=2, N=4000, kv_type="q8_0"),                # R = 6, ragged
    dict(D=64, NQ=1, H=32, Hkv=8, N=4096, kv_type="q8_0", extreme=True),   # D = 64, rescales
], ids=["cfg4", "tail", "f16_r8", "r6_ragged", "d64_extreme"])
def test_gqa_unpacked_decode(dev, case):
    """FATTN_OPT_GQA_UNPACK = 2: a one-row GQA decode takes one q head per
    split tile (one-row tiles, the chunk rows merged inside the launch, each
    K/V byte read by the kv head's R tiles) -- against the oracle, over
    repeated launches on one workspace."""
    import torch
    p = make_problem(seed=77 + case["H"], **case)
    ref = p.oracle()
    t = upload(p, dev)
    with fattn.options({fattn.OPT_GQA_UNPACK: 2}):
        att = fattn.Attention(*views(p, t), t["dst"], p.scale)
        desc = att.describe()
        assert "merge_kernel" not in desc, desc
        for _ in range(3):
            t["dst"].fill_(float("nan"))
            att()
            torch.cuda.synchronize()
            got = t["dst"].cpu().numpy()
            assert attn_rel_err(got, ref) <= RTOL, desc


def test_seq64_decode(dev):
    """SURVEY 8(d)'s alternative reading of config 5 at a reduced cache: 64
    independent sequences (ne03 = 64), one query row each, each its own KV
    (4 heads x 1024 positions, Q8_0), the mask row broadcast -- the bench's
    config5_seq64 line runs the same plan family at 32 heads x 4096."""
    p = make_problem(D=128, NQ=1, H=4, Hkv=4, N=1024, kv_type="q8_0", S=64, seed=64)
    got, ref = run_gpu(p), p.oracle()
    assert attn_rel_err(got, ref) <= RTOL
    assert attn_elem_err(got, ref) <= 1.0
