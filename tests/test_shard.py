"""Multi-rank head sharding on CPU: world_size-2 gloo.

Each rank solves its kv-head group of a GQA problem with the CPU oracle (the
stand-in for its GPU), the outputs meet in ONE all_gather, and the gathered
tensor must equal the single-process oracle bit for bit (heads are
independent; nothing is reduced across ranks).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ggml-cuda-experiments_amd"), ROOT]

from fattn.shard import assemble_heads, gather_heads, head_views, shard_heads  # noqa: E402
from tests.problems import make_problem  # noqa: E402


def test_shard_heads_partition():
    for H, Hkv, W in [(32, 8, 8), (32, 32, 4), (32, 8, 2), (64, 16, 8), (8, 8, 1)]:
        shards = [shard_heads(H, Hkv, W, r) for r in range(W)]
        assert shards[0].kv0 == 0 and shards[-1].kv1 == Hkv
        assert shards[0].h0 == 0 and shards[-1].h1 == H
        for a, b in zip(shards, shards[1:]):
            assert a.kv1 == b.kv0 and a.h1 == b.h0
        for s in shards:
            # every q-head of a shard maps (GQA, flash-llama.h:128-140) into the shard's kv-heads
            r = H // Hkv
            assert all(s.kv0 <= h // r < s.kv1 for h in range(s.h0, s.h1))


@pytest.mark.parametrize("bad", [(32, 8, 3), (30, 8, 2), (32, 8, 16)])
def test_shard_heads_rejects(bad):
    H, Hkv, W = bad
    with pytest.raises(ValueError):
        shard_heads(H, Hkv, W, 0)


def _materialize(base: np.ndarray, view, row_bytes: int) -> np.ndarray:
    """Bytes of a (possibly narrowed) ggml view whose ptr is a byte offset into
    `base`: [ne3][ne2][ne1][row_bytes], made contiguous."""
    ne, nb = view.ne, view.nb
    arr = np.lib.stride_tricks.as_strided(base[view.ptr:], shape=(ne[3], ne[2], ne[1], row_bytes),
                                          strides=(nb[3], nb[2], nb[1], 1), writeable=False)
    return np.ascontiguousarray(arr)


def _slice_problem(prob, sh):
    """The rank's sub-problem through the product's own slicing code
    (fattn.shard.head_views, as bench.py's sharded mode uses it) applied to
    byte-offset views of the full problem."""
    from fattn import View
    from tests.problems import Problem
    qv = View(0, 0, prob.q_ne, prob.q_nb)
    kv = View(0, prob.kv_type, prob.kv_ne, prob.k_nb)
    vv = View(0, prob.kv_type, prob.kv_ne, prob.v_nb)
    qs, ks, vs = head_views(qv, kv, vv, sh)
    rb = prob.k_nb[1]
    qb = _materialize(np.ascontiguousarray(prob.q).view(np.uint8).reshape(-1), qs, prob.D * 4)
    q = qb.view(np.float32).reshape(prob.S, sh.n_heads, prob.NQ, prob.D).transpose(0, 2, 1, 3)
    kb = _materialize(prob.k_bytes, ks, rb)  # [Skv][n_kv][N][rb]
    vb = _materialize(prob.v_bytes, vs, rb)
    nkv = sh.n_kv
    nb = (prob.k_nb[0], rb, rb * prob.N, rb * prob.N * nkv)
    return Problem(prob.D, prob.NQ, sh.n_heads, nkv, prob.N, prob.S, prob.Skv, prob.kv_type, "head", prob.scale,
                   np.ascontiguousarray(q), kb.reshape(-1), vb.reshape(-1), nb, nb, prob.mask_bits)


def _worker(rank, world, port, kv_type, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        prob = make_problem(D=64, NQ=3, H=8, Hkv=4, N=96, kv_type=kv_type, S=2, layout="head", seed=11)
        sh = shard_heads(prob.H, prob.Hkv, world, rank)
        local = torch.from_numpy(_slice_problem(prob, sh).oracle(n_threads=2))
        full = gather_heads(local)
        # the preallocated form bench.py captures into a HIP graph: same bytes
        buf = torch.full((world,) + tuple(local.shape), float("nan"), dtype=local.dtype)
        out = torch.full(tuple(full.shape), float("nan"), dtype=local.dtype)
        assert gather_heads(local, buf=buf, out=out) is out
        assert torch.equal(out, full)
        if rank == 0:
            q.put(full.numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("kv_type", ["q8_0", "q4_0"])
def test_two_rank_gather_equals_single_process(kv_type):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kv_type, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=120)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    prob = make_problem(D=64, NQ=3, H=8, Hkv=4, N=96, kv_type=kv_type, S=2, layout="head", seed=11)
    ref = prob.oracle(n_threads=2)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


def test_assemble_heads_matches_layout():
    """assemble_heads puts rank w's heads at [w*Hl, (w+1)*Hl) of the ggml dst
    [S][n_q][H][D] (src/flash-llama.h:434), for numpy and torch, with and
    without a leading (rotation) axis."""
    W, S, NQ, Hl, D = 4, 2, 3, 2, 5
    full = np.arange(S * NQ * W * Hl * D, dtype=np.float32).reshape(S, NQ, W * Hl, D)
    parts = np.stack([full[:, :, w * Hl:(w + 1) * Hl] for w in range(W)])
    assert np.array_equal(assemble_heads(parts), full)
    assert np.array_equal(assemble_heads(torch.from_numpy(parts)).numpy(), full)
    lead = np.stack([parts, parts + 1], axis=1)  # [W][R][S][NQ][Hl][D]
    got = assemble_heads(lead)
    assert np.array_equal(got[0], full) and np.array_equal(got[1], full + 1)


def test_slice_problem_oracle_matches_full_heads():
    """Single process: every rank's slice (head_views) solved by the oracle
    equals the full problem's heads -- the same check the GPU slice test makes
    with the HIP kernel (tests/test_gpu_parity.py::test_config5_head_shard_slices)."""
    prob = make_problem(D=64, NQ=2, H=8, Hkv=2, N=64, kv_type="q8_0", S=1, layout="head", seed=5)
    ref = prob.oracle(n_threads=2)
    parts = []
    for r in range(2):
        sh = shard_heads(prob.H, prob.Hkv, 2, r)
        parts.append(_slice_problem(prob, sh).oracle(n_threads=2))
    assert np.array_equal(assemble_heads(np.stack(parts)), ref)


def _batch_worker(rank, world, port, q):
    """bench.py's weak-scaling (--multi batch) gather on the CPU: every rank
    solves its own sequence (seed 300 + rank) with the oracle and the outputs
    meet in bench._gather(.., "batch") -- ONE all_gather_into_tensor."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        prob = make_problem(D=64, NQ=1, H=4, N=128, kv_type="q8_0", seed=300 + rank)
        local = torch.from_numpy(prob.oracle(n_threads=2))[None]  # [R=1][S][NQ][H][D]
        full = bench._gather(local, "batch")
        if rank == 0:
            q.put(full.numpy())
    finally:
        dist.destroy_process_group()


def test_two_rank_batch_gather_stacks_sequences():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batch_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=120)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    assert got.shape[:2] == (world, 1)
    for w in range(world):
        ref = make_problem(D=64, NQ=1, H=4, N=128, kv_type="q8_0", seed=300 + w).oracle(n_threads=2)
        assert np.array_equal(got[w, 0], ref)
