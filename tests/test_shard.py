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

from fattn.shard import gather_heads, shard_heads  # noqa: E402
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


def _slice_problem(prob, sh):
    """The rank's sub-problem: q-heads [h0,h1) and kv-heads [kv0,kv1), head layout."""
    from tests.problems import Problem
    rb = prob.k_nb[1]
    kb = prob.k_bytes.reshape(prob.Skv, prob.Hkv, prob.N, rb)[:, sh.kv0:sh.kv1]
    vb = prob.v_bytes.reshape(prob.Skv, prob.Hkv, prob.N, rb)[:, sh.kv0:sh.kv1]
    nkv = sh.n_kv
    nb = (prob.k_nb[0], rb, rb * prob.N, rb * prob.N * nkv)
    return Problem(prob.D, prob.NQ, sh.n_heads, nkv, prob.N, prob.S, prob.Skv, prob.kv_type, "head", prob.scale,
                   np.ascontiguousarray(prob.q[:, :, sh.h0:sh.h1]), np.ascontiguousarray(kb).reshape(-1),
                   np.ascontiguousarray(vb).reshape(-1), nb, nb, prob.mask_bits)


def _worker(rank, world, port, kv_type, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        prob = make_problem(D=64, NQ=3, H=8, Hkv=4, N=96, kv_type=kv_type, S=2, layout="head", seed=11)
        sh = shard_heads(prob.H, prob.Hkv, world, rank)
        local = torch.from_numpy(_slice_problem(prob, sh).oracle(n_threads=2))
        full = gather_heads(local)
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
