"""Heads x batch sharding across the GPUs of one node.

Heads (and ggml ne03 sequences) are independent attention problems: softmax
is per (sequence, head, query row) and the split-KV merge stays on one GPU,
so the path partitions with no collective on the data path.  A rank owns a
contiguous range of kv-heads together with their r = H/Hkv query heads (the
GQA broadcast ik2 = iq2 / r of src/flash-llama.h:128-140 never crosses a
shard), runs the unchanged single-GPU kernel on its slice, and the per-rank
outputs are collected with ONE all_gather (RCCL over xGMI on the GPU box,
gloo in the CPU tests) followed by a local permute into the ggml dst layout
[S][n_q][H][D] (src/flash-llama.h:434).
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class HeadShard:
    rank: int
    world: int
    kv0: int   # first kv-head owned
    kv1: int   # one past the last kv-head owned
    h0: int    # first q-head owned (= kv0 * r)
    h1: int

    @property
    def n_kv(self) -> int:
        return self.kv1 - self.kv0

    @property
    def n_heads(self) -> int:
        return self.h1 - self.h0


def shard_heads(H: int, Hkv: int, world: int, rank: int) -> HeadShard:
    """Contiguous kv-head groups; every rank gets the same count (the gather
    needs equal slices), so world must divide Hkv."""
    if H % Hkv:
        raise ValueError(f"H={H} not a multiple of Hkv={Hkv}")
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of {world}")
    if Hkv % world:
        raise ValueError(f"Hkv={Hkv} kv-heads do not split evenly over {world} ranks")
    r = H // Hkv
    per = Hkv // world
    kv0 = rank * per
    return HeadShard(rank, world, kv0, kv0 + per, kv0 * r, (kv0 + per) * r)


def gather_heads(local, group=None):
    """local: this rank's output [S][n_q][H/world][D] (contiguous).  Returns the
    full [S][n_q][H][D] on every rank via one all_gather_into_tensor."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    S, NQ, Hl, D = local.shape
    buf = torch.empty((world * S, NQ, Hl, D), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(buf, local.contiguous(), group=group)
    # [world][S][NQ][Hl][D] -> [S][NQ][world*Hl][D]: rank w holds heads [w*Hl, (w+1)*Hl)
    return buf.view(world, S, NQ, Hl, D).permute(1, 2, 0, 3, 4).reshape(S, NQ, world * Hl, D)
