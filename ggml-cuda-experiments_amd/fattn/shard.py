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


def narrow(view, dim: int, start: int, count: int):
    """Zero-copy sub-view of a ggml view (fattn.View): elements [start, start+count)
    of ggml dimension `dim` -- the pointer moves by start * nb[dim], the
    strides stay.  `view.ptr` may be a device pointer or a byte offset."""
    from fattn import View
    if not 0 <= start <= start + count <= view.ne[dim]:
        raise ValueError(f"narrow dim {dim} [{start}, {start + count}) of {view.ne[dim]}")
    ne = list(view.ne)
    ne[dim] = count
    return View(view.ptr + start * view.nb[dim], view.type, tuple(ne), tuple(view.nb))


def head_views(q, k, v, sh: HeadShard):
    """The rank's FLASH_ATTN_EXT sub-problem, zero-copy: q heads [h0, h1) and
    kv heads [kv0, kv1) (ggml dim 2 of q / k / v).  The mask is shared by all
    heads (a row per query) and the rank's dst is its own contiguous
    [S][n_q][h1-h0][D]; the GQA map ik2 = iq2 / r (src/flash-llama.h:128-140)
    holds inside the slice because h0 = kv0 * r."""
    return narrow(q, 2, sh.h0, sh.n_heads), narrow(k, 2, sh.kv0, sh.n_kv), narrow(v, 2, sh.kv0, sh.n_kv)


def assemble_heads(parts):
    """[world] x [..., S, n_q, H/world, D] per-rank outputs stacked on a leading
    axis -> [..., S, n_q, H, D] in the ggml dst layout (src/flash-llama.h:434):
    rank w holds heads [w*Hl, (w+1)*Hl).  Works on torch tensors and numpy."""
    world = parts.shape[0]
    *lead, S, NQ, Hl, D = parts.shape[1:]
    nl = len(lead)
    perm = tuple(range(1, 1 + nl)) + (1 + nl, 2 + nl, 0, 3 + nl, 4 + nl)
    x = parts.permute(*perm) if hasattr(parts, "permute") else parts.transpose(perm)
    return x.reshape(*lead, S, NQ, world * Hl, D)


def gather_heads(local, group=None, buf=None, out=None):
    """local: this rank's output [..., S, n_q, H/world, D] (contiguous).  Returns
    the full [..., S, n_q, H, D] on every rank via ONE all_gather_into_tensor
    (RCCL over xGMI on the GPU box, gloo on the CPU) and assemble_heads.
    `buf` ([world, *local.shape]) and `out` (the full shape), when given, are
    used instead of fresh allocations -- the form a captured HIP graph replays
    (the gather lands in `buf`, the permute writes `out`)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if buf is None:
        buf = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(buf.view(world * local.shape[0], *local.shape[1:]), local.contiguous(), group=group)
    if out is None:
        return assemble_heads(buf)
    # one strided copy: out seen as [..., S, n_q, world, H/world, D]
    *lead, S, NQ, Hl, D = buf.shape[1:]
    nl = len(lead)
    perm = tuple(range(1, 1 + nl)) + (1 + nl, 2 + nl, 0, 3 + nl, 4 + nl)
    out.view(*lead, S, NQ, world, Hl, D).copy_(buf.permute(*perm))
    return out
