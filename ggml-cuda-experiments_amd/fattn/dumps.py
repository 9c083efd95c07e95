"""Attention over `.tensor` dumps: the reference's test_llama flow
(src/flash-matrix.cu:67-339) on this library.

Layouts follow the reference's own CPU check of those dumps
(src/flash-matrix.cu:86-110), read from each file's ggml `ne`:
    q     f32 ne = [D, n_q, H]         memory [H][n_q][D]
    k     f16 / Q8_0 / Q4_0 ne = [D, N, Hkv]     memory [Hkv][N][row]
    v     same as k, or f16 transposed ne = [N, D, Hkv]  memory [Hkv][D][N]
    mask  f16 ne = [N', rows >= n_q]   (optional; N' >= N)
    out   f32 [n_q][H][D]  (the permuted FLASH_ATTN_EXT dst, = the qkv dump's layout)
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from . import TYPE_F16, TYPE_F32, Attention, View, row_size
from .tensor_io import Tensor


def _dev_bytes(t: Tensor, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(t.data).view(np.uint8).reshape(-1).copy()).to(dev)


def attention_from_dumps(q: Tensor, k: Tensor, v: Tensor, mask: Optional[Tensor] = None,
                         scale: Optional[float] = None, dev="cuda") -> np.ndarray:
    import torch
    if q.type != TYPE_F32:
        raise ValueError("q dump must be f32")
    D, NQ, H = (tuple(q.ne) + (1, 1))[:3]
    Dk, N, Hkv = (tuple(k.ne) + (1, 1))[:3]
    if Dk != D or H % Hkv:
        raise ValueError(f"q ne={q.ne} and k ne={k.ne} do not match")
    rk = row_size(k.type, D)
    tq, tk, tv = _dev_bytes(q, dev), _dev_bytes(k, dev), _dev_bytes(v, dev)
    qv = View(tq.data_ptr(), TYPE_F32, (D, NQ, H, 1), (4, D * 4, NQ * D * 4, H * NQ * D * 4))
    kb0 = 2 if k.type == TYPE_F16 else rk // (D // 32)
    kv = View(tk.data_ptr(), k.type, (D, N, Hkv, 1), (kb0, rk, N * rk, Hkv * N * rk))
    if v.type == TYPE_F16 and tuple(v.ne[:2]) == (N, D) and N != D:
        # transposed V: element (d, n) at d * N + n
        vv = View(tv.data_ptr(), TYPE_F16, (D, N, Hkv, 1), (N * 2, 2, D * N * 2, Hkv * D * N * 2))
    else:
        if tuple(v.ne[:3]) != (D, N, Hkv) or v.type != k.type:
            raise ValueError(f"v ne={v.ne} type {v.type} does not match k")
        vv = View(tv.data_ptr(), v.type, (D, N, Hkv, 1), (kb0, rk, N * rk, Hkv * N * rk))
    mv = None
    tm = None
    if mask is not None:
        if mask.type != TYPE_F16:
            raise ValueError("mask dump must be f16")
        Np, rows = (tuple(mask.ne) + (1,))[:2]
        if Np < N or rows < NQ:
            raise ValueError(f"mask ne={mask.ne} too small for N={N}, n_q={NQ}")
        if Np % 2 or Np % 8:  # the library wants even-padded, 16-B aligned rows: repack
            Npad = (Np + 7) // 8 * 8
            m = np.full((rows, Npad), -np.inf, dtype=np.float16)
            m[:, :Np] = np.asarray(mask.data).reshape(rows, Np)
            Np, mdata = Npad, m
        else:
            mdata = np.asarray(mask.data).reshape(rows, Np)
        tm = torch.from_numpy(np.ascontiguousarray(mdata)).to(dev)
        mv = View(tm.data_ptr(), TYPE_F16, (Np, rows, 1, 1), (2, Np * 2, Np * rows * 2, Np * rows * 2))
    out = torch.empty((1, NQ, H, D), dtype=torch.float32, device=dev)
    att = Attention(qv, kv, vv, mv, out, float(scale if scale is not None else 1.0 / np.sqrt(D)))
    att()
    torch.cuda.synchronize()
    return out[0].cpu().numpy()
