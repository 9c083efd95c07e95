"""Run a tests/problems.Problem through the GPU path (fattn -> libfattn.so)."""
from __future__ import annotations

import numpy as np

import fattn
from problems import Problem


def upload(prob: Problem, dev="cuda"):
    import torch
    t = {
        "q": torch.from_numpy(np.ascontiguousarray(prob.q)).to(dev),
        "k": torch.from_numpy(prob.k_bytes).to(dev),
        "v": torch.from_numpy(prob.v_bytes).to(dev),
        "mask": (torch.from_numpy(np.ascontiguousarray(prob.mask_bits).view(np.int16)).to(dev)
                 if prob.mask_bits is not None else None),
        "dst": torch.full((prob.S, prob.NQ, prob.H, prob.D), float("nan"), dtype=torch.float32, device=dev),
    }
    return t


def views(prob: Problem, t):
    qv = fattn.View(t["q"].data_ptr(), fattn.TYPE_F32, prob.q_ne, prob.q_nb)
    kv = fattn.View(t["k"].data_ptr(), prob.kv_type, prob.kv_ne, prob.k_nb)
    vv = fattn.View(t["v"].data_ptr(), prob.v_type, prob.kv_ne, prob.v_nb)
    mv = fattn.View(t["mask"].data_ptr(), fattn.TYPE_F16, prob.mask_ne, prob.mask_nb) if t["mask"] is not None else None
    return qv, kv, vv, mv


def run_gpu(prob: Problem, kv_chunk: int = 0, dev="cuda") -> np.ndarray:
    import torch
    t = upload(prob, dev)
    att = fattn.Attention(*views(prob, t), t["dst"], prob.scale, kv_chunk=kv_chunk)
    att()
    torch.cuda.synchronize()
    return t["dst"].cpu().numpy()
