"""The reference's own known answer through the GPU kernels.

src/misc/flash-attn.cu:202-295 holds the only expected attention outputs the
reference ships: d_head 3, seq_len 4, 2 heads, small-integer Q / K / V^T, scale
1/sqrt(3), 24 values printed to 4 dp (tests/golden/kat_misc_flash_attn.json;
test_oracle.py::test_kat_misc_flash_attn checks the CPU oracle against them).
Here the HIP path takes them directly:

* the integers are exact in f16, so K and V go in as f16 with no rounding;
* D is zero-padded from 3 to 64 (the kernels' smallest head dim): q.k and the
  first 3 output dims are unchanged, the padded output dims are exactly 0;
* fattn_row (flash_attn_row + fa_reduce, V transposed [Hkv][D][N]) needs N a
  multiple of 32 for transposed V, so N is padded from 4 to 32 with zero K/V
  rows that the mask sets to -inf: exp(-inf) = 0 adds nothing to m, l or O;
  each (head, query row) is one "query head" of a GQA call with r_kv_heads = 4;
* fattn_ext (flash_attn_ext_f16's ne/nb call, V not transposed) takes the
  4-position cache as is -- 4 query rows x 2 heads, no mask.

Bar: north_star's 1e-3 (the fixture's own print precision is 5e-5).
"""
import json
import os

import numpy as np
import pytest

import fattn
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DP = 64  # padded head dim


def _kat():
    with open(os.path.join(GOLD, "kat_misc_flash_attn.json")) as f:
        k = json.load(f)
    D, N, H = k["d_head"], k["seq_len"], k["num_heads"]
    Q = np.array(k["query"], np.float32).reshape(H, N, D)            # [head][query row][d]
    K = np.array(k["key"], np.float32).reshape(H, N, D)              # [head][position][d]
    V = np.array(k["value_transposed"], np.float32).reshape(H, D, N).transpose(0, 2, 1)  # [head][position][d]
    exp = np.array(k["expected"], np.float32).reshape(H, N, D)       # [head][query row][d]
    return D, N, H, Q, K, V, exp


def _pad_d(x):
    out = np.zeros(x.shape[:-1] + (DP,), np.float32)
    out[..., :x.shape[-1]] = x
    return out


def _t(a, dev):
    import torch
    return torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else np.ascontiguousarray(a)).to(dev)


def test_kat_integers_exact_in_f16():
    _, _, _, Q, K, V, _ = _kat()
    for x in (Q, K, V):
        assert np.array_equal(orc.f16_bits_to_f32(orc.f32_to_f16_bits(x)), x)


def test_kat_through_fattn_row(dev):
    """fattn_row: H = 2 heads x 4 query rows as 8 query heads over Hkv = 2 kv
    heads (r_kv_heads = 4: query head h reads kv head h / 4), V transposed."""
    import torch
    D, N, H, Q, K, V, exp = _kat()
    NP = 32
    kp = np.zeros((H, NP, DP), np.float32)
    kp[:, :N] = _pad_d(K)
    vt = np.zeros((H, DP, NP), np.float32)
    vt[:, :, :N] = _pad_d(V).transpose(0, 2, 1)
    mask = np.full(NP, -np.inf, np.float32)
    mask[:N] = 0.0
    q = _pad_d(Q).reshape(H * N, DP)  # query head h = head * 4 + row
    qkv = torch.full((H * N * DP,), float("nan"), dtype=torch.float32, device=dev)
    fattn.row(_t(q, dev), _t(orc.f32_to_f16_bits(kp), dev), _t(orc.f32_to_f16_bits(vt), dev),
              _t(orc.f32_to_f16_bits(mask), dev), qkv, DP, NP, H * N, 1.0 / np.sqrt(np.float32(D)), DP * NP, N)
    torch.cuda.synchronize()
    got = qkv.cpu().numpy().reshape(H, N, DP)
    assert np.all(got[..., D:] == 0.0)
    assert np.abs(got[..., :D] - exp).max() < 1e-3, got[..., :D]


@pytest.mark.parametrize("layout", ["head", "pos"])
def test_kat_through_fattn_ext(dev, layout):
    """fattn_ext on the fixture's own shape: Q f32 [1][4][2][64], K / V f16
    ggml rows over the 4 positions ([Hkv][N] or llama.cpp's [N][Hkv] row
    order), no mask; dst [1][4][2][64]."""
    import torch
    D, N, H, Q, K, V, exp = _kat()
    q = torch.from_numpy(np.ascontiguousarray(_pad_d(Q).transpose(1, 0, 2))[None]).to(dev)  # [1][n_q][H][D]
    kb = _pad_d(K) if layout == "head" else _pad_d(K).transpose(1, 0, 2)
    vb = _pad_d(V) if layout == "head" else _pad_d(V).transpose(1, 0, 2)
    kd = _t(orc.f32_to_f16_bits(np.ascontiguousarray(kb)).reshape(-1), dev)
    vd = _t(orc.f32_to_f16_bits(np.ascontiguousarray(vb)).reshape(-1), dev)
    kv = fattn.kv_view(kd, fattn.TYPE_F16, DP, N, H, layout=layout)
    vv = fattn.kv_view(vd, fattn.TYPE_F16, DP, N, H, layout=layout)
    dst = torch.full((1, N, H, DP), float("nan"), dtype=torch.float32, device=dev)
    fattn.Attention(fattn.q_view(q), kv, vv, None, dst, 1.0 / np.sqrt(np.float32(D)))()
    torch.cuda.synchronize()
    got = dst.cpu().numpy()[0].transpose(1, 0, 2)  # [head][query row][d]
    assert np.all(got[..., D:] == 0.0)
    assert np.abs(got[..., :D] - exp).max() < 1e-3, got[..., :D]
