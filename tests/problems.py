"""Test-problem builder shared by the parity tests, smoke() and bench.py.

Builds a FLASH_ATTN_EXT problem as raw ggml byte buffers (numpy) with ne/nb
views, so that the CPU oracle (oracle/oracle.py) and the GPU path
(fattn, via the C ABI) consume byte-identical inputs.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from oracle import oracle as orc

TYPES = {"f16": orc.TYPE_F16, "q8_0": orc.TYPE_Q8_0, "q4_0": orc.TYPE_Q4_0}


def row_bytes(typ: int, D: int) -> int:
    return D * 2 if typ == orc.TYPE_F16 else D // 32 * orc.BLOCK_BYTES[typ]


def encode_rows(x: np.ndarray, typ: int) -> np.ndarray:
    """f32 [..., D] -> ggml row bytes [..., row_bytes] (f16 RNE or ggml quantisation)."""
    if typ == orc.TYPE_F16:
        return orc.f32_to_f16_bits(x).view(np.uint8).reshape(x.shape[:-1] + (x.shape[-1] * 2,))
    return orc.quantize(x, typ)


@dataclass
class Problem:
    D: int
    NQ: int
    H: int
    Hkv: int
    N: int
    S: int
    Skv: int
    kv_type: int
    layout: str
    scale: float
    q: np.ndarray                      # f32 [S][NQ][H][D]
    k_bytes: np.ndarray                # flat uint8
    v_bytes: np.ndarray
    k_nb: tuple
    v_nb: tuple
    mask_bits: Optional[np.ndarray]    # uint16 [rows][Npad] or None
    v_trans: bool = False
    k_f32: np.ndarray = field(default=None, repr=False)   # logical [Skv][Hkv][N][D] before encoding
    v_f32: np.ndarray = field(default=None, repr=False)
    v_type: Optional[int] = None                           # V cache type (None: kv_type)

    def __post_init__(self):
        if self.v_type is None:
            self.v_type = self.kv_type

    # ggml views -------------------------------------------------------
    @property
    def q_ne(self):
        return (self.D, self.NQ, self.H, self.S)

    @property
    def q_nb(self):
        return (4, self.H * self.D * 4, self.D * 4, self.NQ * self.H * self.D * 4)

    @property
    def kv_ne(self):
        return (self.D, self.N, self.Hkv, self.Skv)

    @property
    def mask_ne(self):
        r, n = self.mask_bits.shape
        return (n, r, 1, 1)

    @property
    def mask_nb(self):
        r, n = self.mask_bits.shape
        return (2, n * 2, n * r * 2, n * r * 2)

    @property
    def elem_bytes_k(self):
        return 2 if self.kv_type == orc.TYPE_F16 else orc.BLOCK_BYTES[self.kv_type]

    def oracle(self, n_threads=8) -> np.ndarray:
        q = (np.ascontiguousarray(self.q), orc.TYPE_F32, self.q_ne, self.q_nb)
        k = (self.k_bytes, self.kv_type, self.kv_ne, self.k_nb)
        v = (self.v_bytes, self.v_type, self.kv_ne, self.v_nb)
        m = None
        if self.mask_bits is not None:
            m = (np.ascontiguousarray(self.mask_bits), orc.TYPE_F16, self.mask_ne, self.mask_nb)
        return orc.flash_attn_ext(q, k, v, m, self.scale, n_threads=n_threads)

    def algorithmic_bytes(self) -> int:
        """Q (f32) + K + V (stored) + mask (f16, n_q rows) + O (f32), each once."""
        rb = row_bytes(self.kv_type, self.D) + row_bytes(self.v_type, self.D)
        qo = self.S * self.NQ * self.H * self.D * 4
        kv = self.Skv * self.Hkv * self.N * rb
        mk = self.NQ * self.N * 2 if self.mask_bits is not None else 0
        return qo * 2 + kv + mk

    def flops(self) -> int:
        return 4 * self.S * self.NQ * self.H * self.N * self.D


def make_problem(D=128, NQ=1, H=32, Hkv=None, N=4096, kv_type="q8_0", S=1, Skv=None, layout="head",
                 mask="random", seed=0, scale=None, v_trans=False, mask_pad=64, extreme=False,
                 ramp=0.0, v_type=None) -> Problem:
    """Random problem.  mask: "none" | "random" (U[-1,1], like kernel_test.h:48) |
    "zero" | "causal" (query i sees positions <= N - NQ + i) | "neginf_blocks"
    (some 32-position blocks fully -inf for every row) | "tail" (a padded cache:
    -inf from ~3N/8 on, so whole chunks of the split are masked).  v_type: a V
    cache type other than kv_type (llama.cpp's separate K / V cache types)."""
    typ = TYPES[kv_type] if isinstance(kv_type, str) else kv_type
    vtyp = typ if v_type is None else (TYPES[v_type] if isinstance(v_type, str) else v_type)
    Hkv = H if Hkv is None else Hkv
    Skv = S if Skv is None else Skv
    rng = np.random.default_rng(seed)
    u = lambda *shape: (1.0 - 2.0 * rng.random(shape, dtype=np.float32)).astype(np.float32)
    q = u(S, NQ, H, D)
    k = u(Skv, Hkv, N, D)
    v = u(Skv, Hkv, N, D)
    if extreme:
        # large-magnitude scores force many online-softmax rescales
        q *= 8.0
        k[..., ::7, :] *= 4.0
    if ramp:
        # key magnitude growing along the sequence: the running max keeps
        # rising in small steps (the deferred-rescale path) with jumps between
        q *= 4.0
        k *= (1.0 + ramp * np.arange(N, dtype=np.float32) / max(N, 1))[:, None]
    scale = 1.0 / np.sqrt(np.float32(D)) if scale is None else scale
    k_rows = encode_rows(k, typ)   # [Skv][Hkv][N][row bytes]
    v_rows = encode_rows(v, vtyp)

    def place(rows, t):
        rb = row_bytes(t, D)
        eb = 2 if t == orc.TYPE_F16 else orc.BLOCK_BYTES[t]
        if layout == "head":
            return np.ascontiguousarray(rows), (eb, rb, rb * N, rb * N * Hkv)
        if layout == "pos":
            return np.ascontiguousarray(rows.transpose(0, 2, 1, 3)), (eb, rb * Hkv, rb, rb * N * Hkv)  # [Skv][N][Hkv][rb]
        if layout == "padded":
            # rows with a stride larger than the row (forces the dword-granular path)
            pad = rb + 8
            buf = np.zeros((Skv, Hkv, N, pad), dtype=np.uint8)
            buf[..., :rb] = rows
            return buf, (eb, pad, pad * N, pad * N * Hkv)
        raise ValueError(layout)

    k_buf, k_nb = place(k_rows, typ)
    v_buf, v_nb = place(v_rows, vtyp)
    if v_trans:
        assert typ == orc.TYPE_F16 and vtyp == orc.TYPE_F16
        vt = orc.f32_to_f16_bits(np.ascontiguousarray(v.transpose(0, 1, 3, 2)))  # [Skv][Hkv][D][N]
        v_buf = vt.view(np.uint8)
        v_nb = (N * 2, 2, D * N * 2, D * N * 2 * Hkv)

    mask_bits = None
    if mask != "none":
        rows = max(NQ, 1)
        npad = (N + mask_pad - 1) // mask_pad * mask_pad
        if mask == "random":
            m = u(rows, npad)
        elif mask == "zero":
            m = np.zeros((rows, npad), dtype=np.float32)
        elif mask == "causal":
            m = np.zeros((rows, npad), dtype=np.float32)
            for i in range(rows):
                m[i, N - NQ + i + 1:] = -np.inf
        elif mask == "tail":
            # a padded KV cache: positions from ~3/8 of N on are unused (-inf)
            m = u(rows, npad)
            m[:, max(1, 3 * N // 8 + 5):] = -np.inf
        elif mask == "neginf_blocks":
            m = u(rows, npad)
            for b in range(1, N // 32, 3):
                m[:, b * 32:(b + 1) * 32] = -np.inf
        else:
            raise ValueError(mask)
        mask_bits = orc.f32_to_f16_bits(m)
    return Problem(D, NQ, H, Hkv, N, S, Skv, typ, layout, float(np.float32(scale)), q, k_buf.reshape(-1).view(np.uint8),
                   v_buf.reshape(-1).view(np.uint8), k_nb, v_nb, mask_bits, v_trans, k, v, vtyp)


def attn_rel_err(got: np.ndarray, ref: np.ndarray) -> float:
    """Normwise relative error per output row (max over rows of
    max|got-ref| / max|ref|), the "1e-3 rel" of BASELINE.json's north_star.
    NaN positions must coincide (fully masked rows are NaN in the reference,
    src/utils.h:30-49)."""
    got = got.reshape(-1, got.shape[-1]).astype(np.float64)
    ref = ref.reshape(-1, ref.shape[-1]).astype(np.float64)
    gn, rn = np.isnan(got), np.isnan(ref)
    if not np.array_equal(gn, rn):
        return float("inf")
    ok = ~rn.any(axis=1)
    if not ok.any():
        return 0.0
    g, r = got[ok], ref[ok]
    den = np.maximum(np.abs(r).max(axis=1), 1e-30)
    return float((np.abs(g - r).max(axis=1) / den).max())


def attn_elem_err(got: np.ndarray, ref: np.ndarray, rtol: float = 2e-3, atol_row: float = 8e-4) -> float:
    """Elementwise check beside the normwise one: max over elements of
    |got - ref| / (rtol * |ref| + atol_row * max|ref row|) -- <= 1 passes.  The
    absolute part is 0.8 of the normwise 1e-3 bar.  An output element's error
    does not scale with the element: it is the f16 rounding of the
    probabilities (the kernels round unnormalised exponentials, the oracle
    normalised ones, src/utils.h:10) carried through P.V, i.e. a fraction of
    the row's scale.  Measured worst element: 6.6e-4 of its row's max (config
    3, Q8_0, N = 4096).  NaN positions must coincide."""
    got = got.reshape(-1, got.shape[-1]).astype(np.float64)
    ref = ref.reshape(-1, ref.shape[-1]).astype(np.float64)
    gn, rn = np.isnan(got), np.isnan(ref)
    if not np.array_equal(gn, rn):
        return float("inf")
    ok = ~rn.any(axis=1)
    if not ok.any():
        return 0.0
    g, r = got[ok], ref[ok]
    den = rtol * np.abs(r) + atol_row * np.maximum(np.abs(r).max(axis=1, keepdims=True), 1e-30)
    return float((np.abs(g - r) / den).max())
