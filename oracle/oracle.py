"""ctypes bindings for the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product path (ggml-cuda-experiments_amd/fattn, libfattn.so,
the kernel_test harness) never does.

Two libraries:
  liboracle.so          C restatement of the reference's CPU oracle
                        (src/utils.h:5-61, src/kernel_test.h:50-62) plus the
                        upstream-ggml Q8_0/Q4_0 block formats; fattn_oracle.c.
  _ref/libref_utils.so  the reference's OWN src/utils.h compiled from
                        /root/reference (oracle/Makefile); used to pin the
                        restatement and as the CPU baseline ("kind":"reference").
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
TYPE_F32, TYPE_F16, TYPE_Q4_0, TYPE_Q8_0 = 0, 1, 2, 8
BLOCK_BYTES = {TYPE_Q8_0: 34, TYPE_Q4_0: 18}

_fp = C.POINTER(C.c_float)
_u16p = C.POINTER(C.c_uint16)


def _ptr(a: np.ndarray, t=C.c_void_p):
    return a.ctypes.data_as(t) if a is not None else None


class OrcTensor(C.Structure):
    _fields_ = [("data", C.c_void_p), ("type", C.c_int32), ("ne", C.c_int64 * 4), ("nb", C.c_int64 * 4)]


def _load(path):
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built (run `make oracle`)")
    return C.CDLL(path)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load(os.path.join(_HERE, "liboracle.so"))
        L = _lib
        L.orc_f32_to_f16.restype = C.c_uint16
        L.orc_f32_to_f16.argtypes = [C.c_float]
        L.orc_f16_to_f32.restype = C.c_float
        L.orc_f16_to_f32.argtypes = [C.c_uint16]
        L.orc_f32_to_f16_n.argtypes = [_fp, _u16p, C.c_int64]
        L.orc_f16_to_f32_n.argtypes = [_u16p, _fp, C.c_int64]
        L.orc_mulmat_f32.argtypes = [_fp, _fp, _fp, _fp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_float, C.c_int]
        L.orc_mulmat_f16.argtypes = [_fp, _u16p, _u16p, _fp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_float, C.c_int]
        L.orc_softmax.argtypes = [_fp, C.c_int, C.c_int]
        L.orc_random.argtypes = [_fp, C.c_uint32]
        L.orc_srand.argtypes = [C.c_uint]
        L.orc_kernel_test_cpu.argtypes = [_fp, _fp, _fp, _fp, _fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float]
        for n in ("orc_quantize_row_q8_0", "orc_quantize_row_q4_0"):
            getattr(L, n).argtypes = [_fp, C.c_void_p, C.c_int64]
        for n in ("orc_dequantize_row_q8_0", "orc_dequantize_row_q4_0"):
            getattr(L, n).argtypes = [C.c_void_p, _fp, C.c_int64]
        L.orc_flash_attn_ext.argtypes = [C.POINTER(OrcTensor)] * 4 + [_fp, C.c_float, C.c_int]
        L.orc_flash_attn_ext.restype = C.c_int
    return _lib


def ref_available() -> bool:
    return os.path.exists(os.path.join(_HERE, "_ref", "libref_utils.so"))


def ref():
    global _ref
    if _ref is None:
        _ref = _load(os.path.join(_HERE, "_ref", "libref_utils.so"))
        R = _ref
        R.ref_mulmat_f32.argtypes = [_fp, _fp, _fp, _fp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_float, C.c_int]
        R.ref_mulmat_f16.argtypes = [_fp, _u16p, _u16p, _fp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_float, C.c_int]
        R.ref_softmax.argtypes = [_fp, C.c_int, C.c_int]
        R.ref_random.argtypes = [_fp, C.c_uint32]
        R.ref_srand.argtypes = [C.c_uint]
        R.ref_float2half.restype = C.c_uint16
        R.ref_float2half.argtypes = [C.c_float]
        R.ref_half2float.restype = C.c_float
        R.ref_half2float.argtypes = [C.c_uint16]
        R.ref_kernel_test_cpu.argtypes = [_fp, _fp, _fp, _fp, _fp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float,
                                          C.c_int]
    return _ref


# ------------------------------------------------------------------ helpers

def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def f32_to_f16_bits(x: np.ndarray) -> np.ndarray:
    x = f32(x)
    out = np.empty(x.shape, dtype=np.uint16)
    lib().orc_f32_to_f16_n(_ptr(x, _fp), _ptr(out, _u16p), x.size)
    return out


def f16_bits_to_f32(h: np.ndarray) -> np.ndarray:
    h = np.ascontiguousarray(h, dtype=np.uint16)
    out = np.empty(h.shape, dtype=np.float32)
    lib().orc_f16_to_f32_n(_ptr(h, _u16p), _ptr(out, _fp), h.size)
    return out


def random(count: int, impl: str = "oracle") -> np.ndarray:
    """src/utils.h:57-61 -- continues the process-global rand() stream."""
    out = np.empty(count, dtype=np.float32)
    (lib().orc_random if impl == "oracle" else ref().ref_random)(_ptr(out, _fp), count)
    return out


def srand(seed: int, impl: str = "oracle"):
    (lib().orc_srand if impl == "oracle" else ref().ref_srand)(seed)


def mulmat_f32(A, B, mask, M, N, K, scale, B_transposed, impl="oracle"):
    A, B = f32(A), f32(B)
    mask = f32(mask) if mask is not None else None
    C_ = np.zeros(M * N, dtype=np.float32)
    fn = lib().orc_mulmat_f32 if impl == "oracle" else ref().ref_mulmat_f32
    fn(_ptr(A, _fp), _ptr(B, _fp), _ptr(mask, _fp) if mask is not None else None, _ptr(C_, _fp), M, N, K,
       scale, int(B_transposed))
    return C_


def softmax(scores, kv_size, batch, impl="oracle"):
    s = f32(scores).copy()
    (lib().orc_softmax if impl == "oracle" else ref().ref_softmax)(_ptr(s, _fp), kv_size, batch)
    return s


def kernel_test_cpu(query, key, value, mask, kv_size, head_dim, num_heads, num_kv_heads, scale=None,
                    impl="oracle", n_threads=1):
    """src/kernel_test.h:50-62."""
    scale = 1.0 / np.sqrt(np.float32(head_dim)) if scale is None else scale
    query, key, value, mask = f32(query), f32(key), f32(value), f32(mask)
    out = np.zeros(num_heads * head_dim, dtype=np.float32)
    if impl == "oracle":
        lib().orc_kernel_test_cpu(_ptr(query, _fp), _ptr(key, _fp), _ptr(value, _fp), _ptr(mask, _fp),
                                  _ptr(out, _fp), kv_size, head_dim, num_heads, num_kv_heads, np.float32(scale))
    else:
        ref().ref_kernel_test_cpu(_ptr(query, _fp), _ptr(key, _fp), _ptr(value, _fp), _ptr(mask, _fp),
                                  _ptr(out, _fp), kv_size, head_dim, num_heads, num_kv_heads, np.float32(scale),
                                  n_threads)
    return out


def quantize(x: np.ndarray, typ: int) -> np.ndarray:
    """ggml quantize_row_{q8_0,q4_0}_ref over the last axis -> uint8 blocks."""
    x = f32(x)
    k = x.shape[-1]
    assert k % 32 == 0
    rows = x.size // k
    out = np.empty((rows, k // 32 * BLOCK_BYTES[typ]), dtype=np.uint8)
    fn = lib().orc_quantize_row_q8_0 if typ == TYPE_Q8_0 else lib().orc_quantize_row_q4_0
    fn(_ptr(x, _fp), _ptr(out), x.size)
    return out.reshape(x.shape[:-1] + (k // 32 * BLOCK_BYTES[typ],))


def dequantize(blocks: np.ndarray, typ: int, k: int) -> np.ndarray:
    blocks = np.ascontiguousarray(blocks, dtype=np.uint8)
    n = blocks.size // BLOCK_BYTES[typ] * 32
    out = np.empty(n, dtype=np.float32)
    fn = lib().orc_dequantize_row_q8_0 if typ == TYPE_Q8_0 else lib().orc_dequantize_row_q4_0
    fn(_ptr(blocks), _ptr(out, _fp), n)
    return out.reshape(blocks.shape[:-1] + (k,))


def type_elem_bytes(typ):
    return {TYPE_F32: 4, TYPE_F16: 2}[typ]


def tensor(buf: np.ndarray, typ: int, ne, nb) -> OrcTensor:
    t = OrcTensor()
    t.data = buf.ctypes.data if buf is not None else None
    t.type = typ
    for i in range(4):
        t.ne[i] = int(ne[i])
        t.nb[i] = int(nb[i])
    return t


def flash_attn_ext(q, k, v, mask, scale, n_threads=8):
    """Oracle FLASH_ATTN_EXT.  q, k, v, mask are (buffer, type, ne, nb) tuples of
    numpy byte buffers; returns dst f32 [S][n_q][H][D]."""
    qt, kt, vt = (tensor(*x) for x in (q, k, v))
    mt = tensor(*mask) if mask is not None else tensor(None, TYPE_F16, (0, 0, 1, 1), (2, 0, 0, 0))
    D, NQ, H, S = (int(x) for x in q[2])
    dst = np.zeros(S * NQ * H * D, dtype=np.float32)
    rc = lib().orc_flash_attn_ext(C.byref(qt), C.byref(kt), C.byref(vt), C.byref(mt), _ptr(dst, _fp),
                                  np.float32(scale), n_threads)
    if rc != 0:
        raise RuntimeError(f"orc_flash_attn_ext failed: {rc}")
    return dst.reshape(S, NQ, H, D)
