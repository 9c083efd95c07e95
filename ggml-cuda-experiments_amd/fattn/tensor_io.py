""".tensor dump files (the reference's golden-data format, src/utils.h:104-150).

Layout, little endian:
    int32 n_dims, int32 type, int32 ne[n_dims], int32 name_len, name bytes,
    then the data: ne[0] * ... * ne[n_dims-1] elements.

The reference reads type 1 as f16 and anything else as f32, into a 20-byte name
buffer.  This reader takes the ggml type ids the library uses (0 f32, 1 f16,
2 Q4_0, 8 Q8_0; quantised data is whole ggml blocks along ne[0]) and names of
any length -- the reference overflows its buffer past 19 bytes
(src/utils.h:106,130-131).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import numpy as np

TYPE_F32, TYPE_F16, TYPE_Q4_0, TYPE_Q8_0 = 0, 1, 2, 8
_BLOCK = {TYPE_Q4_0: (32, 18), TYPE_Q8_0: (32, 34)}  # (elements, bytes) per ggml block


@dataclass
class Tensor:
    name: str
    type: int
    ne: tuple          # ggml order: ne[0] is the contiguous dimension
    data: np.ndarray   # f32 / f16 array shaped reversed(ne), or raw uint8 blocks for Q8_0 / Q4_0

    @property
    def nbytes(self) -> int:
        return data_bytes(self.type, self.ne)


def data_bytes(ttype: int, ne) -> int:
    n = 1
    for x in ne:
        n *= int(x)
    if ttype == TYPE_F32:
        return 4 * n
    if ttype == TYPE_F16:
        return 2 * n
    if ttype in _BLOCK:
        per, size = _BLOCK[ttype]
        if int(ne[0]) % per:
            raise ValueError(f"ne[0]={ne[0]} is not a multiple of the {per}-element block")
        return n // per * size
    raise ValueError(f"unsupported tensor type {ttype}")


def load_tensor(path: str) -> Tensor:
    with open(path, "rb") as f:
        raw = f.read()
    off = 0

    def i32():
        nonlocal off
        if off + 4 > len(raw):
            raise ValueError(f"{path}: truncated header")
        (v,) = struct.unpack_from("<i", raw, off)
        off += 4
        return v

    n_dims = i32()
    ttype = i32()
    if not 1 <= n_dims <= 4:
        raise ValueError(f"{path}: n_dims={n_dims}")
    ne = tuple(i32() for _ in range(n_dims))
    if any(x <= 0 for x in ne):
        raise ValueError(f"{path}: ne={ne}")
    nlen = i32()
    if nlen < 0 or off + nlen > len(raw):
        raise ValueError(f"{path}: name length {nlen}")
    name = raw[off:off + nlen].decode("utf-8", "replace")
    off += nlen
    nb = data_bytes(ttype, ne)
    if off + nb > len(raw):
        raise ValueError(f"{path}: {len(raw) - off} data bytes, {nb} expected")
    buf = np.frombuffer(raw, dtype=np.uint8, count=nb, offset=off).copy()
    shape = tuple(reversed(ne))
    if ttype == TYPE_F32:
        data = buf.view(np.float32).reshape(shape)
    elif ttype == TYPE_F16:
        data = buf.view(np.float16).reshape(shape)
    else:
        data = buf
    return Tensor(name, ttype, ne, data)


def save_tensor(path: str, name: str, ttype: int, ne, data) -> None:
    ne = tuple(int(x) for x in ne)
    payload = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    if payload.size != data_bytes(ttype, ne):
        raise ValueError(f"{payload.size} data bytes for type {ttype} ne={ne}")
    nm = name.encode("utf-8")
    with open(path, "wb") as f:
        f.write(struct.pack("<ii", len(ne), ttype))
        f.write(struct.pack(f"<{len(ne)}i", *ne))
        f.write(struct.pack("<i", len(nm)))
        f.write(nm)
        f.write(payload.tobytes())
