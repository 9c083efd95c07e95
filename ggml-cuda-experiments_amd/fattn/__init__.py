"""Host-side mirror of the reference's attention interface, over libfattn.so.

The reference drives its kernels from C++ host code (src/kernel_test.h,
src/flash-matrix.cu) with ggml ne/nb views (src/flash-llama.h:7-32).  This
package is the Python face of the same boundary: it binds the C ABI declared
in include/fattn.h with ctypes and takes device pointers from torch tensors
(torch is plumbing here: device memory and the current HIP stream).

There is no fallback: if libfattn.so is missing or fails to load, every entry
point raises.  Nothing here imports the test oracle.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional, Sequence

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_PKG_DIR, "..", "lib", os.environ.get("FATTN_LIB", "libfattn.so")))

# ggml_type numbering (include/fattn.h)
TYPE_F32, TYPE_F16, TYPE_Q4_0, TYPE_Q8_0 = 0, 1, 2, 8
TYPE_NAMES = {"f32": TYPE_F32, "f16": TYPE_F16, "q4_0": TYPE_Q4_0, "q8_0": TYPE_Q8_0}
BLOCK_BYTES = {TYPE_Q8_0: 34, TYPE_Q4_0: 18}

FATTN_OK = 0
ERRORS = {
    -1: "FATTN_ERR_INVALID_ARG", -2: "FATTN_ERR_UNSUPPORTED_TYPE", -3: "FATTN_ERR_UNSUPPORTED_HEAD_DIM",
    -4: "FATTN_ERR_BAD_STRIDE", -5: "FATTN_ERR_WORKSPACE", -6: "FATTN_ERR_LAUNCH", -7: "FATTN_ERR_ALIGNMENT",
}

# every symbol include/fattn.h and include/fattn_debug.h declare
EXPORTS = (
    "fattn_workspace_size", "fattn_workspace_init", "fattn_ext", "fattn_ext_events", "fattn_ext_f16_launch", "fattn_row_workspace_size", "fattn_row",
    "fattn_dequantize", "fattn_quantize", "fattn_strerror", "fattn_row_size", "fattn_version", "fattn_set_option",
    "fattn_describe", "fattn_cpy",
)
OPT_MQ_ROWS_PER_WAVE = 1
OPT_MQ_DISABLE = 2
OPT_SPLIT_STEPS = 3
OPT_SPLIT_INFLIGHT = 4
OPT_PF = 5
OPT_PF_STAGGER = 6
OPT_SPLIT_WAVE_MERGE = 10
OPT_SPLIT_PRIO = 11
OPT_PF_SKIP = 12
OPT_MQ_MIN_ROWS = 13
OPT_SPLIT_WAVES = 19
OPT_SPLIT_SKIP = 20
OPT_SPLIT_MERGE = 21
OPT_BD = 22
OPT_MERGE_IN_KERNEL = 24
OPT_BD_XCD = 25
OPT_SPLIT_XCD = 26
OPT_PF_STAGE = 28
OPT_PF_FORM = 29
OPT_SPLIT_LOADERS = 30
OPT_MERGE_PLAIN = 31
OPT_PART_F16 = 32
OPT_GQA_UNPACK = 33
# every option's default (include/fattn_debug.h): reset_options() restores them
OPTION_DEFAULTS = {
    OPT_MQ_ROWS_PER_WAVE: 0, OPT_MQ_DISABLE: 0, OPT_SPLIT_STEPS: 0, OPT_SPLIT_INFLIGHT: 0, OPT_PF: 0,
    OPT_PF_STAGGER: 2, OPT_SPLIT_WAVE_MERGE: 0, OPT_SPLIT_PRIO: 0, OPT_PF_SKIP: 0, OPT_MQ_MIN_ROWS: 0,
    OPT_SPLIT_WAVES: 0, OPT_SPLIT_SKIP: 0, OPT_SPLIT_MERGE: 0, OPT_BD: 0, OPT_MERGE_IN_KERNEL: 0, OPT_BD_XCD: 0, OPT_SPLIT_XCD: 0,
    OPT_PF_STAGE: 0, OPT_PF_FORM: 0, OPT_SPLIT_LOADERS: 0, OPT_MERGE_PLAIN: 0, OPT_PART_F16: 0, OPT_GQA_UNPACK: 0,
}


class FattnError(RuntimeError):
    def __init__(self, code: int, what: str):
        self.code = code
        super().__init__(f"{what}: {ERRORS.get(code, code)} ({code})")


class FattnTensor(C.Structure):
    _fields_ = [("data", C.c_void_p), ("type", C.c_int32), ("pad_", C.c_int32),
                ("ne", C.c_int64 * 4), ("nb", C.c_int64 * 4)]


class FattnParams(C.Structure):
    _fields_ = [("q", FattnTensor), ("k", FattnTensor), ("v", FattnTensor), ("mask", FattnTensor),
                ("dst", C.c_void_p), ("scale", C.c_float), ("kv_chunk", C.c_int32),
                ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t)]


_lib = None


def lib() -> C.CDLL:
    """Load libfattn.so (fails loudly -- there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libfattn.so not built at {LIB_PATH}; run `make lib` (or __graft_entry__.build())")
        # torch's HIP runtime must be the process's one: libfattn.so's
        # libamdhip64.so.7 dependency then binds to it.  Loaded first, the
        # library would pull in /opt/rocm's runtime beside torch's and see no
        # device through it.
        import torch  # noqa: F401
        L = C.CDLL(LIB_PATH)
        vp, i64, sz = C.c_void_p, C.c_int64, C.c_size_t
        L.fattn_workspace_size.restype = sz
        L.fattn_workspace_size.argtypes = [C.POINTER(FattnParams)]
        L.fattn_set_option.restype = C.c_int
        L.fattn_set_option.argtypes = [C.c_int, C.c_int]
        L.fattn_workspace_init.restype = C.c_int
        L.fattn_workspace_init.argtypes = [vp, sz, vp]
        L.fattn_ext.restype = C.c_int
        L.fattn_ext.argtypes = [C.POINTER(FattnParams), vp]
        L.fattn_ext_events.restype = C.c_int
        L.fattn_ext_events.argtypes = [C.POINTER(FattnParams), vp, vp, vp]
        L.fattn_ext_f16_launch.restype = C.c_int
        L.fattn_ext_f16_launch.argtypes = ([vp, vp, vp, vp, vp, C.c_float] + [C.c_int] * 20 +
                                           [C.c_int, C.c_int, vp, sz, vp])
        L.fattn_row_workspace_size.restype = sz
        L.fattn_row_workspace_size.argtypes = [C.c_int, C.c_int, C.c_int]
        L.fattn_row.restype = C.c_int
        L.fattn_row.argtypes = [vp, vp, vp, vp, vp, sz, vp, C.c_int, C.c_int, C.c_int, C.c_float, C.c_int, C.c_int,
                                vp]
        L.fattn_dequantize.restype = C.c_int
        L.fattn_dequantize.argtypes = [C.c_int, vp, vp, i64, i64, vp]
        L.fattn_quantize.restype = C.c_int
        L.fattn_quantize.argtypes = [C.c_int, vp, vp, i64, i64, vp]
        L.fattn_strerror.restype = C.c_char_p
        L.fattn_strerror.argtypes = [C.c_int]
        L.fattn_row_size.restype = sz
        L.fattn_row_size.argtypes = [C.c_int, i64]
        L.fattn_version.restype = C.c_char_p
        L.fattn_cpy.restype = C.c_int
        L.fattn_cpy.argtypes = [C.POINTER(FattnTensor), C.POINTER(FattnTensor), vp]
        L.fattn_describe.restype = C.c_int
        L.fattn_describe.argtypes = [C.POINTER(FattnParams), C.c_char_p, sz]
        _lib = L
    return _lib


def _check(rc: int, what: str):
    if rc != FATTN_OK:
        raise FattnError(rc, what)


def set_option(option: int, value: int):
    """Planner override (include/fattn_debug.h fattn_set_option): OPT_MQ_ROWS_PER_WAVE
    (0 auto, 16, 32), OPT_MQ_DISABLE (1 = split-KV kernel only), OPT_SPLIT_STEPS
    (32-position steps per wave, 0 auto) or OPT_SPLIT_INFLIGHT (steps in flight, 0 auto)."""
    _check(lib().fattn_set_option(option, value), "fattn_set_option")


def reset_options():
    """Every planner override back to its default (the process-wide state of
    fattn_set_option; tests reset it after each case so a failing one cannot
    leak an override into the next)."""
    for opt, val in OPTION_DEFAULTS.items():
        set_option(opt, val)


class options:
    """Context manager: set planner overrides for a block, restore the defaults
    on exit (also when the block raises).  `with fattn.options({OPT_BD: 2}): ...`"""

    def __init__(self, opts: dict):
        self.opts = dict(opts)

    def __enter__(self):
        try:
            for opt, val in self.opts.items():
                set_option(opt, val)
        except Exception:
            reset_options()
            raise
        return self

    def __exit__(self, *exc):
        reset_options()
        return False


def row_size(typ: int, k: int) -> int:
    return int(lib().fattn_row_size(typ, k))


def strerror(code: int) -> str:
    return lib().fattn_strerror(code).decode()


@dataclass
class View:
    """A ggml tensor view: device pointer, ggml type, ne (elements), nb (bytes)."""
    ptr: int
    type: int
    ne: Sequence[int]
    nb: Sequence[int]

    def c(self) -> FattnTensor:
        t = FattnTensor()
        t.data = self.ptr
        t.type = self.type
        for i in range(4):
            t.ne[i] = int(self.ne[i])
            t.nb[i] = int(self.nb[i])
        return t


def _stream(stream) -> Optional[int]:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return int(stream)


def ext_params(q: View, k: View, v: View, mask: Optional[View], dst_ptr: int, scale: float,
               workspace_ptr: int = 0, workspace_bytes: int = 0, kv_chunk: int = 0) -> FattnParams:
    p = FattnParams()
    p.q, p.k, p.v = q.c(), k.c(), v.c()
    if mask is not None:
        p.mask = mask.c()
    p.dst = dst_ptr
    p.scale = float(scale)
    p.kv_chunk = int(kv_chunk)
    p.workspace = workspace_ptr or None
    p.workspace_bytes = int(workspace_bytes)
    return p


def workspace_size(p: FattnParams) -> int:
    return int(lib().fattn_workspace_size(C.byref(p)))


def describe(p: FattnParams) -> str:
    """The kernel(s) and plan fattn_ext would launch for these params (diagnostic)."""
    buf = C.create_string_buffer(512)
    _check(lib().fattn_describe(C.byref(p), buf, len(buf)), "fattn_describe")
    return buf.value.decode()


def flash_attn_ext(p: FattnParams, stream=None, ev_begin=None, ev_end=None):
    """GGML_OP_FLASH_ATTN_EXT on the GPU (replaces flash_attn_ext_f16, src/flash-llama.h:5-32).
    ev_begin/ev_end: optional raw hipEvent_t handles recorded around the main kernel."""
    if ev_begin is None and ev_end is None:
        _check(lib().fattn_ext(C.byref(p), _stream(stream)), "fattn_ext")
    else:
        _check(lib().fattn_ext_events(C.byref(p), _stream(stream), ev_begin, ev_end), "fattn_ext_events")


# ------------------------------------------------------------------ torch helpers

def _tptr(t) -> int:
    return int(t.data_ptr())


def kv_view(buf, typ: int, D: int, N: int, Hkv: int, S: int = 1, layout: str = "head") -> View:
    """View of a KV cache held in a byte (or f16) torch tensor.

    layout "head": [S][Hkv][N][row]   (per-head contiguous; reference decode layout,
                   src/flash_row_float.h:19,58)
    layout "pos":  [S][N][Hkv][row]   (llama.cpp's KV cache: nb1 = Hkv * row)
    """
    rb = row_size(typ, D)
    nb0 = 2 if typ == TYPE_F16 else BLOCK_BYTES[typ]
    if layout == "head":
        nb = (nb0, rb, rb * N, rb * N * Hkv)
    elif layout == "pos":
        nb = (nb0, rb * Hkv, rb, rb * N * Hkv)
    else:
        raise ValueError(layout)
    return View(_tptr(buf), typ, (D, N, Hkv, S), nb)


def q_view(q) -> View:
    """q: torch f32 contiguous [S][n_q][H][D] (ggml ne = [D, n_q, H, S] with
    nb1 = H*D*4: the permuted query of llama.cpp) -- or any tensor with the
    ggml strides supplied via q_view_strided."""
    S, NQ, H, D = q.shape
    return View(_tptr(q), TYPE_F32, (D, NQ, H, S), (4, H * D * 4, D * 4, NQ * H * D * 4))


def mask_view(mask) -> View:
    """mask: torch f16 [rows][N_padded] (ggml ne = [N, rows])."""
    rows, Np = mask.shape
    return View(_tptr(mask), TYPE_F16, (Np, rows, 1, 1), (2, Np * 2, Np * rows * 2, Np * rows * 2))


class Attention:
    """Reusable FLASH_ATTN_EXT call: builds the params once, owns its workspace."""

    def __init__(self, q: View, k: View, v: View, mask: Optional[View], dst, scale: float, kv_chunk: int = 0):
        import torch
        self.p = ext_params(q, k, v, mask, _tptr(dst), scale, 0, 0, kv_chunk)
        ws = workspace_size(self.p)
        # (zeroing is optional: each launch epoch-stamps the arrival words at its front)
        self.workspace = torch.zeros(max(ws, 16), dtype=torch.uint8, device=dst.device)
        self.p.workspace = _tptr(self.workspace)
        self.p.workspace_bytes = self.workspace.numel()
        self.dst = dst

    def retarget(self, q=None, k=None, v=None, dst=None, mask=None):
        """Point the same call at other buffers with identical shapes/strides."""
        if mask is not None:
            self.p.mask.data = mask
        if q is not None:
            self.p.q.data = q
        if k is not None:
            self.p.k.data = k
        if v is not None:
            self.p.v.data = v
        if dst is not None:
            self.p.dst = dst

    def describe(self) -> str:
        return describe(self.p)

    def __call__(self, stream=None, ev_begin=None, ev_end=None):
        flash_attn_ext(self.p, stream, ev_begin, ev_end)
        return self.dst


def quantize(x, typ: int, stream=None):
    """f32 [rows, k] (cuda) -> ggml blocks uint8 [rows, k/32*bytes] (bit-exact ggml quantize_row_*_ref)."""
    import torch
    assert x.dtype == torch.float32 and x.is_contiguous()
    k = x.shape[-1]
    rows = x.numel() // k
    out = torch.empty((rows, row_size(typ, k)), dtype=torch.uint8, device=x.device)
    _check(lib().fattn_quantize(typ, _tptr(x), _tptr(out), k, rows, _stream(stream)), "fattn_quantize")
    return out


def cpy(src: View, dst: View, stream=None):
    """GGML_OP_CPY f32 -> F16 / Q8_0 / Q4_0 into a strided view (the KV-cache
    write, include/fattn.h fattn_cpy); src/dst are ggml views of device memory."""
    s, d = src.c(), dst.c()
    _check(lib().fattn_cpy(C.byref(s), C.byref(d), _stream(stream)), "fattn_cpy")


def dequantize(blocks, typ: int, k: int, stream=None):
    """ggml blocks (or f16 bits) -> f32 [rows, k] (bit-exact ggml dequantize_row_*)."""
    import torch
    rows = blocks.numel() * (1 if typ != TYPE_F16 else blocks.element_size()) // max(1, row_size(typ, k))
    out = torch.empty((rows, k), dtype=torch.float32, device=blocks.device)
    _check(lib().fattn_dequantize(typ, _tptr(blocks), _tptr(out), k, rows, _stream(stream)), "fattn_dequantize")
    return out


def row(query, key, value_t, mask, qkv, head_dim: int, kv_size: int, num_heads: int, scale: float,
        head_stride: int, r_kv_heads: int, tmp=None, stream=None):
    """flash_attn_row + fa_reduce (src/flash_row_float.h:4-6,415-416): key f16
    [Hkv][N][D], value f16 transposed [Hkv][D][N], mask f16 [N], qkv f32 [H][D]."""
    import torch
    need = int(lib().fattn_row_workspace_size(head_dim, kv_size, num_heads))
    if tmp is None:
        tmp = torch.zeros(max(need, 16), dtype=torch.uint8, device=qkv.device)
    _check(lib().fattn_row(_tptr(query), _tptr(key), _tptr(value_t), _tptr(mask) if mask is not None else None,
                           _tptr(tmp), tmp.numel() * tmp.element_size(), _tptr(qkv), head_dim, kv_size, num_heads,
                           float(scale), head_stride, r_kv_heads, _stream(stream)), "fattn_row")
    return qkv
