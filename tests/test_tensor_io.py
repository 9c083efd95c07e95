"""`.tensor` dump IO (src/utils.h:104-150) and the test_llama flow over dumps
(src/flash-matrix.cu:67-339): CPU tests of the format, GPU test of the flow."""
import struct
import zlib

import numpy as np
import pytest

from fattn import tensor_io as tio


def test_roundtrip_f32_f16(tmp_path):
    rng = np.random.default_rng(1)
    a = rng.standard_normal((3, 5, 8)).astype(np.float32)
    tio.save_tensor(str(tmp_path / "a.tensor"), "fa-cuda-q-256", tio.TYPE_F32, (8, 5, 3), a)
    t = tio.load_tensor(str(tmp_path / "a.tensor"))
    assert t.name == "fa-cuda-q-256" and t.type == tio.TYPE_F32 and t.ne == (8, 5, 3)
    assert np.array_equal(t.data, a)
    h = a.astype(np.float16)
    tio.save_tensor(str(tmp_path / "h.tensor"), "k", tio.TYPE_F16, (8, 15), h)
    t = tio.load_tensor(str(tmp_path / "h.tensor"))
    assert t.data.dtype == np.float16 and np.array_equal(t.data.reshape(-1), h.reshape(-1))


def test_layout_matches_reference_reader(tmp_path):
    """Byte layout the reference's load_tensor_from_file reads: int32 n_dims,
    int32 type, int32 ne[n_dims], int32 name_len, name, data."""
    data = np.arange(6, dtype=np.float32)
    raw = struct.pack("<ii", 2, 0) + struct.pack("<ii", 3, 2) + struct.pack("<i", 4) + b"mask" + data.tobytes()
    (tmp_path / "m.tensor").write_bytes(raw)
    t = tio.load_tensor(str(tmp_path / "m.tensor"))
    assert t.ne == (3, 2) and t.name == "mask" and np.array_equal(t.data.reshape(-1), data)
    tio.save_tensor(str(tmp_path / "m2.tensor"), "mask", 0, (3, 2), data)
    assert (tmp_path / "m2.tensor").read_bytes() == raw


def test_long_name_and_quantised(tmp_path):
    """Names past the reference's 20-byte buffer; Q8_0 / Q4_0 payloads as whole blocks."""
    name = "blk.31.attn_k_cache_view-0 (permuted)"
    q8 = np.arange(34 * 4 * 6, dtype=np.uint8) % 251
    tio.save_tensor(str(tmp_path / "q.tensor"), name, tio.TYPE_Q8_0, (128, 6), q8)
    t = tio.load_tensor(str(tmp_path / "q.tensor"))
    assert t.name == name and t.type == tio.TYPE_Q8_0 and np.array_equal(t.data, q8)
    assert tio.data_bytes(tio.TYPE_Q4_0, (64, 3)) == 2 * 18 * 3
    with pytest.raises(ValueError):
        tio.data_bytes(tio.TYPE_Q8_0, (48, 1))


def test_truncated_and_bad_headers(tmp_path):
    p = tmp_path / "t.tensor"
    tio.save_tensor(str(p), "x", tio.TYPE_F32, (4,), np.zeros(4, np.float32))
    raw = p.read_bytes()
    p.write_bytes(raw[:-1])
    with pytest.raises(ValueError):
        tio.load_tensor(str(p))
    p.write_bytes(struct.pack("<ii", 7, 0))
    with pytest.raises(ValueError):
        tio.load_tensor(str(p))
    with pytest.raises(ValueError):
        tio.save_tensor(str(p), "x", tio.TYPE_F32, (5,), np.zeros(4, np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("kt,vtrans", [("f16", False), ("f16", True), ("q8_0", False), ("q4_0", False)])
def test_attention_from_dumps(dev, tmp_path, kt, vtrans):
    """Write a problem as .tensor dumps in the reference's layouts, run the
    test_llama flow through the library, compare with the oracle."""
    from fattn.dumps import attention_from_dumps
    from problems import attn_rel_err, make_problem
    from oracle import oracle as orc
    case = dict(D=128, NQ=3, H=8, Hkv=2, N=256, kv_type=kt, mask="random")
    p = make_problem(seed=zlib.crc32(str(sorted(case.items())).encode()) % 1000, **case)
    D, NQ, H, Hkv, N = 128, 3, 8, 2, 256
    ttype = {"f16": tio.TYPE_F16, "q8_0": tio.TYPE_Q8_0, "q4_0": tio.TYPE_Q4_0}[kt]
    qd = np.ascontiguousarray(p.q[0].transpose(1, 0, 2))          # [H][n_q][D]
    tio.save_tensor(str(tmp_path / "q.tensor"), "q", tio.TYPE_F32, (D, NQ, H), qd)
    tio.save_tensor(str(tmp_path / "k.tensor"), "k", ttype, (D, N, Hkv), p.k_bytes)
    if vtrans:
        v = p.v_bytes.view(np.float16).reshape(Hkv, N, D).transpose(0, 2, 1)   # [Hkv][D][N]
        tio.save_tensor(str(tmp_path / "v.tensor"), "v", tio.TYPE_F16, (N, D, Hkv), np.ascontiguousarray(v))
    else:
        tio.save_tensor(str(tmp_path / "v.tensor"), "v", ttype, (D, N, Hkv), p.v_bytes)
    rows, Np = p.mask_bits.shape
    tio.save_tensor(str(tmp_path / "m.tensor"), "mask", tio.TYPE_F16, (Np, rows), p.mask_bits.view(np.float16))
    ld = lambda n: tio.load_tensor(str(tmp_path / f"{n}.tensor"))
    got = attention_from_dumps(ld("q"), ld("k"), ld("v"), ld("m"), scale=p.scale)
    ref = p.oracle()[0]
    assert attn_rel_err(got[None], ref[None]) <= 1e-3
