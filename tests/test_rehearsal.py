"""The multi-rank bench path, executed: `bench.py --gpus 2` with
FATTN_BENCH_REHEARSE=1 (both ranks on the one GPU of the box, gloo for the
gather -- the driver's N-GPU runs use RCCL over xGMI, this is the same code path
otherwise: rank spawn, the unchanged kernel per rank, the gather).  Two modes:
--multi head (one config-5 problem, n_q 64, 32 heads, N 4096, Q8_0, sliced by
kv heads into zero-copy views, gathered and permuted into the ggml dst layout:
rank 0 dumps rotation 0's inputs and the gathered output) and --multi batch
(every rank decodes its own config-3 sequence; every rank dumps its inputs,
rank 0 the gathered outputs).  --multi head is the default value line at N > 1
(BASELINE configs[4]), with one gather per timed step.  Each output is checked
against the CPU oracle at full size -- SURVEY.md §8(e): sharding must
reproduce the one-GPU result."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as orc
from problems import attn_rel_err

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _oracle_of(d):
    D, NQ, H, Hkv, N, typ, world = (int(x) for x in d["shape"])
    rb = D // 32 * orc.BLOCK_BYTES[typ]
    kv_nb = (orc.BLOCK_BYTES[typ], rb, rb * N, rb * N * Hkv)  # bench's "head" layout
    q = np.ascontiguousarray(d["q"], dtype=np.float32)        # [1][NQ][H][D]
    mask = np.ascontiguousarray(d["mask"])                   # [NQ][Npad] f16 bits
    rows, npad = mask.shape
    return orc.flash_attn_ext((q, orc.TYPE_F32, (D, NQ, H, 1), (4, H * D * 4, D * 4, NQ * H * D * 4)),
                              (d["k"], typ, (D, N, Hkv, 1), kv_nb), (d["v"], typ, (D, N, Hkv, 1), kv_nb),
                              (mask, orc.TYPE_F16, (npad, rows, 1, 1), (2, npad * 2, npad * rows * 2, npad * rows * 2)),
                              float(np.float32(1.0 / D ** 0.5)), n_threads=16)


def _rehearse(tmp_path, mode):
    out = tmp_path / "rank0.npz"
    env = dict(os.environ, FATTN_BENCH_REHEARSE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "4", "--warmup", "2", "--rotate", "2",
           "--no-side-line", "--dump-out", str(out)] + (["--multi", mode] if mode else [])
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    print(lines[0])
    return json.loads(lines[0]), out


@pytest.mark.gpu
def test_bench_rehearsal_batch_shard_matches_oracle(tmp_path):
    line, out = _rehearse(tmp_path, "batch")
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["parallelism"] == "batch_shard_1seq_per_rank_x2"
    assert line["config"]["bytes_per_step"] == 2 * 35692544  # two config-3 sequences
    assert line["gather"]["gathers_timed"] == line["steps"]
    d0 = np.load(out)
    d1 = np.load(str(out) + ".rank1.npz")
    got = d0["out"]  # [world][1][NQ][H][D]: the last step's outputs of every rank
    assert got.shape[0] == 2
    for w, d in enumerate((d0, d1)):
        D, NQ, H, Hkv, N, typ, world = (int(x) for x in d["shape"])
        assert world == 2 and (D, NQ, H, Hkv, N, typ) == (128, 1, 32, 32, 4096, orc.TYPE_Q8_0)
        ref = _oracle_of(d)
        assert attn_rel_err(got[w].reshape(ref.shape), ref) <= 1e-3, f"sequence of rank {w}"
    assert not np.array_equal(d0["k"], d1["k"])  # the ranks decode different sequences


@pytest.mark.gpu
def test_bench_rehearsal_two_ranks_matches_oracle(tmp_path):
    line, out = _rehearse(tmp_path, None)  # the default N > 1 value line
    assert line["scaling"] == "strong"
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "head_shard_16heads_per_rank_x2"
    assert line["config"]["bytes_per_step"] == 38273024  # BASELINE config 5
    assert line["gather"]["gathers_timed"] == line["steps"]  # one gather per timed step
    assert line["kernel_only"]["value"] > 0
    assert "gather" in line and line["gather"]["per_step_gather_ms_median"] > 0
    d = np.load(out)
    D, NQ, H, Hkv, N, typ, world = (int(x) for x in d["shape"])
    assert world == 2 and (D, NQ, H, Hkv, N, typ) == (128, 64, 32, 32, 4096, orc.TYPE_Q8_0)
    ref = _oracle_of(d)
    got = d["out"].reshape(ref.shape)
    assert attn_rel_err(got, ref) <= 1e-3


def _world1_nccl(tmp_path, mode, extra=()):
    """bench.py --dist under torch.distributed.run with one rank: a real RCCL
    group (init_process_group("nccl", device_id=...)), the per-step
    all_gather_into_tensor on device tensors and its HIP-graph capture -- the
    calls the driver's N-GPU runs make, executed on the one-GPU box."""
    import socket
    out = tmp_path / "rank0.npz"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("FATTN_BENCH_REHEARSE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={port}", "bench.py", "--dist", "--steps", "6",
           "--warmup", "2", "--rotate", "3", "--no-side-line", "--multi", mode, "--dump-out", str(out), *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    print(lines[0])
    return json.loads(lines[0]), out


@pytest.mark.gpu
@pytest.mark.parametrize("eager", [False, True])
def test_bench_nccl_world1_head_matches_oracle(tmp_path, eager):
    line, out = _world1_nccl(tmp_path, "head", ["--eager-gather"] if eager else [])
    assert "rehearsal" not in line and line["n_gpus"] == 1 and "world1" in line
    assert line["config"]["parallelism"] == "head_shard_32heads_per_rank_x1"
    assert line["config"]["bytes_per_step"] == 38273024
    g = line["gather"]
    assert g["gathers_timed"] == line["steps"]
    if eager:
        assert g["timing"] == "eager" and g["device_ms_per_step"] is None
    else:
        # RCCL's all_gather captures into the HIP graph; the line reports the
        # device-side per-step time next to the wall time
        assert g["timing"] == "graph", g["graph_capture_error"]
        assert 0 < g["device_ms_per_step"] <= g["wall_ms_per_step"] * 1.05
    d = np.load(out)
    D, NQ, H, Hkv, N, typ, world = (int(x) for x in d["shape"])
    assert world == 1 and (D, NQ, H, Hkv, N, typ) == (128, 64, 32, 32, 4096, orc.TYPE_Q8_0)
    ref = _oracle_of(d)
    assert attn_rel_err(d["out"].reshape(ref.shape), ref) <= 1e-3


@pytest.mark.gpu
def test_bench_nccl_world1_batch_matches_oracle(tmp_path):
    line, out = _world1_nccl(tmp_path, "batch")
    assert line["scaling"] == "weak" and line["gather"]["timing"] == "graph"
    d = np.load(out)
    got = d["out"]  # [world=1][1][NQ][H][D]
    ref = _oracle_of(d)
    assert attn_rel_err(got[0].reshape(ref.shape), ref) <= 1e-3
