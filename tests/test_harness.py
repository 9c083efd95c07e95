"""The kernel_test harness (ggml-cuda-experiments_amd/host/kernel_test.cpp, the
counterpart of src/kernel_test.h:1-249).

CPU: its host-only mode (BASELINE config 1, `--cpu-only`) must reproduce the
REFERENCE's own CPU output bit for bit -- tests/golden/ holds what
src/utils.h (compiled from /root/reference, oracle/gen_golden.py) printed for
the same srand(1) inputs -- which pins the harness's CPU reference
(kernel_test.cpp cpu_reference) to the reference.
GPU: both of its branches run and pass their own max-diff check.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "ggml-cuda-experiments_amd", "bin", "kernel_test")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _need_bin():
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} not built (make harness)")


@pytest.mark.parametrize("fixture,args", [
    ("kernel_test_cfg1.npz", ["--heads", "1", "--kv-heads", "1", "--head-dim", "64", "--kv-size", "128"]),
    ("kernel_test_default.npz", []),
])
def test_cpu_only_matches_reference_bitexact(tmp_path, fixture, args):
    _need_bin()
    out = tmp_path / "out.bin"
    r = subprocess.run([BIN, "--cpu-only", "--dump", str(out)] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.float32)
    ref = np.load(os.path.join(GOLDEN, fixture))["out"]
    assert got.shape == ref.shape
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert "Reference" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    [],                                                    # flash_attn_row + fa_reduce, f16, V transposed
    ["--no-kv-parallel"],                                  # flash_attn_ext call of kernel_test.h:191-198
    ["--no-kv-parallel", "--kv-type", "q8_0"],
    ["--no-kv-parallel", "--kv-type", "q4_0"],
    ["--kv-size", "4096"],
    ["--no-kv-parallel", "--kv-type", "q8_0", "--kv-size", "4096", "--kv-heads", "32"],
    ["--no-kv-parallel", "--kv-size", "1001"],             # odd kv size: mask rows padded to even
    ["--no-kv-parallel", "--kv-size", "65536"],            # workspace sized by fattn_workspace_size
    ["--config", "2"],                                     # BASELINE configs through the harness
    ["--config", "3"],
    ["--config", "4"],
    ["--config", "5"],                                     # n_q = 64 (the ext branch's ne01)
    ["--config", "prefill", "--check-rows", "32"],         # n_q = N = 4096, zero mask, 3 x 32 rows checked
    ["--config", "3", "--n-q", "7", "--mask", "none"],     # ragged n_q, no mask
    ["--config", "5", "--ngpu", "1"],                      # the --ngpu path (RCCL not needed at 1)
], ids=lambda a: "_".join(a) or "default")
def test_harness_runs_on_gpu(dev, args):
    _need_bin()
    r = subprocess.run([BIN, "--iters", "3"] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout


def test_cpu_only_config_presets_and_n_q(tmp_path):
    """--config presets and --n-q on the host-only path: config 1 is the
    reference's kernel_test call (same bits as the fixture); an n_q = 3 run
    writes three finite, distinct query rows (the rand() stream then fills Q,
    K, V and the mask rows in kernel_test.h's order, so K differs from the
    n_q = 1 run's)."""
    _need_bin()
    out = tmp_path / "c1.bin"
    r = subprocess.run([BIN, "--config", "1", "--dump", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ref = np.load(os.path.join(GOLDEN, "kernel_test_cfg1.npz"))["out"]
    assert np.array_equal(np.fromfile(out, dtype=np.float32).view(np.uint32), ref.view(np.uint32))
    r = subprocess.run([BIN, "--config", "9"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
    a, b = tmp_path / "a.bin", tmp_path / "b.bin"
    base = [BIN, "--cpu-only", "--heads", "2", "--kv-heads", "1", "--head-dim", "64", "--kv-size", "96", "--mask", "zero"]
    assert subprocess.run(base + ["--dump", str(a)], capture_output=True, timeout=60).returncode == 0
    assert subprocess.run(base + ["--n-q", "3", "--dump", str(b)], capture_output=True, timeout=60).returncode == 0
    one, three = np.fromfile(a, dtype=np.float32), np.fromfile(b, dtype=np.float32)
    assert three.size == 3 * one.size and np.isfinite(three).all()
    rows = three.reshape(3, -1)
    assert not np.array_equal(rows[0], rows[1]) and not np.array_equal(rows[1], rows[2])
