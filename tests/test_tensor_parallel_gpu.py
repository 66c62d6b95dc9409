"""MI355X: the tensor-sharded toy-MLP step (parallel/tensor_parallel.py) with real peers on one
GPU (the peer-memory vehicle: collectives as device kernels, capturable): captured == eager
bitwise, both == the one-process global-batch step; and bench.py's --parallel tensor / auto."""
import functools
import json
import os
import subprocess
import sys

import pytest

from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import spawn

import tp_workers as TW  # noqa: E402  (tests/ is on sys.path via conftest)

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(fn, tmp_path, n=2, **kw):
    spawn(functools.partial(fn, **kw) if kw else fn, n, args=(str(tmp_path),), grace=5.0)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_tensor_parallel_captured_with_real_peers(tmp_path, world):
    run(TW.captured_parity, tmp_path, n=world)


@pytest.mark.parametrize("world,chunks", [(2, 4), (4, 2), (8, 2)])
def test_tensor_parallel_overlap_captured_with_real_peers(tmp_path, world, chunks):
    run(TW.captured_parity, tmp_path, n=world, chunks=chunks)


def test_tensor_parallel_syncbn_captured_with_real_peers(tmp_path):
    run(TW.captured_parity, tmp_path, n=2, bn=True)


@pytest.mark.parametrize("world,chunks,bn", [(1, 1, False), (2, 1, False), (4, 2, False),
                                             (2, 1, True), (8, 2, False)])
def test_tensor_parallel_fused_optimizer_captured(tmp_path, world, chunks, bn):
    """register_fused_optimizer: SGD of the shards inside their weight-gradient GEMM
    epilogues, the rest (replicated head, BatchNorm shards) in optimizer.step(): captured ==
    eager bitwise, both == the one-process global-batch step of the full model."""
    run(TW.captured_parity, tmp_path, n=world, chunks=chunks, bn=bn, fused=True,
        backend="nccl" if world == 1 else "peer")


@pytest.mark.parametrize("world", [2, 4])
def test_tensor_parallel_gradient_accumulation(tmp_path, world):
    """Two micro-batches per step (fused + no_sync, unfused, unfused + no_sync) == the torch
    step of the full model on the summed global-batch gradients."""
    run(TW.accumulation_parity, tmp_path, n=world)


def test_tensor_parallel_accumulation_waits_for_a_late_aux_stream(tmp_path):
    """with the aux stream held back by a long kernel, the second
    micro-batch's accumulation into fc2's weight gradient still sees the first pass's value."""
    run(TW.accumulation_parity, tmp_path, n=2, delay_aux=True)


def _peer_bench(*args, diag=False):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    env.update(TDP_GPU_PEER="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4",
           "--warmup", "2", "--mlp-dims", "1024,512,512", "--dataset", "1024", "--batch", "32",
           "--device-warmup-ms", "0", *([] if diag else ["--no-diag"]), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])


def test_bench_tensor_sharded_step_captured():
    c = _peer_bench("--parallel", "tensor")["config"]
    assert c["rung"].startswith("tensor-") and c["fallbacks"] == [], c
    assert c["parallelism"] == "tp2", c
    assert c["sync"]["captured"] is True and c["sync"]["replicas_identical"] is True, c["sync"]


def test_bench_parallel_auto_records_selection():
    c = _peer_bench("--select-steps", "4", "--parallel", "auto")["config"]
    sel = c["selection"]
    # auto: tensor timings are side numbers, the DDP rung is measured
    assert sel is not None and sel["chosen"] == c["rung"] == "full", c
    assert c["parallelism"] == "dp2" and "tensor-sharded_ms" in sel, c
    assert c["sync"]["captured"] is True and c["sync"]["replicas_identical"] is True, c["sync"]


def test_bench_default_is_ddp_on_the_peer_vehicle():
    """``TDP_GPU_PEER=1 python bench.py --gpus 2`` with no --parallel flag
    measures the DDP ladder's full rung and says dp2."""
    c = _peer_bench()["config"]
    assert c["parallelism"] == "dp2" and c["rung"] == "full" and c["selection"] is None, c
    assert c["sync"]["captured"] is True and c["sync"]["replicas_identical"] is True, c["sync"]


def test_bench_tensor_sharded_diagnostics():
    """N > 1 diagnostics of the tensor-sharded step: compute with local-copy collectives, the
    exposed remainder, the busbw sweep and the model's prediction from it."""
    rec = _peer_bench("--parallel", "tensor", diag=True)
    d = rec["diagnostics"]
    assert "error" not in d, d
    assert d["execution"] == rec["config"]["rung"] and d["compute_ms"] > 0, d
    assert d["predicted_step_ms"] > 0 and d["busbw_GBps"], d


def test_bias_act_and_scaled_relu_bias_bwd():
    """csrc bias_act (y = relu?(x + b)) and relu_bias_bwd's gscale (g scaled, db not) against
    torch."""
    import torch

    from tutorial_torch_distributed_data_parallel_amd._native import native

    C = native()
    torch.manual_seed(4)
    x = torch.randn(128, 512, device="cuda")
    b = torch.randn(512, device="cuda")
    for relu in (True, False):
        ref = x + b
        ref = torch.relu(ref) if relu else ref
        assert torch.equal(C.bias_act(x, b, relu), ref)
    y = torch.relu(x + b)
    dy = torch.randn_like(y)
    db = torch.empty(512, device="cuda")
    g = C.relu_bias_bwd(dy, y, db, gscale=0.125)
    m = dy * (y > 0)
    assert torch.equal(g, m * 0.125)
    torch.testing.assert_close(db, m.sum(0), rtol=1e-5, atol=1e-4)
