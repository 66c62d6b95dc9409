"""Multi-process DDP behaviour on CPU/gloo (world_size 2) through our own launcher."""
import os

import pytest
import torch

from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import (
    ProcessRaisedException, spawn)

import ddp_workers as W  # noqa: E402  (tests/ is on sys.path via conftest)


def run(fn, tmp_path, n=2):
    spawn(fn, n, args=(str(tmp_path),), grace=5.0)


def test_ddp_oracles(tmp_path):
    run(W.ddp_oracles, tmp_path)


def test_syncbn_matches_full_batch_bn(tmp_path):
    run(W.syncbn_parity, tmp_path)


def test_training_loop_metrics_and_checkpoints(tmp_path):
    run(W.training_loop, tmp_path)
    files = sorted(os.listdir(tmp_path))
    assert "ckpt_0.pt" in files and "ckpt_5.pt" in files
    sd = torch.load(tmp_path / "ckpt_5.pt", map_location="cpu", weights_only=True)
    assert all(k.startswith("module.") for k in sd)
    lines = (tmp_path / "log.jsonl").read_text().strip().splitlines()
    assert len(lines) == 6


def test_fail_fast_fault_injection(tmp_path, monkeypatch):
    monkeypatch.setenv("TDP_FAULT", "1:3")
    with pytest.raises(ProcessRaisedException) as ei:
        run(W.fault_worker, tmp_path)
    assert "injected fault on rank 1 at step 3" in str(ei.value)


def test_find_unused_parameters(tmp_path):
    run(W.unused_params, tmp_path)


def test_accelerate_facade_two_ranks(tmp_path):
    run(W.accelerate_worker, tmp_path)


def test_replica_consistency_check(tmp_path):
    run(W.replica_check, tmp_path)


def test_stalled_peer_times_out(tmp_path, monkeypatch):
    """a rank that hangs (alive, never reaching the next collective) is detected
    by the surviving rank's collective timeout (TDP_TIMEOUT_S; on MI355X the RCCL watchdog of
    csrc/comm.h aborts the communicator and exits 86), which fails the job instead of hanging."""
    import time

    monkeypatch.setenv("TDP_FAULT", "1:3:stall")
    monkeypatch.setenv("TDP_TIMEOUT_S", "4")
    t0 = time.perf_counter()
    with pytest.raises(ProcessRaisedException) as ei:
        run(W.fault_worker, tmp_path)
    elapsed = time.perf_counter() - t0
    assert elapsed < 60, elapsed
    msg = str(ei.value)
    assert "Process 0" in msg and "Timed out" in msg, msg
