"""Tensor-sharded toy-MLP training step (parallel/tensor_parallel.py) on CPU/gloo against the
one-process global-batch step of the full model (tests/tp_workers.py)."""
import functools

import pytest

from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import spawn

import tp_workers as TW  # noqa: E402  (tests/ is on sys.path via conftest)


def run(fn, tmp_path, n=2, **kw):
    spawn(functools.partial(fn, **kw) if kw else fn, n, args=(str(tmp_path),), grace=5.0)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_tensor_parallel_step_matches_global_batch(tmp_path, world):
    run(TW.step_parity, tmp_path, n=world)


@pytest.mark.parametrize("world", [2, 4])
def test_tensor_parallel_syncbn_matches_global_batch(tmp_path, world):
    run(TW.step_parity, tmp_path, n=world, bn=True)


def test_tensor_parallel_global_batch_input(tmp_path):
    run(TW.step_parity, tmp_path, n=2, global_batch=True)


def test_tensor_parallel_refuses_per_rank_bn(tmp_path):
    run(TW.refuses_plain_bn, tmp_path, n=2)


@pytest.mark.parametrize("world,chunks", [(2, 4), (4, 2)])
def test_tensor_parallel_overlapped_chunks_match_global_batch(tmp_path, world, chunks):
    run(TW.step_parity, tmp_path, n=world, chunks=chunks)


def test_tensor_parallel_adam_matches_global_batch(tmp_path):
    run(TW.step_parity, tmp_path, n=2, kind="adam")


def test_tensor_parallel_checkpoint_is_the_full_models(tmp_path):
    run(TW.checkpoint_roundtrip, tmp_path, n=2)


@pytest.mark.parametrize("world", [2, 4])
def test_tensor_parallel_gradient_accumulation_cpu(tmp_path, world):
    """Two micro-batches per step through the wrapper (with and without no_sync; the fused
    optimizer is GPU-only and refuses here) == the torch step on the summed global-batch
    gradients."""
    run(TW.accumulation_parity, tmp_path, n=world, backend="gloo", device="cpu")


@pytest.mark.parametrize("kind,bn", [("sgd", False), ("adam", False), ("sgd", True)])
def test_tensor_parallel_resume_is_bitwise(tmp_path, kind, bn):
    """3 steps, save, resume into a fresh job, 2 steps == 5 uninterrupted steps (gloo, W=2)."""
    run(TW.resume_parity, tmp_path, n=2, kind=kind, bn=bn)
