"""The production gradient-sync algorithm (csrc/reducer.cpp SyncBackend) multi-rank on CPU/gloo:
sharded update with uneven tails, in-reduction / per-rank clipping, LR changes, Adam step count,
state consolidation and resume -- against stock torch DDP + torch.optim (tests/sync_workers.py)."""
import functools

import pytest

from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import spawn

import sync_workers as SW  # noqa: E402  (tests/ is on sys.path via conftest)


def run(fn, tmp_path, n=2, **kw):
    spawn(functools.partial(fn, **kw) if kw else fn, n, args=(str(tmp_path),), grace=5.0)


@pytest.fixture(autouse=True)
def _poison(monkeypatch):
    # slices a rank does not own after a reduce-scatter become NaN: any read of them fails a test
    monkeypatch.setenv("TDP_POISON_UNOWNED", "1")


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind", ["sgd", "adam"])
def test_sharded_fused_optimizer_matches_torch_ddp(tmp_path, world, kind):
    run(SW.fused_parity, tmp_path, n=world, kind=kind, shard=True)


@pytest.mark.parametrize("kind", ["adamw", "amsgrad"])
def test_sharded_fused_adam_variants(tmp_path, kind):
    run(SW.fused_parity, tmp_path, n=3, kind=kind, shard=True, steps=4)


def test_replicated_fused_optimizer_matches_torch_ddp(tmp_path):
    run(SW.fused_parity, tmp_path, n=2, kind="adam", shard=False)


@pytest.mark.parametrize("world,shard", [(2, True), (3, False)])
def test_fused_global_clip_matches_clip_grad_norm(tmp_path, world, shard):
    run(SW.fused_parity, tmp_path, n=world, kind="sgd", shard=shard, clip=0.05)


@pytest.mark.parametrize("fused", [True, False])
def test_clip_before_aggregation(tmp_path, fused):
    run(SW.local_clip_parity, tmp_path, n=2, fused=fused)


def test_comm_hook_keeps_fused_state(tmp_path):
    run(SW.comm_hook_keeps_fused_state, tmp_path, n=2)


def test_shared_parameter_gradient(tmp_path):
    run(SW.shared_parameter, tmp_path, n=2)


def test_ddp_logger_runtime_stats(tmp_path):
    run(SW.logger_stats, tmp_path, n=2)


@pytest.mark.parametrize("fused", [True, False])
def test_bucket_rebuild_from_ready_order(tmp_path, fused):
    run(SW.bucket_rebuild, tmp_path, n=2, fused=fused)


@pytest.mark.parametrize("world,kind,replicate", [
    (2, "sgd", True), (2, "adam", False), (3, "sgd", False), (3, "adam", True),
    (4, "sgd", False), (4, "adam", True), (3, "sgd", "mixed")])
def test_factored_sync_matches_torch_ddp(tmp_path, world, kind, replicate):
    run(SW.factored_parity, tmp_path, n=world, kind=kind, replicate=replicate)


@pytest.mark.parametrize("world", [2, 3])
def test_factored_mode_tuning(tmp_path, world):
    run(SW.factored_tuning, tmp_path, n=world)


def test_factored_sync_refuses_foreign_gradient(tmp_path):
    run(SW.factored_foreign_gradient, tmp_path, n=2)


def test_capture_failure_on_one_rank_makes_all_eager(tmp_path):
    run(SW.capture_agreement, tmp_path, n=2)


@pytest.mark.parametrize("fused", [False, True])
def test_gradient_accumulation_skips_communication(tmp_path, fused):
    run(SW.accumulation_parity, tmp_path, n=2, fused=fused)


@pytest.mark.parametrize("kind", ["sgd", "adam"])
def test_rebuild_moves_sharded_optimizer_state(tmp_path, kind):
    run(SW.rebuild_moves_shards, tmp_path, n=2, kind=kind)


def test_factored_batch_over_slot_fails_fast(tmp_path):
    from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import (
        ProcessRaisedException)

    with pytest.raises(ProcessRaisedException, match="factor_capacity"):
        run(SW.factored_batch_over_slot, tmp_path, n=2)


def test_factored_capacity_agreed_up_front(tmp_path):
    run(SW.factored_batch_over_slot, tmp_path, n=2, agree_first=True)
