"""MI355X, two or more GPUs: the multi-rank paths on RCCL with one rank per GPU (VERDICT r4
missing 1 / next 2a). Every multi-rank GPU test elsewhere runs several ranks on ONE GPU through
the relay / peer vehicles; this tier runs the same bodies -- DDP parity against the fp32 torch
oracle eager and CAPTURED (RCCL inside hipGraph capture), factored replicated / sharded / split
modes, the bucket path, SyncBN, the Accelerate facade, a CNN, check_replicas -- with
backend="nccl" at W = 2 and W = min(8, GPUs). It skips on a one-GPU box (counting devices does
not initialise HIP in the test process)."""
import functools
import json
import os
import subprocess
import sys

import pytest
import torch

from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import spawn

import peer_workers as PW  # noqa: E402  (tests/ is on sys.path via conftest)
import relay_workers as RW  # noqa: E402
import tp_workers as TW  # noqa: E402

NGPU = torch.cuda.device_count()
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(NGPU < 2, reason=f"needs >= 2 GPUs (found {NGPU})")]
WORLDS = sorted({2, min(8, max(NGPU, 2))})
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(fn, tmp_path, n, **kw):
    # the vehicles' environment must not leak into a real multi-GPU job
    for k in ("TDP_GPU_PEER", "TDP_GPU_RELAY"):
        os.environ.pop(k, None)
    spawn(functools.partial(fn, **kw), n, args=(str(tmp_path),), grace=10.0)


@pytest.mark.parametrize("world", WORLDS)
def test_rccl_collectives(tmp_path, world):
    run(RW.collectives, tmp_path, world, backend="nccl")


@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("kind,factor,replicate,fused", [
    ("sgd", True, None, True), ("adam", True, False, True), ("sgd", True, True, True),
    ("adam", True, 0.5, True), ("sgd", False, None, True), ("sgd", False, None, False)])
def test_rccl_eager_ddp_matches_oracle(tmp_path, world, kind, factor, replicate, fused):
    run(RW.ddp_parity, tmp_path, world, kind=kind, factor=factor, replicate=replicate,
        fused=fused, backend="nccl")


@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("kind,factor,replicate", [
    ("sgd", True, None), ("adam", True, False), ("sgd", True, 0.5), ("adam", False, None)])
def test_rccl_captured_ddp_matches_eager_and_oracle(tmp_path, world, kind, factor, replicate):
    run(PW.captured_ddp_parity, tmp_path, world, kind=kind, factor=factor, replicate=replicate,
        backend="nccl")


@pytest.mark.parametrize("world", WORLDS)
def test_rccl_syncbn(tmp_path, world):
    run(RW.syncbn_parity, tmp_path, world, backend="nccl")
    run(PW.captured_syncbn_parity, tmp_path, world, backend="nccl")


@pytest.mark.parametrize("world", WORLDS)
def test_rccl_accelerate_captured(tmp_path, world):
    run(PW.captured_accelerate_parity, tmp_path, world, backend="nccl")


@pytest.mark.parametrize("world", WORLDS)
def test_rccl_cnn_captured(tmp_path, world):
    run(PW.captured_cnn_parity, tmp_path, world, backend="nccl")


@pytest.mark.parametrize("world", WORLDS)
@pytest.mark.parametrize("bn,chunks,fused", [(False, 1, False), (False, 2, False),
                                              (True, 1, False), (False, 2, True),
                                              (True, 1, True)])
def test_rccl_tensor_parallel_captured(tmp_path, world, bn, chunks, fused):
    """The tensor-sharded step (parallel/tensor_parallel.py) on RCCL: reduce-scatter / all-gather
    of activations over xGMI inside hipGraph capture, captured == eager bitwise, both == the
    one-process global-batch step to fp32 accuracy."""
    run(TW.captured_parity, tmp_path, world, backend="nccl", bn=bn, chunks=chunks, fused=fused)


@pytest.mark.parametrize("world", WORLDS)
def test_rccl_bench_tensor_record(world):
    """``python bench.py --gpus N --parallel tensor`` on N real GPUs: a tensor-sharded rung,
    captured, replicas identical, RCCL saw N ranks."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "TDP_GPU_PEER", "TDP_GPU_RELAY")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "6",
           "--warmup", "3", "--mlp-dims", "1024,512,512", "--dataset", "2048", "--batch", "32",
           "--device-warmup-ms", "0", "--parallel", "tensor"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    c = rec["config"]
    assert rec["n_gpus"] == world and c["comm_nranks"] == world, c
    assert c["parallelism"] == f"tp{world}", c
    assert c["rung"].startswith("tensor-") and c["fallbacks"] == [], c
    assert c["sync"]["captured"] is True and c["sync"]["replicas_identical"] is True, c["sync"]


@pytest.mark.parametrize("world", WORLDS)
def test_rccl_bench_record(world):
    """``python bench.py --gpus N`` on N real GPUs: one valid record, captured, replicas
    bit-identical, RCCL saw N ranks, no fallback taken; the default execution is the DDP
    reducer's ladder (labelled dp{N}), never the tensor-sharded step."""
    from bench import LADDER

    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "TDP_GPU_PEER", "TDP_GPU_RELAY")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "6",
           "--warmup", "3", "--mlp-dims", "1024,512,512", "--dataset", "2048", "--batch", "32",
           "--device-warmup-ms", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    c = rec["config"]
    assert rec["n_gpus"] == world and c["parallelism"] == f"dp{world}"
    assert c["rung"] in [r["name"] for r in LADDER] and c["bucket_mb"], c
    assert c["comm_nranks"] == world and c["sync"]["backend"] == "rccl"
    assert c["sync"]["captured"] is True and c["sync"]["replicas_identical"] is True, c["sync"]
    assert c["fallbacks"] == [], c["fallbacks"]
