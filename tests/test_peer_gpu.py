"""MI355X: W ranks on ONE GPU through the peer-memory vehicle (csrc/peer.hip): collectives as
device kernels, the captured multi-rank DDP step replayed with real peers,
bounded device-side waits, and the RCCL watchdog firing on a stalled collective (item 7)."""
import functools
import json
import os
import subprocess
import sys

import pytest

from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import (
    ProcessExitedException, spawn)

import peer_workers as PW  # noqa: E402  (tests/ is on sys.path via conftest)
import relay_workers as RW  # noqa: E402
from test_relay_gpu import _check_tuning_applied  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(fn, tmp_path, n=2, **kw):
    spawn(functools.partial(fn, **kw) if kw else fn, n, args=(str(tmp_path),), grace=5.0)


@pytest.mark.parametrize("n", [2, 3])
def test_peer_collectives_chunked_and_captured(tmp_path, n):
    run(PW.chunked_collectives, tmp_path, n=n)


def test_peer_relay_semantics(tmp_path):
    """The relay's collective checks, unchanged, on the peer vehicle."""
    run(RW.collectives, tmp_path, n=3, backend="peer")


@pytest.mark.parametrize("world,kind,factor,replicate", [
    (2, "sgd", True, None), (2, "adam", True, False), (3, "sgd", True, False),
    (3, "adam", True, True), (2, "sgd", False, None), (3, "adam", False, None),
    (2, "sgd", True, 0.5), (3, "adam", True, 0.5)])
def test_captured_step_with_real_peers(tmp_path, world, kind, factor, replicate):
    run(PW.captured_ddp_parity, tmp_path, n=world, kind=kind, factor=factor, replicate=replicate)


@pytest.mark.parametrize("world,kind,replicate", [(2, "adam", False), (4, "sgd", True),
                                                  (4, "adam", 0.5)])
def test_peer_eager_device_path_matches_oracle(tmp_path, world, kind, replicate):
    run(RW.ddp_parity, tmp_path, n=world, kind=kind, factor=True, replicate=replicate,
        backend="peer")


def test_peer_syncbn_matches_global_batch(tmp_path):
    run(RW.syncbn_parity, tmp_path, n=2, backend="peer")


def test_stalled_peer_exits_86(tmp_path):
    with pytest.raises(ProcessExitedException) as ei:
        run(PW.stalled_peer_times_out, tmp_path, n=2)
    assert ei.value.exit_code == 86


def test_rccl_watchdog_fires_on_stalled_collective():
    """the collective watchdog (TORCH/distributed/constants.py:21 in the
    reference's stack) aborts a stuck RCCL collective and ends the rank with exit code 86;
    the parent process is unaffected."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "peer_workers.py")],
                       capture_output=True, text=True, timeout=120, cwd=ROOT,
                       env=dict(os.environ, PYTHONPATH=os.path.join(ROOT, "tests") + os.pathsep +
                                ROOT))
    assert r.returncode == 86, (r.returncode, r.stderr[-2000:])
    assert "RCCL watchdog" in r.stderr and "stalled collective" in r.stderr, r.stderr[-2000:]


def test_capture_beside_pending_watch():
    """The communicator's watchdog thread polls a pending watch while the main thread records a
    hipGraph: the capture succeeds (the thread runs in relaxed capture mode; before, its event
    queries invalidated a concurrent capture -- a one-rank capture failure in bench's tuning)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "peer_workers.py"),
                        "capture_beside_pending_watch"], capture_output=True, text=True,
                       timeout=120, cwd=ROOT,
                       env=dict(os.environ, PYTHONPATH=os.path.join(ROOT, "tests") + os.pathsep +
                                ROOT))
    assert r.returncode == 0 and "capture-ok" in r.stdout, (r.returncode, r.stderr[-2000:])


def test_bench_self_launch_peer_captured():
    """``TDP_GPU_PEER=1 python bench.py --gpus 2``: bench.py spawns its two ranks itself, the
    multi-rank step is CAPTURED with real peers, replicas end bit-identical."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    env.update(TDP_GPU_PEER="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5",
           "--warmup", "3", "--mlp-dims", "1024,512,512", "--dataset", "1024", "--batch", "32",
           "--no-diag", "--device-warmup-ms", "0", "--parallel", "ddp"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    from bench import LADDER
    assert rec["config"]["rung"] in [c["name"] for c in LADDER], rec["config"]["rung"]
    assert rec["config"]["launched_by"].startswith("bench.py (self-launched 2 ranks")
    assert rec["config"]["comm_nranks"] == 2
    sync = rec["config"]["sync"]
    assert sync["backend"] == "peer" and sync["captured"] is True, sync
    assert sync["replicas_identical"] is True, sync
    assert sync["modes"]["fc1.weight"].startswith("factored"), sync
    tun = sync["factor_tuning"]
    assert tun["captured"] is True and set(tun["chosen"]) == {"fc1.weight", "fc2.weight"}, tun
    _check_tuning_applied(sync)


def _peer_bench(extra_env, *args):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    env.update(TDP_GPU_PEER="1", **extra_env)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4",
           "--warmup", "2", "--mlp-dims", "1024,512,512", "--dataset", "1024", "--batch", "32",
           "--no-diag", "--device-warmup-ms", "0", "--parallel", "ddp", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert rec["n_gpus"] == 2 and rec["value"] > 0
    if rec["config"]["parallelism"] == "dp2":  # a dp{N} record is always a DDP ladder rung
        from bench import LADDER
        assert rec["config"]["rung"] in [c["name"] for c in LADDER], rec["config"]
    return rec


def test_bench_ladder_tuning_failure_keeps_model_choice():
    """VERDICT r4 next 2b, rung 'tuning': the factored-mode tuning raises on every rank; the
    bench keeps the model's choice, still captures, and records the fallback."""
    rec = _peer_bench({"TDP_BENCH_FAULT": "tune"})
    c = rec["config"]
    assert c["rung"] == "full" and any("tuning failed" in f for f in c["fallbacks"]), c
    assert c["sync"]["captured"] is True and c["sync"]["replicas_identical"] is True, c["sync"]
    assert c["sync"]["factor_tuning"] is None
    assert c["sync"]["modes"]["fc1.weight"].startswith("factored"), c["sync"]


def test_bench_ladder_factored_failure_falls_back_to_sharded_buckets():
    """Rung 'factored': setup with factored weights raises on every rank; the next rung runs
    plain sharded buckets (reduce-scatter -> 1/W update -> all-gather), captured."""
    rec = _peer_bench({"TDP_BENCH_FAULT": "factored"})
    c = rec["config"]
    assert c["rung"] == "sharded-buckets" and len(c["fallbacks"]) == 1, c
    assert c["sync"]["captured"] is True and c["sync"]["replicas_identical"] is True, c["sync"]
    assert not any(m.startswith("factored") for m in c["sync"]["modes"].values()), c["sync"]


def test_bench_ladder_capture_failure_on_one_rank_runs_eagerly():
    """Rung 'capture': rank 1's capture fails; every rank runs the step eagerly (agreed)."""
    rec = _peer_bench({"TDP_FAULT_CAPTURE": "1"})
    c = rec["config"]
    assert c["sync"]["captured"] is False and c["sync"]["replicas_identical"] is True, c["sync"]
    assert any("capture failed" in f for f in c["fallbacks"]), c


@pytest.mark.parametrize("sync1d", [False, True])
@pytest.mark.parametrize("world", [2, 3])
def test_captured_syncbn_with_real_peers(tmp_path, world, sync1d):
    run(PW.captured_syncbn_parity, tmp_path, n=world, sync1d=sync1d)


@pytest.mark.parametrize("world", [2, 3])
def test_captured_accelerate_with_real_peers(tmp_path, world):
    run(PW.captured_accelerate_parity, tmp_path, n=world)


@pytest.mark.parametrize("world", [2, 3])
def test_captured_cnn_with_real_peers(tmp_path, world):
    run(PW.captured_cnn_parity, tmp_path, n=world)
