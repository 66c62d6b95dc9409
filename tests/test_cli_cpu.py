"""Entry points end to end on CPU/gloo: YAML handling, spawn, checkpoints, HTCondor writer."""
import os
import subprocess
import sys

import torch
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _settings(tmp_path, **train):
    s = {"script_path": os.path.join(ROOT, "scripts", "train_ddp.py"),
         "out_dir": str(tmp_path / "out"),
         "optional_args": {"set_epoch": True, "print_rand": True},
         "local": {"device": "cuda", "condor": {"bid": 50, "num_cpus": 2, "memory_cpus": 1000,
                                                "num_gpus": 2, "memory_gpus": 60000}},
         "train": dict(model="toy_mlp", n_train=64, n_test=20, train_batch_size=8,
                       test_batch_size=10, num_epochs=2, checkpoint_epoch=1, lr=1e-3,
                       max_steps_per_epoch=2, **train)}
    p = tmp_path / "local_settings.yaml"
    p.write_text(yaml.safe_dump(s))
    return p, s


def _run(args, env_extra=None, timeout=300):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.update(env_extra or {})
    env = {k: v for k, v in env.items() if v is not None}  # None: drop the variable
    return subprocess.run([sys.executable, *args], capture_output=True, text=True, env=env,
                          timeout=timeout, cwd=ROOT)


def test_train_ddp_two_ranks(tmp_path):
    p, s = _settings(tmp_path)
    r = _run([os.path.join(ROOT, "scripts", "train_ddp.py"), "--settings_file", str(p)])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = s["out_dir"]
    assert os.path.exists(os.path.join(out, "local_settings.yaml"))  # YAML copied (R10)
    assert os.path.exists(os.path.join(out, "ckpt_0.pt")) and os.path.exists(
        os.path.join(out, "ckpt_1.pt"))
    sd = torch.load(os.path.join(out, "ckpt_1.pt"), map_location="cpu", weights_only=True)
    assert all(k.startswith("module.") for k in sd)
    assert "Epoch 2/2, Train Loss:" in r.stdout
    assert r.stdout.count("Epoch 2/2, Train Loss:") == 1  # rank 0 only
    assert "Python random state" in r.stdout  # print_rand


def test_train_accelerate_single_process(tmp_path):
    p, s = _settings(tmp_path)
    r = _run([os.path.join(ROOT, "scripts", "train_accelerate.py"), "--settings_file", str(p)])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert os.path.exists(os.path.join(s["out_dir"], "model.safetensors"))
    assert "Finished Training." in r.stdout


def test_launch_writes_condor_file(tmp_path):
    p, s = _settings(tmp_path)
    r = _run([os.path.join(ROOT, "scripts", "launch.py"), "--settings_file", str(p),
              "--write-condor"])
    assert r.returncode == 0, r.stderr
    sub = open(os.path.join(s["out_dir"], "submission_file.sub")).read()
    assert "request_gpus = 2" in sub and "TARGET.CUDAGlobalMemoryMb > 60000" in sub
    assert sub.strip().endswith("queue")


import json  # noqa: E402

import pytest  # noqa: E402


@pytest.mark.parametrize("api", ["ddp", "accelerate"])
def test_bench_two_ranks_one_json_line(api):
    """bench.py under the launcher on 2 gloo ranks: exactly one JSON line on stdout (RCCL/native
    banners go to stderr), whole-job throughput, dp2."""
    r = _run(["-m", "tutorial_torch_distributed_data_parallel_amd.parallel.launcher", "--nproc",
              "2", "bench.py", "--cpu", "--gpus", "2", "--steps", "3", "--warmup", "1",
              "--dataset", "256", "--batch", "16", "--mlp-dims", "64,32,32", "--api", api])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 32
    assert rec["value"] > 0 and rec["steps"] == 3 and rec["warmup"] == 1
    assert ("Accelerator.prepare" in rec["config"]["impl"]) == (api == "accelerate")


def test_bench_self_launches_n_ranks():
    """``python bench.py --gpus 3`` with no launcher environment spawns its own 3 ranks (no
    torchrun), relays rank 0's single JSON line, and reports dp3 / 3x the per-rank batch."""
    env = {k: None for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    r = _run(["bench.py", "--cpu", "--gpus", "3", "--steps", "2", "--warmup", "1",
              "--dataset", "192", "--batch", "16", "--mlp-dims", "64,32,32"],
             env_extra=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["config"]["parallelism"] == "dp3" and rec["config"]["global_batch"] == 48
    assert rec["config"]["launched_by"].startswith("bench.py (self-launched 3 ranks")
    assert rec["steps"] == 2 and rec["warmup"] == 1


def test_bench_refuses_more_gpus_than_visible():
    """Without a one-GPU vehicle, --gpus N on a box with fewer GPUs exits non-zero instead of
    reporting a one-rank number as an N-GPU one."""
    env = {k: None for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "TDP_GPU_RELAY", "TDP_GPU_PEER")}
    r = _run(["bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0"], env_extra=env,
             timeout=120)
    assert r.returncode == 2, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.strip() == ""
    assert "only 0 GPU(s) are visible" in r.stderr


def test_train_ddp_host_pipeline_two_ranks(tmp_path):
    """train.data: cifar_uint8 -- CIFAR-layout uint8 host images through the native prefetcher
    and the Resize / Flip / Normalize transform into AlexNet, 2 gloo ranks."""
    p, s = _settings(tmp_path)
    s["train"].update(model="alexnet", data="cifar_uint8", image_size=64, n_train=32,
                      n_test=16, train_batch_size=4, test_batch_size=4, num_epochs=1,
                      max_steps_per_epoch=2)
    p.write_text(yaml.safe_dump(s))
    r = _run([os.path.join(ROOT, "scripts", "train_ddp.py"), "--settings_file", str(p)])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "Epoch 1/1, Train Loss:" in r.stdout


def test_launcher_hosts_the_rendezvous_store():
    """The launcher binds the rendezvous store itself (OS-picked port, held for the job): no
    window between probing a free port and rank 0 binding it; ranks connect as clients."""
    import socket

    from tutorial_torch_distributed_data_parallel_amd.parallel.launcher import _launcher_store

    store, port, env = _launcher_store("127.0.0.1", 2)
    assert store is not None and port > 0
    assert env == {"TORCHELASTIC_USE_AGENT_STORE": "True"}
    with socket.socket() as s, pytest.raises(OSError):
        s.bind(("127.0.0.1", port))  # held by the store for the job's lifetime
    store.set("k", "v")
    assert store.get("k") == b"v"
    one, _, env1 = _launcher_store("127.0.0.1", 1)
    assert one is None and env1 == {}


def _bench_cpu2(env_extra, *args):
    env = {k: None for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    env.update(env_extra)
    return _run(["bench.py", "--cpu", "--gpus", "2", "--steps", "2", "--warmup", "1",
                 "--dataset", "128", "--batch", "16", "--mlp-dims", "64,32,32", *args],
                env_extra=env)


def test_bench_fallback_ladder_records_the_rung():
    """a failure in a rung (here: the first warm-up step, on every rank)
    moves every rank to the next rung, and the record says which rung ran and why."""
    r = _bench_cpu2({"TDP_BENCH_FAULT": "warmup"}, "--parallel", "ddp")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert rec["config"]["rung"] == "sharded-buckets", rec["config"]
    assert len(rec["config"]["fallbacks"]) == 1 and "full failed" in rec["config"]["fallbacks"][0]
    assert rec["value"] > 0 and rec["steps"] == 2


def test_bench_fallback_ladder_exhausted_exits_nonzero():
    r = _bench_cpu2({"TDP_BENCH_FAULT": "warmup@*"}, "--parallel", "ddp")
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "every rung of the fallback ladder failed" in r.stderr


def test_bench_clean_run_reports_no_fallback():
    r = _bench_cpu2({}, "--parallel", "ddp")
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert rec["config"]["rung"] == "full" and rec["config"]["fallbacks"] == []


LADDER_NAMES = ("full", "sharded-buckets", "allreduce+optimizer.step", "eager-allreduce")


def test_bench_default_is_the_ddp_headline():
    """with no --parallel flag the N > 1 record is the DDP reducer's step,
    labelled dp{N}, and no tensor-sharded candidate is built or timed."""
    r = _bench_cpu2({})
    assert r.returncode == 0, r.stderr[-3000:]
    c = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])["config"]
    assert c["parallelism"] == "dp2" and c["rung"] in LADDER_NAMES, c
    assert c["selection"] is None and c["bucket_mb"], c
    assert "tensor" not in c["impl"], c


def test_bench_parallel_auto_keeps_the_ddp_headline():
    """--parallel auto at N > 1: the tensor-sharded variants are timed as SIDE numbers; the
    measured value is always the DDP rung's, recorded as dp{N}."""
    r = _bench_cpu2({}, "--select-steps", "2", "--parallel", "auto")
    assert r.returncode == 0, r.stderr[-3000:]
    c = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])["config"]
    sel = c["selection"]
    assert set(sel) == {"tensor-sharded_ms", "tensor-overlap_ms", "full_ms", "chosen"}, sel
    assert sel["chosen"] == "full" == c["rung"] and c["parallelism"] == "dp2", c
    assert c["selection_ms"] == sel["full_ms"], c
    assert c["sync"]["replicas_identical"] is True, c["sync"]


def test_bench_parallel_tensor_is_labelled_tp():
    r = _bench_cpu2({}, "--parallel", "tensor")
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    c = rec["config"]
    assert c["rung"] in ("tensor-sharded", "tensor-overlap"), c
    assert c["selection"]["chosen"] == c["rung"] and c["selection_ms"] > 0, c
    assert c["parallelism"] == "tp2" and "tensor-sharded" in c["impl"], c
    assert "DDP" not in rec["metric"].replace("not DDP", ""), rec["metric"]
    assert c["sync"]["modes"]["fc1"] == "column-sharded" and c["bucket_mb"] is None
    assert c["sync"]["replicas_identical"] is True


def test_bench_parallel_tensor_ignores_the_ladder():
    """--parallel tensor never builds the DDP ladder: a ladder-wide fault does not touch it."""
    r = _bench_cpu2({"TDP_BENCH_FAULT": "warmup@*"}, "--parallel", "tensor")
    assert r.returncode == 0, r.stderr[-3000:]
    c = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])["config"]
    assert c["rung"].startswith("tensor-") and c["fallbacks"] == [], c


def test_bench_parallel_auto_needs_a_ddp_rung():
    """auto never falls back to the tensor-sharded step for its headline."""
    r = _bench_cpu2({"TDP_BENCH_FAULT": "warmup@*"}, "--parallel", "auto", "--select-steps", "1")
    assert r.returncode != 0 and r.stdout.strip() == ""
    assert "every rung of the fallback ladder failed" in r.stderr
