"""Entry points with the reference's CLI and YAML contract.

* ``train_ddp``  -- REF/multi-GPU-training-torch.py: ``--settings_file``;
  YAML copied into out_dir; world size from ``local.condor.num_gpus``; ``optional_args``
  {set_epoch, print_rand}; one process per GPU (our launcher, or torchrun-style env); per rank:
  init -> per-rank seeds -> DistributedSampler loaders -> model -> DDP -> CE + Adam(1e-3) ->
  run_training_loop (rank-0 ``ckpt_{epoch}.pt``) -> cleanup.
* ``train_accelerate`` -- REF/multi-GPU-training-accelerate.py (§3.4, R11-R16): plain loaders
  (no sampler, no shuffle), ``Accelerator.prepare(model, optimizer, train_loader)``,
  ``accelerator.backward``, full-test-set evaluation on every rank, local-main-process prints,
  ``wait_for_everyone`` + ``save_model`` -> ``model.safetensors`` every 5 epochs.
* ``launch`` -- replaces REF/submit_job.py (§3.5, R19/R20): spawns ``num_gpus`` ranks of
  ``script_path`` on this node; ``--write-condor`` still emits the HTCondor submission file with the
  reference's keys for users who schedule through a cluster.
Data is synthetic (no network): CIFAR-10-shaped tensors resident on the device, or (train.data:
cifar_uint8) CIFAR-layout uint8 host images through the native input pipeline (data/host.py).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch


def _settings(argv, desc):
    from .utils.config import copy_settings_to_out_dir, load_settings

    ap = argparse.ArgumentParser(description=desc)
    ap.add_argument("--settings_file", type=str, required=True,
                    help="Path to local_settings.yaml file specifying cluster settings and "
                         "other parameters.")
    a = ap.parse_args(argv)
    s = load_settings(a.settings_file)
    copy_settings_to_out_dir(a.settings_file, s)
    return a.settings_file, s


def _datasets(t, device):
    """``train.data``: "synthetic" (default: model-shaped float tensors resident on the device),
    "cifar10_bin" (the real CIFAR-10 binary files under ``train.data_dir``, default ./data as in
    REF/data_and_toy_model.py:31-36) or "cifar_uint8" (synthetic CIFAR-10-layout uint8 images);
    host images go through the native prefetcher and the on-device Resize / Flip / Normalize,
    the reference's input pipeline."""
    from .data import SyntheticDataset, cifar_like_uint8, load_cifar10_bin
    from .models.registry import input_shape

    kind = t.get("data", "synthetic")
    if kind in ("cifar_uint8", "cifar10_bin"):
        if t["model"].lower().startswith(("toy_mlp", "mlp")):
            raise ValueError(f"data: {kind} feeds image models (alexnet, resnet50)")
        if kind == "cifar10_bin":  # the real dataset, CIFAR-10 binary files under data_dir
            root = t.get("data_dir") or "./data"
            return load_cifar10_bin(root, train=True), load_cifar10_bin(root, train=False)
        return (cifar_like_uint8(t["n_train"], seed=0), cifar_like_uint8(t["n_test"], seed=1))
    shape = input_shape(t["model"], t["image_size"])
    return (SyntheticDataset(t["n_train"], shape, 10, seed=0, device=device),
            SyntheticDataset(t["n_test"], shape, 10, seed=1, device=device))


def _loader(t, ds, batch, sampler, device, train: bool):
    """DeviceLoader over device-resident data, or the host pipeline (PrefetchLoader: native
    prefetch threads, uint8 H2D, on-device transform) for host datasets."""
    from .data import DeviceLoader, HostImageDataset, ImageTransform, PrefetchLoader

    if isinstance(ds, HostImageDataset):
        tf = ImageTransform(size=t["image_size"], flip_p=0.5 if train else 0.0)
        return PrefetchLoader(ds, batch, sampler=sampler, transform=tf, device=device,
                              seed=t.get("base_seed") or 0)
    return DeviceLoader(ds, batch, sampler=sampler)


def _optimizer(t, params):
    from . import optim

    if t["optimizer"].lower() == "sgd":
        return optim.SGD(params, lr=t["lr"], momentum=t["momentum"])
    if t["optimizer"].lower() == "adamw":
        return optim.AdamW(params, lr=t["lr"])
    return optim.Adam(params, lr=t["lr"])


def _want_fused(t, device) -> bool:
    from .utils.config import tristate

    v = tristate(t.get("fused_optimizer"))
    return device.type == "cuda" if v is None else (v and device.type == "cuda")


# ----------------------------------------------------------------------------- native DDP
def basic_ddp_training_loop(rank: int, world_size: int, save_dir: str, optional_args: dict,
                            train_cfg: dict):
    from . import nn as tnn
    from .data import DeviceLoader, DistributedSampler
    from .models.registry import build_model
    from .parallel import DDP, destroy_process_group, init_process_group
    from .parallel import runtime as rt
    from .train import run_training_loop
    from .utils.config import tristate
    from .utils.seed import set_seed_based_on_rank

    print(f"Running DDP checkpoint example on rank {rank}.")
    init_process_group(None)
    print(f"Process group initialized with backend {rt.get_backend()}, rank {rt.get_rank()}, "
          f"world size {rt.get_world_size()}.")
    set_seed_based_on_rank(rank, train_cfg.get("base_seed"))
    device = rt.device()
    train_ds, test_ds = _datasets(train_cfg, device)
    train_sampler = DistributedSampler(train_ds, num_replicas=world_size, rank=rank, shuffle=True)
    test_sampler = DistributedSampler(test_ds, num_replicas=world_size, rank=rank, shuffle=True)
    train_loader = _loader(train_cfg, train_ds, train_cfg["train_batch_size"], train_sampler,
                           device, train=True)
    test_loader = _loader(train_cfg, test_ds, train_cfg["test_batch_size"], test_sampler, device,
                          train=False)
    model = build_model(train_cfg["model"], device=device)
    ddp_model = DDP(model, device_ids=[device.index] if device.type == "cuda" else None,
                    bucket_cap_mb=train_cfg.get("bucket_cap_mb"))
    criterion = tnn.CrossEntropyLoss()
    optimizer = _optimizer(train_cfg, ddp_model.parameters())
    if _want_fused(train_cfg, device):
        # the update runs inside the gradient reduction (per bucket, sharded over ranks; in the
        # weight-gradient GEMM epilogues at world size 1); optimizer.step() becomes a no-op
        ddp_model.register_fused_optimizer(optimizer)
    run_training_loop(ddp_model, train_loader, train_sampler, test_loader, criterion, optimizer,
                      device, rank, save_dir, num_epochs=train_cfg["num_epochs"],
                      capture=tristate(train_cfg.get("capture")),
                      checkpoint_epoch=train_cfg["checkpoint_epoch"],
                      set_epoch=optional_args.get("set_epoch", True),
                      print_rand=optional_args.get("print_rand", False),
                      max_steps_per_epoch=train_cfg.get("max_steps_per_epoch"),
                      json_log=os.path.join(save_dir, "metrics.jsonl") if rank == 0 else None)
    destroy_process_group()


def train_ddp(argv=None):
    from .parallel.launcher import spawn
    from .utils.config import world_size_from

    _, s = _settings(argv, "Run script based on local_settings.yaml file.")
    optional_args = s.get("optional_args") or {}
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:  # already launched per rank
        basic_ddp_training_loop(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]),
                                s["out_dir"], optional_args, s["train"])
        return 0
    world = world_size_from(s)
    # counting devices does not initialise HIP in this (launcher) process
    have = torch.cuda.device_count()
    vehicle = os.environ.get("TDP_GPU_RELAY", "0") == "1" or \
        os.environ.get("TDP_GPU_PEER", "0") == "1"  # (these share one GPU among ranks)
    if have > 0 and world > have and not vehicle:
        # the reference fails too (cuda:{rank} does not exist, REF/multi-GPU-training-torch.py
        # :241); silently training at fewer ranks would change the global batch
        print(f"train_ddp: local.condor.num_gpus = {world} but only {have} GPU(s) are visible; "
              f"refusing to train with a different world size (set num_gpus <= {have})",
              file=sys.stderr, flush=True)
        return 2
    spawn(basic_ddp_training_loop, world, args=(world, s["out_dir"], optional_args, s["train"]))
    return 0


# ----------------------------------------------------------------------------- accelerate
def train_accelerate(argv=None):
    from . import nn as tnn
    from .accelerate import Accelerator
    from .data import DeviceLoader
    from .models.registry import build_model
    from .ops import count_correct
    from .train.graph import GraphedStep
    from .utils.config import tristate

    _, s = _settings(argv, "Run script based on local_settings.yaml file.")
    t = s["train"]
    accelerator = Accelerator()
    device = accelerator.device
    train_ds, test_ds = _datasets(t, device)
    # no sampler, no shuffle (R11)
    train_loader = _loader(t, train_ds, t["train_batch_size"], None, device, train=True)
    test_loader = _loader(t, test_ds, t["test_batch_size"], None, device, train=False)
    model = build_model(t["model"], device=device)
    criterion = tnn.CrossEntropyLoss()
    optimizer = _optimizer(t, model.parameters())
    model, optimizer, train_loader = accelerator.prepare(model, optimizer, train_loader)
    world = accelerator.num_processes
    if _want_fused(t, device):
        # the prepared model's DDP (the wrapper, or the hidden world-1 DDP of one process)
        accelerator.fuse_optimizer(model, optimizer)
    run = torch.zeros(1, device=device)  # persistent: the captured step accumulates into it

    def body(inputs, labels):  # the reference's step (REF/multi-GPU-training-accelerate.py:45-55)
        optimizer.zero_grad()
        loss = criterion(model(inputs), labels)
        accelerator.backward(loss)
        optimizer.step()
        run.add_(loss.detach())
        return loss

    cap = tristate(t.get("capture"))
    cap = (device.type == "cuda" and world > 1) if cap is None else cap
    # a captured step replays accelerator.backward's host bookkeeping once: no accumulation
    step = GraphedStep(body, warmup=2,
                       capture=cap and accelerator.gradient_accumulation_steps == 1)
    for epoch in range(t["num_epochs"]):
        model.train()
        run.zero_()
        nb = 0
        for i, (inputs, labels) in enumerate(train_loader):
            if t.get("max_steps_per_epoch") and i >= t["max_steps_per_epoch"]:
                break
            step(inputs, labels)
            nb += 1
        train_loss = (run / max(nb, 1)).item()  # per-rank mean of batch means, not reduced (R12)
        model.eval()
        acc = torch.zeros(3, device=device)
        tl = torch.zeros(1, device=device)
        nt = 0
        with torch.no_grad():
            for i, (inputs, labels) in enumerate(test_loader):  # full test set, every rank (R13)
                if t.get("max_steps_per_epoch") and i >= t["max_steps_per_epoch"]:
                    break
                out = model(inputs)
                tl += criterion(out, labels)
                count_correct(out, labels, acc)
                nt += 1
        test_loss = (tl / max(nt, 1)).item()
        test_acc = 100.0 * acc[1].item() / max(acc[2].item(), 1)
        if accelerator.is_local_main_process:
            print(f"Epoch {epoch + 1}/{t['num_epochs']}, Train Loss: {train_loss:.4f}, "
                  f"Test Loss: {test_loss:.4f}, Test Accuracy: {test_acc:.2f}%")
        if epoch % 5 == 0:
            accelerator.wait_for_everyone()
            accelerator.save_model(model, s["out_dir"])
    accelerator.print("Finished Training.")
    accelerator.end_training()
    return 0


# ----------------------------------------------------------------------------- launch
def write_condor_submission(out_dir: str, condor: dict, arguments: str, executable: str,
                            filename: str = "submission_file.sub") -> str:
    """The reference's HTCondor .sub writer (REF/submit_job.py:7-43), same keys and layout."""
    lines = [f"executable = {executable}",
             f"request_cpus = {condor['num_cpus']}",
             f"request_memory = {condor['memory_cpus']}"]
    if "num_gpus" in condor:
        lines.append(f"request_gpus = {condor['num_gpus']}")
    if "memory_gpus" in condor:
        lines.append(f"requirements = TARGET.CUDAGlobalMemoryMb > {condor['memory_gpus']}")
    lines += [f'arguments = "{arguments}"',
              f"error = {os.path.join(out_dir, 'info.err')}",
              f"output = {os.path.join(out_dir, 'info.out')}",
              f"log = {os.path.join(out_dir, 'info.log')}",
              "queue"]
    path = os.path.join(out_dir, filename)
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def launch(argv=None):
    from .parallel.launcher import run_script
    from .utils.config import load_settings, world_size_from

    ap = argparse.ArgumentParser(description="Launch a training script on this node.")
    ap.add_argument("--settings_file", required=True)
    ap.add_argument("--write-condor", action="store_true",
                    help="also write out_dir/submission_file.sub (HTCondor) and do not run")
    a = ap.parse_args(argv)
    s = load_settings(a.settings_file)
    os.makedirs(s["out_dir"], exist_ok=True)
    script = s["script_path"]
    if a.write_condor:
        p = write_condor_submission(s["out_dir"], s["local"]["condor"],
                                    f"{script} --settings_file {a.settings_file}",
                                    sys.executable)
        print(p)
        return 0
    world = world_size_from(s)
    return run_script(world, [script, "--settings_file", a.settings_file])
