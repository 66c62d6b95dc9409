"""Checkpoints, compatible with both reference entry points.

* native-DDP path (REF/multi-GPU-training-torch.py:217-223): rank 0 writes
  ``torch.save(ddp_model.state_dict(), out_dir/ckpt_{epoch}.pt)`` -- keys carry the ``module.``
  prefix, tensors stay on the rank-0 device (so loading elsewhere needs ``map_location``,
  REF/README.md:51-52) -- then every rank meets at a barrier.
* Accelerate path (REF/multi-GPU-training-accelerate.py:104-108, ACC/accelerator.py:3439-3550):
  the main process writes ``model.safetensors`` with unwrapped (prefix-free) keys.
* Addition: ``save_training_state`` / ``load_training_state`` (model + optimizer + epoch) for
  resume, which the reference lacks.
Parameters are views into a flat arena; every writer clones them into independent tensors first
(safetensors refuses shared storage, and torch.save would otherwise store the whole arena).
"""
from __future__ import annotations

import os

import torch

from ..parallel import runtime as rt


def _detach_clone(sd):
    return {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in sd.items()}


def save_on_main(obj, path: str) -> None:
    """Rank 0 writes ``obj`` with torch.save; all ranks then synchronise."""
    if rt.get_rank() == 0:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = path + ".tmp"
        torch.save(obj, tmp)
        os.replace(tmp, path)
    rt.barrier()


def save_ddp_checkpoint(ddp_model, save_dir: str, epoch: int) -> str:
    path = os.path.join(save_dir, f"ckpt_{epoch}.pt")
    if getattr(ddp_model, "full_state_dict", None) is not None:
        # a sharded model (parallel/tensor_parallel.py): assembling the full state dict is a
        # collective every rank joins; rank 0 writes it with the DDP key contract ("module."
        # prefix, REF/multi-GPU-training-torch.py:221), so a DDP model loads it unchanged
        full = ddp_model.full_state_dict()
        sd = {f"module.{k}": v for k, v in _detach_clone(full).items()} \
            if rt.get_rank() == 0 else None
    else:
        sd = _detach_clone(ddp_model.state_dict()) if rt.get_rank() == 0 else None
    save_on_main(sd, path)
    return path


def unwrap_model(model):
    while hasattr(model, "module") and isinstance(model.module, torch.nn.Module):
        model = model.module
    return model


def strip_prefix(sd: dict, prefix: str = "module.") -> dict:
    return {(k[len(prefix):] if k.startswith(prefix) else k): v for k, v in sd.items()}


def load_checkpoint(model, path: str, map_location=None, strict: bool = True):
    """Load a ckpt_{epoch}.pt (or model.safetensors) into a wrapped or bare model."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file

        sd = load_file(path, device=str(map_location) if map_location is not None else "cpu")
    else:
        sd = torch.load(path, map_location=map_location, weights_only=True)
    target = unwrap_model(model)
    return target.load_state_dict(strip_prefix(sd), strict=strict)


def save_model_safetensors(model, save_dir: str, filename: str = "model.safetensors") -> str:
    """Accelerate-style save_model: unwrapped keys, main process only."""
    path = os.path.join(save_dir, filename)
    m = unwrap_model(model)
    full = None
    if getattr(m, "full_state_dict", None) is not None:
        # a sharded model: the full state dict is a collective (all-gathers) every rank joins
        full = m.full_state_dict()
    if rt.get_rank() == 0:
        from safetensors.torch import save_file

        os.makedirs(save_dir, exist_ok=True)
        sd = {k: v.detach().to("cpu").contiguous().clone()
              for k, v in (full if full is not None else m.state_dict()).items()}
        save_file(sd, path, metadata={"format": "pt"})
    return path


def save_training_state(path: str, model, optimizer=None, epoch: int | None = None,
                        extra: dict | None = None) -> None:
    """Model + optimizer + epoch, rank 0 writes (every rank must call it: a sharded model's
    state and a sharded optimizer's state are assembled by collectives first)."""
    m = unwrap_model(model)
    obj = {"model": _detach_clone(m.state_dict()), "epoch": epoch, "extra": extra or {}}
    if optimizer is not None:
        ddp = getattr(optimizer, "_fused_ddp", None)
        if ddp is not None:  # sharded in-reduction updates: gather the state slices first
            ddp.consolidate_optimizer_state()
        if getattr(m, "full_optim_state_dict", None) is not None:
            # tensor-sharded model: every rank's slice of the momentum / moments, gathered into
            # the full model's layout (not rank 0's shard)
            obj["optimizer"] = m.full_optim_state_dict(optimizer)
        else:
            obj["optimizer"] = optimizer.state_dict()
    save_on_main(obj if rt.get_rank() == 0 else None, path)


def load_training_state(path: str, model, optimizer=None, map_location=None) -> dict:
    obj = torch.load(path, map_location=map_location, weights_only=True)
    m = unwrap_model(model)
    m.load_state_dict(strip_prefix(obj["model"]))
    if optimizer is not None and "optimizer" in obj:
        if getattr(m, "load_full_optim_state_dict", None) is not None:
            m.load_full_optim_state_dict(optimizer, obj["optimizer"])  # re-shard
        else:
            optimizer.load_state_dict(obj["optimizer"])
    return obj
