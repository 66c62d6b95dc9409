"""YAML settings with the reference schema (REF/local_settings.yaml:1-14).

Keys read by the reference: ``out_dir``, ``optional_args.{set_epoch, print_rand}``,
``local.condor.num_gpus`` (world size); ``script_path`` and ``local.condor.*`` by the submitter;
``local.device`` is dead config. Optional additions (absent -> reference values) live under
``train:`` -- model, batch sizes, epochs, checkpoint interval, optimizer, lr, bucket MiB,
synthetic-data sizes, seed.
"""
from __future__ import annotations

import copy
import os

import yaml

TRAIN_DEFAULTS = {
    "model": "alexnet",          # alexnet | toy_mlp | toy_mlp_syncbn | resnet50
    "train_batch_size": 128,     # REF/multi-GPU-training-torch.py:88
    "test_batch_size": 100,      # :95
    "num_epochs": 20,            # :166
    "checkpoint_epoch": 5,       # :167
    "optimizer": "adam",         # :249
    "lr": 0.001,
    "momentum": 0.9,
    "bucket_cap_mb": None,
    "n_train": 50000,            # CIFAR-10 sizes
    "n_test": 10000,
    "image_size": 224,           # Resize(224), REF/data_and_toy_model.py:13
    "data": "synthetic",         # synthetic (device-resident) | cifar10_bin | cifar_uint8
    "data_dir": "./data",        # cifar10_bin: CIFAR-10 binary batches (REF root="./data")
    "base_seed": None,
    "max_steps_per_epoch": None,
    # MI355X execution (not in the reference): apply the optimizer inside the gradient
    # reduction (DDP.register_fused_optimizer) and replay the step as a captured hipGraph so the
    # bucket collectives overlap backward; "auto" = on a GPU (capture: with more than one rank)
    "fused_optimizer": "auto",
    "capture": "auto",
}


def load_settings(path: str) -> dict:
    with open(path) as f:
        s = yaml.safe_load(f) or {}
    s.setdefault("optional_args", {})
    s.setdefault("local", {}).setdefault("condor", {})
    t = copy.deepcopy(TRAIN_DEFAULTS)
    t.update(s.get("train") or {})
    s["train"] = t
    return s


def copy_settings_to_out_dir(settings_path: str, settings: dict) -> str:
    """The reference re-dumps the YAML into out_dir for provenance (:300-303)."""
    out_dir = settings["out_dir"]
    os.makedirs(out_dir, exist_ok=True)
    dst = os.path.join(out_dir, os.path.basename(settings_path))
    with open(dst, "w") as f:
        yaml.dump(settings, f)
    return dst


def tristate(v):
    """YAML "auto" / true / false -> None / True / False."""
    if v is None or (isinstance(v, str) and v.lower() == "auto"):
        return None
    if isinstance(v, str):
        return v.lower() in ("1", "true", "yes", "on")
    return bool(v)


def world_size_from(settings: dict, default: int = 1) -> int:
    return int(settings.get("local", {}).get("condor", {}).get("num_gpus", default) or default)
