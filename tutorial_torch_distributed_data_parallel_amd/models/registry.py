"""Model factory used by the entry scripts (`train.model` in the settings YAML)."""
from __future__ import annotations

import torch


def build_model(name: str, num_classes: int = 10, device=None) -> torch.nn.Module:
    name = name.lower()
    if name in ("toy_mlp", "mlp"):
        from .mlp import ToyMLP

        return ToyMLP(num_classes=num_classes, device=device)
    if name in ("toy_mlp_syncbn", "mlp_syncbn"):
        from ..nn import convert_sync_batchnorm
        from .mlp import ToyMLP

        return convert_sync_batchnorm(ToyMLP(num_classes=num_classes, batchnorm=True,
                                             device=device))
    if name == "alexnet":
        from .alexnet import alexnet

        return alexnet(num_classes=num_classes, device=device)
    if name in ("resnet50", "resnet-50"):
        from .resnet import resnet50

        return resnet50(num_classes=num_classes, device=device)
    raise ValueError(f"unknown model {name!r}")


def input_shape(name: str, image_size: int = 224):
    name = name.lower()
    if name.startswith("toy_mlp") or name.startswith("mlp"):
        return (9216,)
    return (3, image_size, image_size)
