"""AlexNet with a 10-class head -- the reference's model (REF/data_and_toy_model.py:41-45).

Same topology and ``state_dict`` keys as ``torchvision.models.alexnet`` (``features.{0,3,6,8,10}``,
``classifier.{1,4,6}``), so torchvision checkpoints load unchanged (the reference loads ImageNet
weights and replaces ``classifier[6]`` by ``Linear(4096, 10)``; there is no network here, so
weights are random-init with torchvision's default initialisers). ReLUs are fused into the
producing conv / linear epilogues; the ReLU slots stay as parameter-free placeholders to keep the
Sequential indices (and hence the checkpoint keys) identical. Input: 3x224x224 (CIFAR-10 resized,
REF/data_and_toy_model.py:13-36).
"""
from __future__ import annotations

import torch.nn as nn

from .. import ops
from ..nn import AdaptiveAvgPool2d, Conv2d, Dropout, Linear, MaxPool2d


class FusedReLU(nn.Module):
    """Placeholder for a ReLU that the previous layer already applied in its epilogue."""

    def forward(self, x):
        return x


class AlexNet(nn.Module):
    def __init__(self, num_classes: int = 10, dropout: float = 0.5, device=None):
        super().__init__()
        kw = dict(device=device)
        self.features = nn.Sequential(
            Conv2d(3, 64, kernel_size=11, stride=4, padding=2, relu=True, **kw), FusedReLU(),
            MaxPool2d(kernel_size=3, stride=2),
            Conv2d(64, 192, kernel_size=5, padding=2, relu=True, **kw), FusedReLU(),
            MaxPool2d(kernel_size=3, stride=2),
            Conv2d(192, 384, kernel_size=3, padding=1, relu=True, **kw), FusedReLU(),
            Conv2d(384, 256, kernel_size=3, padding=1, relu=True, **kw), FusedReLU(),
            Conv2d(256, 256, kernel_size=3, padding=1, relu=True, **kw), FusedReLU(),
            MaxPool2d(kernel_size=3, stride=2),
        )
        self.avgpool = AdaptiveAvgPool2d((6, 6))
        self.classifier = nn.Sequential(
            Dropout(p=dropout),
            Linear(256 * 6 * 6, 4096, relu=True, **kw), FusedReLU(),
            Dropout(p=dropout),
            Linear(4096, 4096, relu=True, **kw), FusedReLU(),
            Linear(4096, num_classes, **kw),
        )

    def forward(self, x):
        x = self.features(x)
        x = self.avgpool(x)
        x = ops.flatten(x)  # channels_last -> torch's (C, H, W) feature order, natively
        return self.classifier(x)


def alexnet(num_classes: int = 10, device=None, **kw) -> AlexNet:
    return AlexNet(num_classes=num_classes, device=device, **kw)
