"""Plain ``torch.nn`` versions of the benchmark models, for the stock-PyTorch comparison rows.

torchvision is not installed in this image, so the torchvision AlexNet / ResNet-50 topologies are
written out here with stock modules only (ATen -> MIOpen / hipBLASLt on ROCm). Same parameter
counts as ``models/alexnet.py`` and ``models/resnet.py``.
"""
from __future__ import annotations

import torch.nn as nn


def stock_mlp(syncbn: bool = False, dims=(9216, 4096, 4096)):
    d_in, h1, h2 = dims
    layers = [nn.Linear(d_in, h1)]
    if syncbn:
        layers.append(nn.BatchNorm1d(h1))
    layers += [nn.ReLU(inplace=True), nn.Linear(h1, h2)]
    if syncbn:
        layers.append(nn.BatchNorm1d(h2))
    layers += [nn.ReLU(inplace=True), nn.Linear(h2, 10)]
    m = nn.Sequential(*layers)
    return nn.SyncBatchNorm.convert_sync_batchnorm(m) if syncbn else m


def stock_alexnet(num_classes: int = 10):
    return nn.Sequential(
        nn.Conv2d(3, 64, 11, 4, 2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
        nn.Conv2d(64, 192, 5, padding=2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
        nn.Conv2d(192, 384, 3, padding=1), nn.ReLU(inplace=True),
        nn.Conv2d(384, 256, 3, padding=1), nn.ReLU(inplace=True),
        nn.Conv2d(256, 256, 3, padding=1), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
        nn.AdaptiveAvgPool2d((6, 6)), nn.Flatten(),
        nn.Dropout(0.5), nn.Linear(9216, 4096), nn.ReLU(inplace=True),
        nn.Dropout(0.5), nn.Linear(4096, 4096), nn.ReLU(inplace=True),
        nn.Linear(4096, num_classes))


class _Bottleneck(nn.Module):
    def __init__(self, cin, planes, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = None
        if stride != 1 or cin != planes * 4:
            self.downsample = nn.Sequential(nn.Conv2d(cin, planes * 4, 1, stride, bias=False),
                                            nn.BatchNorm2d(planes * 4))

    def forward(self, x):
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        idn = x if self.downsample is None else self.downsample(x)
        return self.relu(out + idn)


def stock_resnet50(num_classes: int = 10):
    layers = [nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
              nn.MaxPool2d(3, 2, 1)]
    cin = 64
    for planes, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for i in range(blocks):
            layers.append(_Bottleneck(cin, planes, stride if i == 0 else 1))
            cin = planes * 4
    layers += [nn.AdaptiveAvgPool2d((1, 1)), nn.Flatten(), nn.Linear(2048, num_classes)]
    m = nn.Sequential(*layers)
    for mod in m.modules():
        if isinstance(mod, nn.Conv2d):
            nn.init.kaiming_normal_(mod.weight, mode="fan_out", nonlinearity="relu")
    return m


def stock_model(name: str, syncbn: bool = False, dims=(9216, 4096, 4096)):
    if name == "toy_mlp":
        return stock_mlp(syncbn, dims)
    m = stock_alexnet() if name == "alexnet" else stock_resnet50()
    return nn.SyncBatchNorm.convert_sync_batchnorm(m) if syncbn else m
