"""ResNet-50 (torchvision v1.5 topology) -- BASELINE.json config "ResNet-50-sized CNN DDP 8x".

``state_dict`` keys match ``torchvision.models.resnet50`` (conv1/bn1/layer1-4/fc, Bottleneck
conv1-3/bn1-3/downsample.{0,1}); stride sits on the 3x3 conv (v1.5). 25.6 M parameters in 161
tensors -- many small gradients, which is what stresses the bucketed all-reduce overlap (SURVEY.md
§2.6). ReLU is fused into the batch-norm kernels (``relu=True``) and the residual join
``relu(bn3(conv3) + identity)`` is fused into bn3's normalisation pass (and its backward). ``convert_sync_batchnorm`` turns the BatchNorm2d layers into SyncBatchNorm.
Weights use torchvision's initialisation (Kaiming-normal fan_out convs, BN gamma=1 beta=0).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from ..ops._grad import SharedGrad, fork
from ..nn import AdaptiveAvgPool2d, BatchNorm2d, Conv2d, Linear, MaxPool2d


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, device=None):
        super().__init__()
        kw = dict(bias=False, device=device)
        self.conv1 = Conv2d(inplanes, planes, 1, **kw)
        self.bn1 = BatchNorm2d(planes, relu=True, device=device)
        self.conv2 = Conv2d(planes, planes, 3, stride=stride, padding=1, **kw)
        self.bn2 = BatchNorm2d(planes, relu=True, device=device)
        self.conv3 = Conv2d(planes, planes * 4, 1, **kw)
        self.bn3 = BatchNorm2d(planes * 4, device=device)
        self.downsample = downsample
        self.stride = stride
        self._fused_join = True

    def forward(self, x):
        if self._fused_join and hasattr(self.bn3, "relu_join"):
            return self._forward_fused(x)
        out = self.bn1(self.conv1(x))
        out = self.bn2(self.conv2(out))
        identity = self.downsample(x) if self.downsample is not None else x
        out = self.bn3(self.conv3(out))
        return ops.add_relu(out, identity)

    def _forward_fused(self, x):
        # relu(bn3(conv3(.)) + identity) in the normalisation pass; its backward writes the
        # identity gradient in the same pass as bn3's (no separate add/ReLU-mask kernels).
        # x's two consumers (conv1, identity path) share ONE gradient buffer (ops/_grad.py
        # SharedGrad): bn3's backward (or the downsample conv's input gradient) writes it and
        # conv1's input-gradient GEMM accumulates into it -- no autograd add of the two.
        sink = None
        xa = xb = x
        if torch.is_grad_enabled() and x.requires_grad:
            sink = SharedGrad()
            xa, xb = fork(x, sink)
        out = self.bn1(self.conv1(xa, grad_into=sink) if _takes_sink(self.conv1) else
                       self.conv1(xa))
        out = self.bn2(self.conv2(out))
        ds = self.downsample
        if ds is None:
            return self.bn3.relu_join(self.conv3(out), xb, grad_into=sink)
        if isinstance(ds, nn.Sequential) and len(ds) == 2 and _takes_sink(ds[0]):
            identity = ds[1](ds[0](xb, grad_into=sink))
        else:
            identity = ds(xb)
        return self.bn3.relu_join(self.conv3(out), identity)


def _takes_sink(m) -> bool:
    return isinstance(m, Conv2d)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 10, device=None):
        super().__init__()
        self.inplanes = 64
        self.conv1 = Conv2d(3, 64, 7, stride=2, padding=3, bias=False, device=device)
        self.bn1 = BatchNorm2d(64, relu=True, device=device)
        self.maxpool = MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(64, layers[0], 1, device)
        self.layer2 = self._make_layer(128, layers[1], 2, device)
        self.layer3 = self._make_layer(256, layers[2], 2, device)
        self.layer4 = self._make_layer(512, layers[3], 2, device)
        self.avgpool = AdaptiveAvgPool2d((1, 1))
        self.fc = Linear(512 * Bottleneck.expansion, num_classes, device=device)
        # every convolution here feeds a BatchNorm: its GEMM epilogue emits the statistics
        self.conv1.bn_stats = True
        for m in self.modules():
            if isinstance(m, Bottleneck):
                for c in (m.conv1, m.conv2, m.conv3):
                    c.bn_stats = True
                if m.downsample is not None and isinstance(m.downsample[0], Conv2d):
                    m.downsample[0].bn_stats = True
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, blocks, stride, device):
        downsample = None
        if stride != 1 or self.inplanes != planes * Bottleneck.expansion:
            downsample = nn.Sequential(
                Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False, device=device),
                BatchNorm2d(planes * 4, device=device))
        layers = [Bottleneck(self.inplanes, planes, stride, downsample, device)]
        self.inplanes = planes * 4
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes, device=device))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.bn1(self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = self.avgpool(x)
        return self.fc(x.reshape(x.shape[0], -1))


def resnet50(num_classes: int = 10, device=None) -> ResNet:
    return ResNet((3, 4, 6, 3), num_classes=num_classes, device=device)
