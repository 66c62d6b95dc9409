"""Toy MLP: the flagship model of the benchmark (BASELINE.json "toy MLP (Linear+ReLU)").

Shape follows SURVEY.md §7.1 layer 5: 9216 -> 4096 -> 4096 -> 10, i.e. exactly the classifier of
the reference's AlexNet (torchvision ``classifier``: Linear(9216,4096)+ReLU, Linear(4096,4096)+ReLU,
Linear(4096,10); REF/data_and_toy_model.py:41-45), so the gradient all-reduce per step has the
reference's message sizes (54.6 M params = 208 MiB fp32). With ``batchnorm=True`` each hidden
Linear is followed by BatchNorm1d(+ReLU), which ``convert_sync_batchnorm`` turns into SyncBN
(BASELINE.json config "toy MLP + SyncBatchNorm"). Dropout is omitted (toy model).
"""
from __future__ import annotations

import torch.nn as nn

from ..nn import BatchNorm1d, Linear


class ToyMLP(nn.Module):
    def __init__(self, in_features: int = 9216, hidden=(4096, 4096), num_classes: int = 10,
                 batchnorm: bool = False, device=None):
        super().__init__()
        self.in_features = in_features
        layers = []
        prev = in_features
        for i, h in enumerate(hidden):
            if batchnorm:
                # Linear -> BN(+ReLU fused)
                layers.append((f"fc{i + 1}", Linear(prev, h, relu=False, device=device)))
                layers.append((f"bn{i + 1}", BatchNorm1d(h, relu=True, device=device)))
            else:
                layers.append((f"fc{i + 1}", Linear(prev, h, relu=True, device=device)))
            prev = h
        layers.append((f"fc{len(hidden) + 1}", Linear(prev, num_classes, device=device)))
        for name, m in layers:
            self.add_module(name, m)
        self._order = [n for n, _ in layers]

    def forward(self, x, target=None, acc=None):
        """Logits; with ``target`` the mean cross-entropy loss instead (``acc``: the device
        metric accumulator of ops.cross_entropy): the head Linear and the loss run as ONE fused
        op (ops.linear_cross_entropy: head GEMM, loss, logits gradient and the head's input
        gradient in one launch on MI355X) -- ``model(x, target=y)`` equals
        ``cross_entropy(model(x), y)`` bit for bit."""
        x = x.reshape(x.shape[0], -1)
        order = self._order if target is None else self._order[:-1]
        for n in order:
            x = getattr(self, n)(x)
        if target is None:
            return x
        from ..ops import linear_cross_entropy

        head = getattr(self, self._order[-1])
        return linear_cross_entropy(x, head.weight, head.bias, target, acc=acc)


def toy_mlp(**kw) -> ToyMLP:
    return ToyMLP(**kw)
