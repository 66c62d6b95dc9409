"""nn.Module front-ends over the native ops (drop-in for the torch modules the reference uses).

Each subclasses its torch counterpart, so parameter names, initialisation, ``state_dict`` keys and
``repr`` are identical to torch's -- checkpoints stay interchangeable with stock PyTorch -- and
only ``forward`` is replaced. ReLU can be fused into the producing layer (``relu=True``), which is
how the models in ``models/`` express torchvision's ``Linear -> ReLU`` pairs.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from ..parallel import runtime as rt


class Linear(nn.Linear):
    def __init__(self, in_features: int, out_features: int, bias: bool = True,
                 relu: bool = False, device=None, dtype=None):
        super().__init__(in_features, out_features, bias=bias, device=device, dtype=dtype)
        self.relu = relu

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias, relu=self.relu)

    def extra_repr(self) -> str:
        return super().extra_repr() + (", relu=True" if self.relu else "")


class Conv2d(nn.Conv2d):
    """``nn.Conv2d`` (groups=1, dilation=1, zero padding) on the implicit-GEMM kernels, with an
    optional fused ReLU."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 bias: bool = True, relu: bool = False, device=None, dtype=None):
        super().__init__(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                         bias=bias, device=device, dtype=dtype)
        self.relu = relu
        self.bn_stats = False  # output feeds a BatchNorm: emit its statistics (ops.conv2d)
        # The weight lives in channels_last memory ([Cout][R][S][C]): exactly the operand layout
        # of the implicit-GEMM kernels (forward B, input-gradient taps, weight-gradient output),
        # so no step permutes or copies it. Shape and state_dict keys stay torch's [Cout, C, R, S].
        if in_channels % 4 == 0:
            self.weight.data = self.weight.data.contiguous(memory_format=torch.channels_last)

    def forward(self, x, grad_into=None):
        return ops.conv2d(x, self.weight, self.bias, self.stride, self.padding, relu=self.relu,
                          grad_into=grad_into, bn_stats=self.bn_stats and self.training)

    def extra_repr(self) -> str:
        return super().extra_repr() + (", relu=True" if self.relu else "")


class ReLU(nn.ReLU):
    """Standalone ReLU (models fuse it into the producer where possible)."""

    def forward(self, x):
        return torch.relu(x)


class MaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        return ops.max_pool2d(x, self.kernel_size, self.stride, self.padding)


class AdaptiveAvgPool2d(nn.AdaptiveAvgPool2d):
    def forward(self, x):
        return ops.adaptive_avg_pool2d(x, self.output_size)


class Dropout(nn.Dropout):
    def forward(self, x):
        return ops.dropout(x, self.p, self.training)


class _NativeBN(nn.modules.batchnorm._BatchNorm):
    """Shared forward for BatchNorm{1,2}d / SyncBatchNorm."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True,
                 track_running_stats=True, relu: bool = False, device=None, dtype=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats,
                         device=device, dtype=dtype)
        self.relu = relu
        self._nbt = 0  # host mirror of num_batches_tracked: no device->host sync per step

    def _group(self):
        return None

    def relu_join(self, x, residual, grad_into=None):
        """``relu(bn(x) + residual)`` as one normalisation pass (ResNet's residual join);
        ``grad_into``: the residual's gradient goes into that ``SharedGrad``."""
        return self.forward(x, residual, relu=True, residual_grad_into=grad_into)

    def forward(self, x, residual=None, relu=None, residual_grad_into=None):
        """``relu?(bn(x) [+ residual])``; ``residual`` fuses a residual join into the
        normalisation (ResNet's ``relu(bn3(conv3(.)) + identity)``, one pass instead of two)."""
        self._check_input_dim(x)
        use_batch = self.training or not self.track_running_stats
        factor = 0.0
        nbt = None
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            if x.is_cuda:
                nbt = self.num_batches_tracked  # incremented by the merge kernel (no ATen add_)
            else:
                self.num_batches_tracked.add_(1)
            self._nbt += 1
            factor = (1.0 / self._nbt) if self.momentum is None else self.momentum
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        return ops.batch_norm(x, rm, rv, self.weight, self.bias, training=use_batch,
                              momentum=factor, eps=self.eps,
                              relu=self.relu if relu is None else relu,
                              group=self._group() if use_batch else None, residual=residual,
                              num_batches_tracked=nbt, residual_grad_into=residual_grad_into)

    def extra_repr(self) -> str:
        return super().extra_repr() + (", relu=True" if self.relu else "")


class BatchNorm1d(_NativeBN):
    def _check_input_dim(self, x):
        if x.dim() not in (2, 3):
            raise ValueError(f"expected 2D or 3D input (got {x.dim()}D input)")


class BatchNorm2d(_NativeBN):
    def _check_input_dim(self, x):
        if x.dim() != 4:
            raise ValueError(f"expected 4D input (got {x.dim()}D input)")


class SyncBatchNorm(_NativeBN):
    """Batch statistics over the whole job (README pitfall, REF/README.md:79-81).

    Synchronises only in training mode with world_size > 1 (torch semantics,
    TORCH/nn/modules/batchnorm.py:744-839); otherwise it is a plain batch norm.
    """

    def _check_input_dim(self, x):
        if x.dim() < 2:
            raise ValueError(f"expected at least 2D input (got {x.dim()}D input)")

    def _group(self):
        if self.training and rt.is_initialized() and rt.get_world_size() > 1:
            return rt.SyncGroup()
        return None

    @classmethod
    def convert_sync_batchnorm(cls, module: nn.Module, process_group=None) -> nn.Module:
        """Recursively replace every BatchNorm*D (torch's or ours) with SyncBatchNorm."""
        out = module
        if isinstance(module, nn.modules.batchnorm._BatchNorm) and not isinstance(module, cls):
            out = cls(module.num_features, module.eps, module.momentum, module.affine,
                      module.track_running_stats, relu=getattr(module, "relu", False))
            if module.affine:
                with torch.no_grad():
                    out.weight = module.weight
                    out.bias = module.bias
            out.running_mean = module.running_mean
            out.running_var = module.running_var
            out.num_batches_tracked = module.num_batches_tracked
            out._nbt = getattr(module, "_nbt", 0)
            out.training = module.training
        for name, child in module.named_children():
            out.add_module(name, cls.convert_sync_batchnorm(child, process_group))
        return out


class CrossEntropyLoss(nn.CrossEntropyLoss):
    def forward(self, input, target):
        if self.weight is not None:
            raise NotImplementedError("class weights are not supported by the native loss")
        return ops.cross_entropy(input, target, ignore_index=self.ignore_index,
                                 label_smoothing=self.label_smoothing, reduction=self.reduction)


convert_sync_batchnorm = SyncBatchNorm.convert_sync_batchnorm
