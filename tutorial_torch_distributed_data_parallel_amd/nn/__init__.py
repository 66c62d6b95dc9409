"""Native-backed drop-in modules (same parameter names / state_dict keys as torch.nn)."""
from . import utils
from .modules import (AdaptiveAvgPool2d, BatchNorm1d, BatchNorm2d, Conv2d, CrossEntropyLoss,
                      Dropout, Linear, MaxPool2d, ReLU, SyncBatchNorm, convert_sync_batchnorm)

__all__ = ["Linear", "Conv2d", "ReLU", "MaxPool2d", "AdaptiveAvgPool2d", "Dropout",
           "BatchNorm1d", "BatchNorm2d", "SyncBatchNorm", "CrossEntropyLoss",
           "convert_sync_batchnorm", "utils"]
