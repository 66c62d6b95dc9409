"""Native-backed drop-in modules (same parameter names / state_dict keys as torch.nn)."""
from .modules import (BatchNorm1d, BatchNorm2d, CrossEntropyLoss, Linear, SyncBatchNorm,
                      convert_sync_batchnorm)

__all__ = ["Linear", "BatchNorm1d", "BatchNorm2d", "SyncBatchNorm", "CrossEntropyLoss",
           "convert_sync_batchnorm"]
