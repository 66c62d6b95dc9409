"""Model zoo: the flagship toy MLP (+SyncBN variant), AlexNet (reference) and ResNet-50."""
from .mlp import ToyMLP, toy_mlp

__all__ = ["ToyMLP", "toy_mlp"]
