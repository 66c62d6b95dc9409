"""Training orchestration (reference train / evaluate / run_training_loop semantics)."""
from .loop import evaluate, run_training_loop, train

__all__ = ["train", "evaluate", "run_training_loop"]
