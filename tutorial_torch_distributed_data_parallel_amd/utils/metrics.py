"""Epoch metrics kept on the device and reduced with ONE collective.

The reference accumulates ``loss.item() * batch_size`` every step (a device->host sync per
iteration) and then issues five separate 1-element all-reduces per epoch
(REF/multi-GPU-training-torch.py:198-204, §2.6 M8). Here the loss kernel adds into a device
accumulator and the epoch summary is a single coalesced all-reduce; printed values use the
reference's exact line format (:209-215).
"""
from __future__ import annotations

import time

import torch

from ..parallel import runtime as rt


class EpochMeter:
    def __init__(self, device):
        # [train_loss_sum, train_correct, train_count, test_loss_sum, test_correct, test_count]
        self.device = torch.device(device)
        self.train = torch.zeros(3, device=self.device)
        self.test = torch.zeros(3, device=self.device)
        self.t0 = time.perf_counter()
        self.steps = 0

    def reset(self):
        self.train.zero_()
        self.test.zero_()
        self.t0 = time.perf_counter()
        self.steps = 0

    def local(self):
        tr, te = self.train.tolist(), self.test.tolist()
        return {"train_loss": tr[0] / max(tr[2], 1), "train_n": int(tr[2]),
                "test_loss": te[0] / max(te[2], 1), "test_n": int(te[2])}

    def reduce(self) -> dict:
        both = torch.cat([self.train, self.test])
        rt.all_reduce(both, "sum")
        v = both.tolist()
        return {"train_loss": v[0] / max(v[2], 1), "train_n": int(v[2]),
                "test_loss": v[3] / max(v[5], 1), "test_acc": 100.0 * v[4] / max(v[5], 1),
                "test_n": int(v[5])}


def epoch_line(epoch: int, num_epochs: int, m: dict) -> str:
    return (f"Epoch {epoch + 1}/{num_epochs}, Train Loss: {m['train_loss']:.4f}, "
            f"Test Loss: {m['test_loss']:.4f}, Test Accuracy: {m['test_acc']:.2f}%")
