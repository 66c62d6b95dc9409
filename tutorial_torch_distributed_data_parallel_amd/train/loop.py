"""Training orchestration with the reference's observable behaviour.

``train`` / ``evaluate`` / ``run_training_loop`` mirror REF/multi-GPU-training-torch.py:104-225:
per-rank debug prints (data sample every 100 batches, per-rank losses), ``set_epoch`` per epoch,
optional RNG-state print, barrier, globally reduced metrics printed by rank 0 in the reference's
exact format, rank-0 checkpoint ``ckpt_{epoch}.pt`` every ``checkpoint_epoch`` epochs followed by
a barrier. What changes is where the work happens: metric sums stay on the device (no
``loss.item()`` per step), the five metric all-reduces are one, and batches are gathered on the
device by the sampler's indices.
"""
from __future__ import annotations

import json
import os
import time

import torch

from .. import ops
from ..nn import CrossEntropyLoss
from ..parallel import runtime as rt
from ..utils import fault
from ..utils import profiling as prof
from ..utils.checkpoint import save_ddp_checkpoint
from ..utils.metrics import EpochMeter, epoch_line
from ..utils.seed import rng_report
from .graph import GraphedStep


def _loss(criterion, outputs, labels, acc):
    if isinstance(criterion, CrossEntropyLoss) or criterion is None:
        ignore = criterion.ignore_index if criterion is not None else -100
        smooth = criterion.label_smoothing if criterion is not None else 0.0
        return ops.cross_entropy(outputs, labels, ignore_index=ignore, label_smoothing=smooth,
                                 acc=acc)
    loss = criterion(outputs, labels)
    with torch.no_grad():
        n = labels.shape[0]
        acc[0] += loss.detach().float() * n
        acc[2] += n
    return loss


def _sample_repr(inputs):
    if inputs.dim() == 4 and inputs.shape[2] > 100 and inputs.shape[3] > 103:
        return inputs[0, 0, 100, 100:104]  # the reference's per-rank data check (:112-115)
    return inputs.reshape(inputs.shape[0], -1)[0, :4]


def make_step(model, criterion, optimizer, meter: EpochMeter):
    """One training step ``body(inputs, labels) -> loss`` (the reference's hot loop body,
    REF/multi-GPU-training-torch.py:118-126): zero_grad -> forward -> loss (accumulated into the
    device meter) -> backward (the DDP reducer syncs buckets here) -> optimizer step. Safe to
    capture: every tensor it touches persists across calls."""

    def body(inputs, labels):
        optimizer.zero_grad(set_to_none=True)
        with prof.range("forward"):
            outputs = model(inputs)
            loss = _loss(criterion, outputs, labels, meter.train)
        with prof.range("backward+reduce"):
            ops.backward(loss)  # loss.backward() seeded with a cached 1 (no fill kernel per step)
        with prof.range("optimizer"):
            optimizer.step()
        return loss
    return body


def train(model, train_loader, criterion, optimizer, device, meter: EpochMeter | None = None,
          print_every: int = 100, max_steps: int | None = None, global_step: int = 0,
          verbose: bool = True, stepper=None):
    """One epoch. ``stepper(inputs, labels)`` runs the step (a :class:`GraphedStep` replaying a
    captured hipGraph, train/graph.py); None = ``make_step`` eagerly."""
    model.train()
    meter = meter or EpochMeter(device)
    step = stepper or make_step(model, criterion, optimizer, meter)
    steps = 0
    for batch_idx, (inputs, labels) in enumerate(train_loader):
        if max_steps is not None and batch_idx >= max_steps:
            break
        inputs = inputs.to(device, non_blocking=True)
        labels = labels.to(device, non_blocking=True)
        if verbose and print_every and batch_idx % print_every == 0:
            print(f"TRAIN: Device {device}, Batch {batch_idx}, Data {_sample_repr(inputs)}")
        fault.maybe_inject(rt.get_rank(), global_step + batch_idx)
        step(inputs, labels)
        steps += 1
    meter.steps += steps
    return meter.train[0:1].clone(), meter.train[2:3].clone()


@torch.no_grad()
def evaluate(model, test_loader, criterion, device, meter: EpochMeter | None = None,
             max_steps: int | None = None):
    model.eval()
    meter = meter or EpochMeter(device)
    for i, (inputs, labels) in enumerate(test_loader):
        if max_steps is not None and i >= max_steps:
            break
        inputs = inputs.to(device, non_blocking=True)
        labels = labels.to(device, non_blocking=True)
        outputs = model(inputs)
        _loss(criterion, outputs, labels, meter.test)  # CE: loss + correct + count, one kernel
        if not (isinstance(criterion, CrossEntropyLoss) or criterion is None):
            scratch = torch.zeros(3, device=meter.test.device)
            ops.count_correct(outputs, labels, scratch)
            meter.test[1] += scratch[1]
    return meter.test[0:1].clone(), meter.test[1:2].clone(), meter.test[2:3].clone()


def run_training_loop(model, train_loader, train_sampler, test_loader, criterion, optimizer,
                      device, rank: int, save_dir: str | None, num_epochs: int = 20,
                      checkpoint_epoch: int = 5, set_epoch: bool = True,
                      print_rand: bool = False, max_steps_per_epoch: int | None = None,
                      json_log: str | None = None, verbose: bool = True,
                      capture: bool | None = None):
    """``capture``: run the training step as a captured hipGraph (GraphedStep) -- None = auto:
    on a GPU with more than one rank, where it is what overlaps the gradient collectives with
    backward; TDP_CAPTURE=0/1 overrides auto."""
    print(f"Training on {len(train_loader)} samples, test on {len(test_loader)} samples")
    meter = EpochMeter(device)
    if capture is None:
        env = os.environ.get("TDP_CAPTURE")
        capture = (env == "1") if env in ("0", "1") else \
            (device.type == "cuda" and rt.get_world_size() > 1)
    stepper = GraphedStep(make_step(model, criterion, optimizer, meter), warmup=2,
                          capture=capture and device.type == "cuda")
    history = []
    global_step = 0
    for epoch in range(num_epochs):
        if verbose:
            print(f"Device {device}, Epoch {epoch}")
        if set_epoch and train_sampler is not None:
            train_sampler.set_epoch(epoch)  # reshuffle differently every epoch
            if verbose:
                print("DistributedSampler.set_epoch:", set_epoch)
        if print_rand:
            print(rng_report(device))
        meter.reset()
        t0 = time.perf_counter()
        train(model, train_loader, criterion, optimizer, device, meter,
              max_steps=max_steps_per_epoch, global_step=global_step, verbose=verbose,
              stepper=stepper)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        t_train = time.perf_counter() - t0
        global_step += meter.steps
        loc = meter.local()
        if verbose:
            print(f"Train loss on device {device}: {loc['train_loss']} based on "
                  f"{loc['train_n']} samples")
        evaluate(model, test_loader, criterion, device, meter, max_steps=max_steps_per_epoch)
        loc = meter.local()
        if verbose:
            print(f"Test loss on device {device}: {loc['test_loss']} based on "
                  f"{loc['test_n']} samples")
        rt.barrier()  # sync all processes before aggregating
        if verbose:
            print("Aggregating loss values ...")
        m = meter.reduce()
        m["epoch"] = epoch
        m["train_samples_per_s"] = m["train_n"] / t_train if t_train > 0 else None
        m["captured_step"] = stepper.captured
        history.append(m)
        if rank == 0:
            print(epoch_line(epoch, num_epochs, m))
            if json_log:
                with open(json_log, "a") as f:
                    f.write(json.dumps(m) + "\n")
        if save_dir is not None and checkpoint_epoch and epoch % checkpoint_epoch == 0:
            save_ddp_checkpoint(model, save_dir, epoch)  # rank 0 writes, then barrier
    print(f"Finished Training on device {device}.")
    return history
