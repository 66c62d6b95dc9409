"""Accelerate-style facade over the native runtime (the reference's second entry point).

Covers the Accelerator surface the reference uses (REF/multi-GPU-training-accelerate.py:39-141,
SURVEY.md §2.2 B16-B21): ``Accelerator()``, ``.device``, ``.is_main_process``,
``.is_local_main_process``, ``.num_processes``, ``.process_index``, ``.prepare(model, optimizer,
dataloader)``, ``.backward(loss)``, ``.wait_for_everyone()``, ``.save_model(model, dir)`` (->
``model.safetensors`` with unwrapped keys, main process only), ``.unwrap_model``, ``.print``,
plus ``gather`` / ``reduce`` / ``save_state`` / ``load_state`` / ``end_training``.

State comes from the environment like Accelerate's PartialState (ACC/state.py:177-328,769-791):
with LOCAL_RANK / WORLD_SIZE set (our launcher or torchrun) the process joins a multi-rank job
(RCCL on GPUs); under plain ``python`` it is a single process. ``prepare`` places the model on the
device and wraps it in the native DDP when there is more than one process (ACC/accelerator.py:
1882-1896); data loaders are sharded by whole batches (BatchSamplerShard semantics) and moved to
the device per batch (DataLoaderShard); optimizers are passed through (gradient accumulation
gating as AcceleratedOptimizer does).
"""
from __future__ import annotations

import contextlib
import os

import torch

from ..data.sampler import BatchShardSampler
from ..data.synthetic import DeviceLoader
from ..parallel import runtime as rt
from ..parallel.arena import flatten_module
from ..parallel.ddp import DistributedDataParallel
from ..utils import checkpoint as ckpt


class AcceleratedOptimizer:
    def __init__(self, optimizer, accelerator):
        self.optimizer = optimizer
        self._acc = accelerator

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @property
    def state(self):
        return self.optimizer.state

    def zero_grad(self, set_to_none: bool = True):
        if self._acc.sync_gradients:
            self.optimizer.zero_grad(set_to_none=set_to_none)

    def step(self, closure=None):
        if self._acc.sync_gradients:
            return self.optimizer.step(closure)
        return None

    def state_dict(self):
        return self.optimizer.state_dict()

    def load_state_dict(self, sd):
        return self.optimizer.load_state_dict(sd)


class ShardedLoader:
    """Batches of a base loader dealt to ranks round-robin, moved to the device."""

    def __init__(self, base, accelerator, even_batches: bool = True):
        self.base = base
        self.acc = accelerator
        self.even = even_batches
        self.sampler = getattr(base, "sampler", None)

    def set_epoch(self, epoch: int):
        if self.sampler is not None and hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

    def _device_loader(self):
        b = self.base
        order = list(b.sampler) if b.sampler is not None else list(range(len(b.dataset)))
        bs = BatchShardSampler(len(order), b.batch_size, self.acc.num_processes,
                               self.acc.process_index, drop_last=b.drop_last,
                               even_batches=self.even, order=order)
        return DeviceLoader(b.dataset, b.batch_size, batch_sampler=bs, device=self.acc.device)

    def epoch_indices(self) -> torch.Tensor:
        """This rank's whole epoch of sample indices as one device tensor (its batches, in
        order): callers that gather batches themselves (bench.py's captured step)."""
        if not isinstance(self.base, DeviceLoader):
            raise TypeError("epoch_indices needs a DeviceLoader base")
        return self._device_loader().epoch_indices()

    def __iter__(self):
        # Accelerate's GradientState.end_of_dataloader: the last batch of an epoch always syncs
        # gradients inside accumulate() (ACC/data_loader.py DataLoaderShard look-ahead)
        self.acc.end_of_dataloader = False
        if isinstance(self.base, DeviceLoader):
            dl = self._device_loader()
            n = len(dl)
            for i, batch in enumerate(dl):
                self.acc.end_of_dataloader = i == n - 1
                yield batch
            return
        # host datasets: the same one-batch look-ahead, so the last batch this rank yields --
        # the even_batches completion round included -- is flagged end_of_dataloader
        dev = self.acc.device
        it = self._host_batches()
        cur = next(it, None)
        while cur is not None:
            nxt = next(it, None)
            self.acc.end_of_dataloader = nxt is None
            yield _to_device(cur, dev)
            cur = nxt

    def _host_batches(self):
        """This rank's batches of a host loader: round-robin over whole batches
        (BatchSamplerShard with split_batches=False, ACC/data_loader.py:213-271)."""
        W, r = self.acc.num_processes, self.acc.process_index
        batches = []
        for batch in self.base:
            batches.append(batch)
            if len(batches) == W:
                yield batches[r]
                batches = []
        if batches and self.even:
            # complete the last round with batches from the start, like even_batches=True
            head = iter(self.base)
            while len(batches) < W:
                batches.append(next(head))
            yield batches[r]
        elif len(batches) > r:
            yield batches[r]

    def __len__(self):
        n = len(self.base)
        W = self.acc.num_processes
        return -(-n // W) if self.even else len(range(self.acc.process_index, n, W))


def _to_device(batch, dev):
    if torch.is_tensor(batch):
        return batch.to(dev, non_blocking=True)
    if isinstance(batch, (list, tuple)):
        return type(batch)(_to_device(b, dev) for b in batch)
    if isinstance(batch, dict):
        return {k: _to_device(v, dev) for k, v in batch.items()}
    return batch


class Accelerator:
    def __init__(self, cpu: bool = False, gradient_accumulation_steps: int = 1,
                 even_batches: bool = True, ddp_kwargs: dict | None = None):
        if not rt.is_initialized():
            multi = int(os.environ.get("WORLD_SIZE", "1")) > 1 or "LOCAL_RANK" in os.environ
            backend = "gloo" if (cpu or not torch.cuda.is_available()) else "nccl"
            if multi:
                rt.init_process_group(backend)
            else:
                rt.init_process_group(backend, rank=0, world_size=1, local_rank=0)
        self.device = rt.device()
        self.gradient_accumulation_steps = max(1, int(gradient_accumulation_steps))
        self.even_batches = even_batches
        self.ddp_kwargs = ddp_kwargs or {}
        self._step = 0
        self.sync_gradients = True
        self.end_of_dataloader = False
        self._models = []
        self._hidden = {}  # id(prepared one-process model) -> its world-1 DDP

    # ------------------------------------------------------------------ process state
    @property
    def num_processes(self) -> int:
        return rt.get_world_size()

    @property
    def process_index(self) -> int:
        return rt.get_rank()

    @property
    def local_process_index(self) -> int:
        return rt.get_local_rank()

    @property
    def is_main_process(self) -> bool:
        return rt.get_rank() == 0

    @property
    def is_local_main_process(self) -> bool:
        return rt.get_local_rank() == 0

    @property
    def distributed_type(self) -> str:
        return "MULTI_GPU" if (self.num_processes > 1 and self.device.type == "cuda") else (
            "MULTI_CPU" if self.num_processes > 1 else "NO")

    def print(self, *a, **k):
        if self.is_local_main_process:
            print(*a, **k)

    # ------------------------------------------------------------------ prepare
    def prepare_model(self, model):
        model = model.to(self.device)
        dev_ids = [self.device.index] if self.device.type == "cuda" else None
        if isinstance(model, DistributedDataParallel) or id(model) in self._hidden:
            pass  # already prepared (or wrapped by the caller)
        elif self.num_processes > 1:
            model = DistributedDataParallel(model, device_ids=dev_ids, **self.ddp_kwargs)
        elif self.device.type == "cuda":
            # one process: Accelerate hands the module back unwrapped, and so does this. A
            # world-1 DDP still runs underneath (no collectives): its forward pre-hook does the
            # per-iteration bookkeeping, and it is what a fused optimizer registers on, so the
            # update can run in the weight-gradient GEMM epilogues as with the native DDP
            # entry point (ddp_of / fuse_optimizer)
            d = DistributedDataParallel(model, device_ids=dev_ids, **self.ddp_kwargs)

            def pre(_m, _inp, _d=d):
                _d._hidden_sample = _d._pre_forward()

            def post(_m, _inp, _out, _d=d):
                if getattr(_d, "_hidden_sample", False):
                    _d._cur_ev["fwd1"] = _d._event()
            model.register_forward_pre_hook(pre)
            model.register_forward_hook(post)
            self._hidden[id(model)] = d
        else:
            flatten_module(model)  # single CPU process: still one flat arena for the flat step
        self._models.append(model)
        return model

    def ddp_of(self, model):
        """The DDP behind a prepared model: the model itself when it is one (several
        processes), the hidden world-1 DDP of a one-process GPU model, else None."""
        if isinstance(model, DistributedDataParallel):
            return model
        return self._hidden.get(id(model))

    def fuse_optimizer(self, model, optimizer) -> bool:
        """Apply ``optimizer`` inside the gradient reduction of ``model``'s DDP (in the
        weight-gradient GEMM epilogues at world size 1): ``DDP.register_fused_optimizer``.
        False when the model has no DDP (a CPU process) or the optimizer is not fusable."""
        d = self.ddp_of(model)
        opt = optimizer.optimizer if isinstance(optimizer, AcceleratedOptimizer) else optimizer
        return bool(d is not None and d.register_fused_optimizer(opt))

    def prepare_optimizer(self, opt):
        return AcceleratedOptimizer(opt, self)

    def prepare_data_loader(self, loader):
        return ShardedLoader(loader, self, even_batches=self.even_batches)

    def _prepare_one(self, obj):
        if isinstance(obj, torch.nn.Module):
            return self.prepare_model(obj)
        if isinstance(obj, torch.optim.Optimizer):
            return self.prepare_optimizer(obj)
        if isinstance(obj, (torch.utils.data.DataLoader, DeviceLoader)):
            return self.prepare_data_loader(obj)
        return obj

    def prepare(self, *objs):
        # models first (parameters move into the arena before optimizers are wrapped)
        out = [None] * len(objs)
        for i, o in enumerate(objs):
            if isinstance(o, torch.nn.Module):
                out[i] = self._prepare_one(o)
        for i, o in enumerate(objs):
            if out[i] is None:
                out[i] = self._prepare_one(o)
        return out[0] if len(out) == 1 else tuple(out)

    # ------------------------------------------------------------------ training
    @contextlib.contextmanager
    def accumulate(self, *models):
        """Gradient accumulation (ACC/accelerator.py ``accumulate`` / ``_do_sync``): every call
        is one micro-step; gradients are synchronised on every
        ``gradient_accumulation_steps``-th one (and on an epoch's last batch). The other
        micro-steps run the DDP models under ``no_sync()`` -- the reducer issues no collective
        and gradients accumulate locally in the arena -- and the prepared optimizer's ``step`` /
        ``zero_grad`` are skipped. With a fused optimizer registered, its in-reduction update
        happens on the synchronising micro-step only (the accumulated gradient goes through the
        bucket path)."""
        # Accelerate's _do_sync: the epoch's last batch forces a sync AND restarts the window
        # (step = 0), so every epoch's windows start at its first batch
        if self.end_of_dataloader:
            self._step = 0
            self.sync_gradients = True
        else:
            self._step += 1
            self.sync_gradients = self._step % self.gradient_accumulation_steps == 0
        with contextlib.ExitStack() as stack:
            if not self.sync_gradients:
                for m in models or self._models:
                    d = self.ddp_of(m)
                    if d is not None:
                        stack.enter_context(d.no_sync())
            yield

    @contextlib.contextmanager
    def no_sync(self, model):
        d = self.ddp_of(model)
        with (d.no_sync() if d is not None else contextlib.nullcontext()):
            yield

    def backward(self, loss, **kwargs):
        """``loss / gradient_accumulation_steps`` then backward (ACC/accelerator.py:2818-2850);
        whether this backward synchronises is decided by :meth:`accumulate`."""
        if "gradient" in kwargs:
            (loss / self.gradient_accumulation_steps).backward(**kwargs)
        else:  # seeded with a cached 1/steps tensor: no fill or division kernel per step
            from ..ops.loss import backward
            backward(loss, 1.0 / self.gradient_accumulation_steps, **kwargs)

    def clip_grad_norm_(self, parameters, max_norm: float, norm_type: float = 2.0):
        """Clip the (already averaged) gradients: native on MI355X (tdp.nn.utils)."""
        from ..nn.utils import clip_grad_norm_

        return clip_grad_norm_(parameters, max_norm, norm_type)

    def wait_for_everyone(self):
        rt.barrier()

    def gather(self, t: torch.Tensor) -> torch.Tensor:
        return rt.all_gather_flat(t).reshape(self.num_processes * t.shape[0], *t.shape[1:]) \
            if t.dim() > 0 else rt.all_gather_flat(t.reshape(1))

    def reduce(self, t: torch.Tensor, reduction: str = "sum") -> torch.Tensor:
        t = t.clone()
        rt.all_reduce(t, "sum")
        if reduction == "mean":
            t /= self.num_processes
        return t

    def unwrap_model(self, model):
        return ckpt.unwrap_model(model)

    def save_model(self, model, save_directory: str, safe_serialization: bool = True):
        if not safe_serialization:
            path = os.path.join(save_directory, "pytorch_model.bin")
            if self.is_main_process:
                os.makedirs(save_directory, exist_ok=True)
                torch.save({k: v.detach().cpu().clone()
                            for k, v in self.unwrap_model(model).state_dict().items()}, path)
            return path
        return ckpt.save_model_safetensors(model, save_directory)

    def save_state(self, output_dir: str, model=None, optimizer=None):
        model = model if model is not None else (self._models[0] if self._models else None)
        opt = optimizer.optimizer if isinstance(optimizer, AcceleratedOptimizer) else optimizer
        ckpt.save_training_state(os.path.join(output_dir, "state.pt"), model, opt)

    def load_state(self, input_dir: str, model=None, optimizer=None):
        model = model if model is not None else (self._models[0] if self._models else None)
        opt = optimizer.optimizer if isinstance(optimizer, AcceleratedOptimizer) else optimizer
        return ckpt.load_training_state(os.path.join(input_dir, "state.pt"), model, opt,
                                        map_location=self.device)

    def end_training(self):
        rt.destroy_process_group()
