"""Accelerate-style facade on CPU: gradient-accumulation windows across epochs and the
end-of-dataloader flag on host loaders (ACC/accelerator.py _do_sync, ACC/data_loader.py
DataLoaderShard look-ahead)."""
import torch

import tutorial_torch_distributed_data_parallel_amd as tdp
from tutorial_torch_distributed_data_parallel_amd.accelerate import Accelerator
from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt


def _host_loader(n_batches, bs=2):
    ds = torch.utils.data.TensorDataset(torch.randn(n_batches * bs, 4),
                                        torch.randint(0, 3, (n_batches * bs,)))
    return torch.utils.data.DataLoader(ds, batch_size=bs, shuffle=False)


def _sync_pattern(acc, loader, epochs):
    out = []
    for _ in range(epochs):
        row = []
        for i, _batch in enumerate(loader):
            with acc.accumulate():
                row.append((i, acc.sync_gradients, acc.end_of_dataloader))
        out.append(row)
    return out


def test_accumulation_windows_restart_every_epoch():
    """GA=4, 10 batches per epoch: every epoch syncs after its 4th, 8th and 10th batch (the
    forced end-of-epoch sync restarts the window), not 2nd/6th/10th in epoch 2."""
    acc = Accelerator(cpu=True, gradient_accumulation_steps=4)
    try:
        loader = acc.prepare(_host_loader(10))
        pat = _sync_pattern(acc, loader, epochs=2)
        for row in pat:
            assert [i for i, s, _ in row if s] == [3, 7, 9], row
            assert [i for i, _, e in row if e] == [9], row  # host branch flags the last batch
    finally:
        rt.destroy_process_group()


def test_host_loader_end_of_dataloader_uneven():
    """A ragged epoch (7 batches, GA=3): syncs at 3, 6 and the last batch, every epoch."""
    acc = Accelerator(cpu=True, gradient_accumulation_steps=3)
    try:
        loader = acc.prepare(_host_loader(7))
        pat = _sync_pattern(acc, loader, epochs=3)
        for row in pat:
            assert len(row) == 7
            assert [i for i, s, _ in row if s] == [2, 5, 6], row
    finally:
        rt.destroy_process_group()
        assert not tdp.parallel.is_initialized()
