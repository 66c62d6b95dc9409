"""Multi-rank workers for the tensor-sharded toy-MLP step (parallel/tensor_parallel.py) on
CPU/gloo. Oracle: the one-process step of the FULL model on the node's batch (every rank's
batch in rank order, mean loss) with torch.optim -- what DDP's averaged all-reduce computes."""
import contextlib
import copy

import torch
import torch.distributed as dist
import torch.nn.functional as F

import tutorial_torch_distributed_data_parallel_amd as tdp
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt
from tutorial_torch_distributed_data_parallel_amd.parallel.tensor_parallel import \
    TensorParallelMLP

DIMS = dict(in_features=37, hidden=(32, 20), num_classes=5)
B = 6


def _batch(r, step):
    g = torch.Generator().manual_seed(1000 * step + r)
    return torch.randn(B, 37, generator=g) * (1 + r), torch.randint(0, 5, (B,), generator=g)


def _ref_model(bn):
    torch.manual_seed(0)
    return ToyMLP(batchnorm=bn, **DIMS)


def step_parity(rank, out_dir, bn=False, global_batch=False, steps=4, chunks=1, kind="sgd"):
    tdp.init_process_group("gloo")
    W = rt.get_world_size()
    ref = _ref_model(bn)
    model = copy.deepcopy(ref)
    if bn:
        model = tdp.nn.convert_sync_batchnorm(model)
    tp = TensorParallelMLP(model, global_batch=global_batch, overlap_chunks=chunks)
    if kind == "sgd":
        hp = dict(lr=0.05, momentum=0.9, weight_decay=1e-3)
        opt = tdp.optim.SGD(tp.parameters(), **hp)
        ropt = torch.optim.SGD(ref.parameters(), **hp)
    else:
        hp = dict(lr=1e-2, weight_decay=1e-3)
        opt = tdp.optim.Adam(tp.parameters(), **hp)
        ropt = torch.optim.Adam(ref.parameters(), **hp)
    for step in range(steps):
        xs, ys = zip(*[_batch(r, step) for r in range(W)])
        X, Y = torch.cat(xs), torch.cat(ys)
        x, y = (X, Y) if global_batch else (xs[rank], ys[rank])
        opt.zero_grad()
        out = tp(x)
        assert out.shape == (B, 5)
        tdp.ops.cross_entropy(out, ys[rank]).backward()
        tp.sync_grads()
        opt.step()
        ropt.zero_grad()
        F.cross_entropy(ref(X), Y).backward()
        ropt.step()
    full = tp.full_state_dict()
    sd = ref.state_dict()
    assert set(full) == set(sd), (sorted(full), sorted(sd))
    for k, v in sd.items():
        torch.testing.assert_close(full[k].float(), v.float(), atol=2e-5, rtol=1e-4,
                                   msg=lambda m: f"{k}: {m}")
    # every rank holds the same full model
    if W > 1:
        allsd = [None] * W
        dist.all_gather_object(allsd, {k: v.clone() for k, v in full.items()})
        for other in allsd[1:]:
            for k in full:
                assert torch.equal(other[k], allsd[0][k]), k
    # load the full state into a differently initialised wrapper: same full state back
    torch.manual_seed(5)
    fresh = ToyMLP(batchnorm=bn, **DIMS)
    if bn:
        fresh = tdp.nn.convert_sync_batchnorm(fresh)
    tp2 = TensorParallelMLP(fresh, global_batch=global_batch)
    tp2.load_full_state_dict(full)
    back = tp2.full_state_dict()
    for k in full:
        assert torch.equal(back[k], full[k]), k
    tdp.destroy_process_group()


def refuses_plain_bn(rank, out_dir):
    tdp.init_process_group("gloo")
    try:
        TensorParallelMLP(ToyMLP(batchnorm=True, **DIMS))
    except ValueError as e:
        assert "SyncBN" in str(e)
    else:
        raise AssertionError("plain BatchNorm1d before the row-parallel layer was accepted")
    tdp.destroy_process_group()


GDIMS = dict(in_features=256, hidden=(128, 64), num_classes=10)
GB = 16


def _gbatch(r, step, device="cuda"):
    g = torch.Generator().manual_seed(77 * step + r)
    return (torch.randn(GB, 256, generator=g) * (1 + 0.5 * r)).to(device), \
        torch.randint(0, 10, (GB,), generator=g).to(device)


def captured_parity(rank, out_dir, backend="peer", bn=False, steps=5, chunks=1, fused=False):
    """GPU, W ranks (peer vehicle on one GPU, or RCCL): the tensor-sharded step captured into a
    hipGraph and replayed == the same step run eagerly, BITWISE; both match the one-process
    global-batch step of the full model (torch fp32 on the GPU) to fp32 accuracy."""
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    tdp.init_process_group(backend)
    W = rt.get_world_size()

    def build():
        torch.manual_seed(0)
        m = ToyMLP(batchnorm=bn, device="cuda", **GDIMS)
        if bn:
            m = tdp.nn.convert_sync_batchnorm(m)
        t = TensorParallelMLP(m, overlap_chunks=chunks)
        o = tdp.optim.SGD(t.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        if fused:  # the shards' update inside their weight-gradient GEMMs
            assert t.register_fused_optimizer(o)
        return t, o

    t1, o1 = build()
    t2, o2 = build()
    torch.manual_seed(0)
    ref = torch.nn.Sequential()
    full = ToyMLP(batchnorm=bn, device="cuda", **GDIMS)
    rsd = {k: v.clone() for k, v in full.state_dict().items()}
    import torch.nn as nn
    layers = [nn.Linear(256, 128), nn.BatchNorm1d(128) if bn else nn.Identity(), nn.ReLU(),
              nn.Linear(128, 64), nn.BatchNorm1d(64) if bn else nn.Identity(), nn.ReLU(),
              nn.Linear(64, 10)]
    ref = nn.Sequential(*layers).cuda()
    keymap = {"0": "fc1", "1": "bn1", "3": "fc2", "4": "bn2", "6": "fc3"}
    ref.load_state_dict({f"{i}.{k.split('.', 1)[1]}": v for i, n in keymap.items()
                         for k, v in rsd.items() if k.split(".")[0] == n}, strict=True)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    sx = torch.empty(GB, 256, device="cuda")
    sy = torch.empty(GB, dtype=torch.long, device="cuda")

    def step2():
        o2.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(t2(sx), sy))
        t2.sync_grads()
        o2.step()

    g = None
    for step in range(steps):
        xs, ys = zip(*[_gbatch(r, step) for r in range(W)])
        x, y = xs[rank], ys[rank]
        o1.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(t1(x), y))
        t1.sync_grads()
        o1.step()
        sx.copy_(x)
        sy.copy_(y)
        if g is None:
            g = CapturedStep(step2, warmup=1)
        else:
            g.replay()
        ropt.zero_grad()
        F.cross_entropy(ref(torch.cat(xs)), torch.cat(ys)).backward()
        ropt.step()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(t1.parameters(), t2.parameters())):
        assert torch.equal(a, b), f"rank {rank}: captured != eager for param {i} " \
                                  f"(max diff {float((a - b).abs().max())})"
    got = t2.full_state_dict()
    want = {f"{n}.{k.split('.', 1)[1]}": v for i, n in keymap.items()
            for k, v in ref.state_dict().items() if k.split(".")[0] == i}
    for k, v in want.items():
        torch.testing.assert_close(got[k].float(), v.float(), atol=5e-5, rtol=1e-3,
                                   msg=lambda m: f"W={W} bn={bn} {k}: {m}")
    t1.check_replicas()
    t2.check_replicas()
    rt.barrier()
    tdp.destroy_process_group()


def checkpoint_roundtrip(rank, out_dir):
    """save_ddp_checkpoint of the sharded job = the unsharded ToyMLP's checkpoint: it loads into
    a plain ToyMLP (equal to the gathered state) and back into a fresh sharded wrapper."""
    import os

    from tutorial_torch_distributed_data_parallel_amd.utils.checkpoint import (
        load_checkpoint, save_ddp_checkpoint)

    tdp.init_process_group("gloo")
    torch.manual_seed(0)
    tp = TensorParallelMLP(ToyMLP(**DIMS))
    opt = tdp.optim.SGD(tp.parameters(), lr=0.05, momentum=0.9)
    x, y = _batch(rank, 0)
    tdp.ops.cross_entropy(tp(x), y).backward()
    tp.sync_grads()
    opt.step()
    path = save_ddp_checkpoint(tp, out_dir, 0)
    assert os.path.exists(path)
    full = tp.state_dict()
    # the DDP key contract (REF/multi-GPU-training-torch.py:221): "module."-prefixed keys that a
    # DDP-wrapped ToyMLP loads with load_state_dict as they are
    raw = torch.load(path, map_location="cpu", weights_only=True)
    assert set(raw) == {f"module.{k}" for k in full}, sorted(raw)
    plain = ToyMLP(**DIMS)
    load_checkpoint(plain, path)
    for k, v in plain.state_dict().items():
        assert torch.equal(v, full[k]), k
    torch.manual_seed(9)
    tp2 = TensorParallelMLP(ToyMLP(**DIMS))
    load_checkpoint(tp2, path)
    back = tp2.state_dict()
    for k in full:
        assert torch.equal(back[k], full[k]), k
    tdp.destroy_process_group()


def accumulation_parity(rank, out_dir, backend="peer", steps=3, device="cuda", delay_aux=False):
    """GPU: gradient accumulation over two micro-batches, three ways -- the fused optimizer with
    the first micro-batch under ``no_sync()``; unfused without no_sync (the first backward
    all-reduces the replicated gradients early, the second waits for it and sync_grads reduces
    the sum again; fc2's accumulated weight gradient is computed on the compute stream, where
    autograd adds it); unfused with no_sync -- each == the torch step of the full model on the
    summed global-batch gradients (r9an: before the fix of the aux-stream race, fc2.weight was
    0.3-0.5 off)."""
    import torch.nn as nn

    tdp.init_process_group(backend)
    W = rt.get_world_size()

    def build(fused):
        torch.manual_seed(0)
        t = TensorParallelMLP(ToyMLP(device=device, **GDIMS))
        o = tdp.optim.SGD(t.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
        if fused:
            assert t.register_fused_optimizer(o) == (device != "cpu")
        return t, o

    torch.manual_seed(0)
    full = ToyMLP(device=device, **GDIMS)
    rsd = {k: v.clone() for k, v in full.state_dict().items()}
    ref = nn.Sequential(nn.Linear(256, 128), nn.ReLU(), nn.Linear(128, 64), nn.ReLU(),
                        nn.Linear(64, 10)).to(device)
    keymap = {"0": "fc1", "2": "fc2", "4": "fc3"}
    ref.load_state_dict({f"{i}.{k.split('.', 1)[1]}": v for i, n in keymap.items()
                         for k, v in rsd.items() if k.split(".")[0] == n}, strict=True)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    var = {"A fused+no_sync": (build(True), True), "B unfused": (build(False), False),
           "C unfused+no_sync": (build(False), True)}
    for step in range(steps):
        for (t, o), ns in var.values():
            o.zero_grad(set_to_none=True)
            for micro in range(2):
                xs, ys = zip(*[_gbatch(r, 2 * step + micro, device) for r in range(W)])
                ctx = t.no_sync() if micro == 0 and ns else contextlib.nullcontext()
                if delay_aux and micro == 0 and t.aux_stream() is not None:
                    # a long kernel queued on the aux stream makes the first pass's
                    # fc2 weight gradient land late; the second pass's accumulation must wait
                    # for it (without the forward's wait it read the slot before the write)
                    big = torch.randn(2048, 2048, device=device)
                    with torch.cuda.stream(t.aux_stream()):
                        for _ in range(24):
                            big = big @ big
                            big = big / big.abs().max()
                with ctx:
                    tdp.ops.backward(tdp.ops.cross_entropy(t(xs[rank]), ys[rank]))
            t.sync_grads()
            o.step()
        ropt.zero_grad()
        for micro in range(2):
            xs, ys = zip(*[_gbatch(r, 2 * step + micro, device) for r in range(W)])
            F.cross_entropy(ref(torch.cat(xs)), torch.cat(ys)).backward()
        ropt.step()
    if device != "cpu":
        torch.cuda.synchronize()
    want = {f"{n}.{k.split('.', 1)[1]}": v for i, n in keymap.items()
            for k, v in ref.state_dict().items() if k.split(".")[0] == i}
    for name, ((t, o), ns) in var.items():
        got = t.full_state_dict()
        for k, v in want.items():
            torch.testing.assert_close(got[k].float(), v.float(), atol=5e-5, rtol=1e-3,
                                       msg=lambda m: f"{name} {k}: {m}")
        t.check_replicas()
    rt.barrier()
    tdp.destroy_process_group()


def resume_parity(rank, out_dir, kind="sgd", bn=False):
    """train 3 steps, save_training_state, resume into a FRESH wrapper and
    optimizer (different init), 2 more steps == 5 uninterrupted steps, bitwise, on every rank;
    the saved optimizer state is the full model's (every rank's momentum / moment slices), and
    save_model_safetensors of the sharded model completes (a collective every rank joins)."""
    import os

    from tutorial_torch_distributed_data_parallel_amd.utils.checkpoint import (
        load_training_state, save_model_safetensors, save_training_state)

    tdp.init_process_group("gloo")
    W = rt.get_world_size()

    def build(seed):
        torch.manual_seed(seed)
        m = ToyMLP(batchnorm=bn, **DIMS)
        if bn:
            m = tdp.nn.convert_sync_batchnorm(m)
        t = TensorParallelMLP(m)
        o = (tdp.optim.SGD(t.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-3)
             if kind == "sgd" else tdp.optim.Adam(t.parameters(), lr=1e-2, weight_decay=1e-3))
        return t, o

    def train(t, o, steps):
        for step in steps:
            x, y = _batch(rank, step)
            o.zero_grad()
            tdp.ops.cross_entropy(t(x), y).backward()
            t.sync_grads()
            o.step()

    ta, oa = build(0)
    train(ta, oa, range(5))
    tb, ob = build(0)
    train(tb, ob, range(3))
    path = os.path.join(out_dir, "state.pt")
    save_training_state(path, tb, ob, epoch=3)
    sf = save_model_safetensors(tb, out_dir)
    rt.barrier()
    assert os.path.exists(sf)
    obj = torch.load(path, map_location="cpu", weights_only=True)
    full = obj["optimizer"]
    key = "momentum_buffer" if kind == "sgd" else "exp_avg"
    # state index 0 = fc1.weight in the full layout: all W row slices present, not one
    assert full["state"][0][key].shape == ta.full_state_dict()["fc1.weight"].shape
    tc, oc = build(123)  # a fresh job with different weights
    load_training_state(path, tc, oc)
    train(tc, oc, range(3, 5))
    for (n, a), (_, c) in zip(ta.named_parameters(), tc.named_parameters()):
        assert torch.equal(a, c), f"rank {rank} W={W} {kind}: {n} differs after resume " \
                                  f"(max {float((a - c).abs().max())})"
    for qa, qc in zip(ta.parameters(), tc.parameters()):
        sa, sc = oa.state[qa], oc.state[qc]
        for k, v in sa.items():
            if torch.is_tensor(v) and v.dim():
                assert torch.equal(v, sc[k]), (kind, k)
    tdp.destroy_process_group()
