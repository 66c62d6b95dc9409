"""Multi-rank workers for the DEVICE sync path on ONE GPU (host-relay communicator).

Every rank of these workers runs on the same MI355X with ``init_process_group("relay")``
(parallel/relay.py): parameters, gradients, optimizer state and every kernel are on the GPU and
the C++ reducer drives RcclOps exactly as over RCCL -- sharded reduce-scatter / update /
all-gather with this rank's slices, factored Linear weights (slot-r staging, the m0 row-offset
shard GEMM, bias column sums over W*B rows, replicated updates), SyncBatchNorm -- only the bytes
travel through the host (gloo). The oracle needs no collective: every rank regenerates every
rank's batch from its seed and applies DDP semantics (average of the per-rank mean-loss
gradients) to an fp32 torch model with torch.optim.
"""
import copy

import torch
import torch.nn as nn
import torch.nn.functional as F

import tutorial_torch_distributed_data_parallel_amd as tdp
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt

# fc1 [384, 192] and fc2 [192, 384] are factor candidates at W = 2, 3, 4 (out % 4W == 0, whole
# 64-element row shards) and factoring pays at B = 16 (2 W B (out + in) <= out * in)
DIMS = dict(in_features=192, hidden=(384, 192), num_classes=10)
B = 16


def _batch(r, step, ragged_rank=-1, ragged_step=-1):
    g = torch.Generator(device="cuda").manual_seed(1000 * step + r)
    b = B // 2 if (r == ragged_rank and step == ragged_step) else B
    return (torch.randn(b, DIMS["in_features"], device="cuda", generator=g) * (1 + 0.5 * r),
            torch.randint(0, 10, (b,), device="cuda", generator=g))


def _torch_mlp(model):
    """Stock torch modules with the same parameters as a tdp ToyMLP (fp32 oracle)."""
    layers, names = [], []
    for n in model._order:
        m = getattr(model, n)
        if hasattr(m, "in_features"):
            lin = nn.Linear(m.in_features, m.out_features, device="cuda")
            lin.weight.data.copy_(m.weight.detach())
            lin.bias.data.copy_(m.bias.detach())
            layers.append(lin)
            if getattr(m, "relu", False):
                layers.append(nn.ReLU())
        else:  # tdp BatchNorm1d(relu=True)
            bn = nn.BatchNorm1d(m.num_features, eps=m.eps, momentum=m.momentum, device="cuda")
            bn.weight.data.copy_(m.weight.detach())
            bn.bias.data.copy_(m.bias.detach())
            layers.append(bn)
            if getattr(m, "relu", False):
                layers.append(nn.ReLU())
        names.append(n)
    return nn.Sequential(*layers)


def _opts(kind, ours, ref, lr):
    if kind == "sgd":
        hp = dict(lr=lr, momentum=0.9, weight_decay=1e-4)
        return tdp.optim.SGD(ours, **hp), torch.optim.SGD(ref, **hp)
    hp = dict(lr=lr, weight_decay=1e-4)
    return tdp.optim.Adam(ours, **hp), torch.optim.Adam(ref, **hp)


def _oracle_step(ref, ropt, W, step, ragged_rank, ragged_step):
    """DDP semantics without DDP: mean over ranks of each rank's mean-loss gradient."""
    ropt.zero_grad(set_to_none=True)
    for r in range(W):
        x, y = _batch(r, step, ragged_rank, ragged_step)
        (F.cross_entropy(ref(x), y) / W).backward()
    ropt.step()


def _close(model, ref, tag, atol=5e-5, rtol=2e-4):
    ours = [p.detach() for p in model.parameters()]
    theirs = [p.detach() for p in ref.parameters()]
    assert len(ours) == len(theirs)
    for i, (a, b) in enumerate(zip(ours, theirs)):
        torch.testing.assert_close(a, b, atol=atol, rtol=rtol, msg=lambda m: f"{tag} param {i}: {m}")


def collectives(rank, out_dir, backend="relay"):
    """The relay's (and the peer vehicle's) collectives have RCCL's semantics, in place
    included."""
    tdp.init_process_group(backend)
    r, W = rt.get_rank(), rt.get_world_size()
    want = "rccl" if backend in ("nccl", "rccl") else backend  # RCCL: the multi-GPU tier
    assert rt.get_backend() == want and bool(rt.comm().native_rccl) == (want == "rccl")
    t = torch.full((5,), float(r + 1), device="cuda")
    rt.all_reduce(t, "sum")
    assert torch.equal(t, torch.full_like(t, W * (W + 1) / 2))
    t = torch.full((3,), float(r), device="cuda")
    rt.all_reduce(t, "max")
    assert float(t[0]) == W - 1
    t = torch.full((4,), float(r), device="cuda", dtype=torch.bfloat16)
    rt.comm().all_reduce(t, "avg")
    torch.testing.assert_close(t.float(), torch.full((4,), (W - 1) / 2, device="cuda"))
    b = torch.full((7,), float(r), device="cuda")
    rt.broadcast(b, W - 1)
    assert torch.equal(b, torch.full_like(b, W - 1))
    g = rt.all_gather_flat(torch.tensor([r, 10 + r], device="cuda"))
    assert g.tolist() == sum([[k, 10 + k] for k in range(W)], [])
    # in place, RCCL style: send buffer = this rank's slice of the receive buffer
    flat = torch.full((W * 3,), -1.0, device="cuda")
    flat[r * 3: (r + 1) * 3] = r
    rt.comm().all_gather(flat, flat[r * 3: (r + 1) * 3])
    assert flat.tolist() == sum([[float(k)] * 3 for k in range(W)], [])
    full = torch.arange(W * 4, dtype=torch.float32, device="cuda") * (r + 1)
    rt.comm().reduce_scatter(full[r * 4: (r + 1) * 4], full, "sum")
    want = torch.arange(r * 4, (r + 1) * 4, dtype=torch.float32, device="cuda") * W * (W + 1) / 2
    assert torch.equal(full[r * 4: (r + 1) * 4], want)
    rt.barrier()
    tdp.destroy_process_group()


def ddp_parity(rank, out_dir, kind="sgd", factor=True, replicate=None, fused=True, steps=5,
               ragged=True, backend="relay"):
    """The production world>1 step on the device path vs the fp32 torch oracle: fused (sharded
    or factored) optimizer, an LR change at step 3, a ragged batch on the last rank at step 4,
    replicas bit-identical (checksum all-gather) and the reported sync plan."""
    tdp.init_process_group(backend)
    r, W = rt.get_rank(), rt.get_world_size()
    torch.manual_seed(0)
    model = ToyMLP(**DIMS, device="cuda")
    ref = _torch_mlp(model)
    ddp = tdp.DDP(model, device_ids=[rt.device().index], factor_sync=factor)
    ddp.factor_replicate = replicate
    opt, ropt = _opts(kind, ddp.parameters(), ref.parameters(), 0.05 if kind == "sgd" else 2e-3)
    if fused:
        assert ddp.register_fused_optimizer(opt)
    ragged_rank, ragged_step = (W - 1, 4) if ragged else (-1, -1)
    for step in range(steps):
        if step == 3:
            for o in (opt, ropt):
                o.param_groups[0]["lr"] *= 0.5
        x, y = _batch(r, step, ragged_rank, ragged_step)
        opt.zero_grad(set_to_none=True)
        tdp.ops.cross_entropy(ddp(x), y).backward()
        opt.step()
        _oracle_step(ref, ropt, W, step, ragged_rank, ragged_step)
    torch.cuda.synchronize()
    plan = ddp.sync_plan()
    if fused and factor:
        if isinstance(replicate, float):  # a split job: part of the rows replicated
            want = "factored-split"
        elif replicate is None:  # auto: measured bandwidth + step model (ddp._rep_rows_for)
            want = None
        else:
            want = {True: "factored-replicated", False: "factored-sharded"}[replicate]
        if want is None:
            assert plan["fc1.weight"].startswith("factored"), plan
        else:
            assert plan["fc1.weight"] == want and plan["fc2.weight"] == want, plan
        assert plan["fc1.bias"] == "factored-bias", plan
        assert set(ddp._factor_cap.values()) == {B}, ddp._factor_cap
    elif fused:
        assert plan["fc1.weight"] == "sharded", plan
    else:
        assert plan["fc1.weight"] == "allreduce", plan
    _close(model, ref, f"W={W} {kind} factor={factor} replicate={replicate} fused={fused}")
    ddp.check_replicas()  # raises if any rank's parameters differ bit-wise from rank 0's
    rt.barrier()
    tdp.destroy_process_group()


def syncbn_parity(rank, out_dir, steps=3, backend="relay"):
    """SyncBatchNorm on the device path at W ranks == BatchNorm over the concatenated global
    batch (forward statistics all-gathered, backward sums all-reduced), running stats included."""
    tdp.init_process_group(backend)
    r, W = rt.get_rank(), rt.get_world_size()
    torch.manual_seed(0)
    model = tdp.nn.convert_sync_batchnorm(ToyMLP(**DIMS, batchnorm=True, device="cuda"))
    ref = _torch_mlp(model)
    ddp = tdp.DDP(model, device_ids=[rt.device().index])
    opt = tdp.optim.SGD(ddp.parameters(), lr=0.05, momentum=0.9)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    for step in range(steps):
        x, y = _batch(r, step)
        opt.zero_grad(set_to_none=True)
        tdp.ops.cross_entropy(ddp(x), y).backward()
        opt.step()
        ropt.zero_grad(set_to_none=True)
        xs, ys = zip(*[_batch(k, step) for k in range(W)])
        out = ref(torch.cat(xs))
        # DDP averages per-rank mean losses: sum_k CE(chunk_k) / W
        sum(F.cross_entropy(o, t) for o, t in zip(out.split(B), ys)).div(W).backward()
        ropt.step()
    _close(model, ref, f"SyncBN W={W}", atol=1e-4, rtol=1e-3)
    bns = [m for m in model.modules() if hasattr(m, "running_mean")]
    rbns = [m for m in ref.modules() if isinstance(m, nn.BatchNorm1d)]
    for a, b in zip(bns, rbns):
        torch.testing.assert_close(a.running_mean, b.running_mean, atol=1e-5, rtol=1e-4)
        torch.testing.assert_close(a.running_var, b.running_var, atol=1e-4, rtol=1e-4)
    ddp.check_replicas()
    tdp.destroy_process_group()


def capture_falls_back_everywhere(rank, out_dir):
    """Injected capture failure on rank 1 (TDP_FAULT_CAPTURE=1): every rank runs eagerly, and
    the eager step still trains identically on every rank."""
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep, try_capture

    tdp.init_process_group("relay")
    r = rt.get_rank()
    torch.manual_seed(0)
    w = torch.randn(64, 64, device="cuda")
    x = torch.randn(32, 64, device="cuda")
    out = torch.empty(32, 64, device="cuda")

    def step():  # collective-free: it captures fine on rank 0
        torch.mm(x, w, out=out)
        return out

    got = try_capture(step, warmup=1, log=lambda m: None)
    assert got is step, f"rank {r}: captured while another rank fell back"
    assert not isinstance(got, CapturedStep)
    tdp.destroy_process_group()
