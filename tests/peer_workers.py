"""Multi-rank workers for the peer-memory vehicle (parallel/peer.py, csrc/peer.hip): W rank
processes on ONE GPU whose collectives are device kernels over IPC-mapped windows -- so, unlike
the host relay, the multi-rank training step can be CAPTURED into a hipGraph and replayed with
real peers. The captured-parity workers also take backend="nccl": the multi-GPU RCCL tier
(tests/test_multigpu_rccl.py) runs the same bodies with one rank per GPU. Oracles: closed-form collective results, the eager run of the same step (bitwise)
and the fp32 torch DDP-semantics oracle of relay_workers."""
import os
import sys
import time

import torch

import tutorial_torch_distributed_data_parallel_amd as tdp
from tutorial_torch_distributed_data_parallel_amd._native import native
from tutorial_torch_distributed_data_parallel_amd.models import ToyMLP
from tutorial_torch_distributed_data_parallel_amd.parallel import runtime as rt

from relay_workers import DIMS, B, _batch, _close, _oracle_step, _torch_mlp


def chunked_collectives(rank, out_dir):
    """Collectives larger than the staging slot (chunked launches), every dtype / op the
    framework issues, in place and out of place, and a CAPTURED all-reduce / all-gather pair
    replayed with new inputs (epochs live on the device)."""
    os.environ["TDP_PEER_SLOT_MB"] = "0.0625"  # 64 KiB slots: every case below is chunked
    tdp.init_process_group("peer")
    r, W = rt.get_rank(), rt.get_world_size()
    comm = rt.comm()
    assert rt.get_backend() == "peer" and not comm.native_rccl and comm.nranks == W
    assert comm.slot_bytes == 65536
    n = 50_001  # odd: vector body + scalar tail in every chunk
    base = torch.arange(n, device="cuda", dtype=torch.float64)
    for dt in (torch.float32, torch.float64, torch.int64, torch.int32):
        t = (base * (r + 1)).to(dt)
        comm.all_reduce(t, "sum")
        assert torch.equal(t, (base * (W * (W + 1) // 2)).to(dt)), dt
        t = (base + r).to(dt)
        comm.all_reduce(t, "max")
        assert torch.equal(t, (base + W - 1).to(dt)), dt
        t = (base + r).to(dt)
        comm.all_reduce(t, "min")
        assert torch.equal(t, base.to(dt)), dt
    t = torch.full((n,), float(r), device="cuda")
    comm.all_reduce(t, "avg")
    assert torch.equal(t, torch.full_like(t, sum(range(W)) / W))
    hb = torch.full((n,), float(r + 1), device="cuda", dtype=torch.bfloat16)
    comm.all_reduce(hb, "sum")
    assert torch.equal(hb.float(), torch.full((n,), float(W * (W + 1) // 2), device="cuda"))
    # all-gather, in place (send = own slice of recv)
    flat = torch.full((W * n,), -1.0, device="cuda")
    flat[r * n: (r + 1) * n] = torch.arange(n, device="cuda", dtype=torch.float32) + 1000 * r
    comm.all_gather(flat, flat[r * n: (r + 1) * n])
    want = torch.cat([torch.arange(n, device="cuda", dtype=torch.float32) + 1000 * k
                      for k in range(W)])
    assert torch.equal(flat, want)
    # reduce-scatter, in place (recv = own slice of send)
    full = torch.arange(W * n, dtype=torch.float32, device="cuda") * (r + 1)
    comm.reduce_scatter(full[r * n: (r + 1) * n], full, "sum")
    want = torch.arange(r * n, (r + 1) * n, dtype=torch.float32, device="cuda") * W * (W + 1) / 2
    assert torch.equal(full[r * n: (r + 1) * n], want)
    b = torch.full((n,), float(r), device="cuda")
    comm.broadcast(b, W - 1)
    assert torch.equal(b, torch.full_like(b, W - 1))
    # captured: the kernels' epoch comes from device memory, so replays stay in step
    x = torch.zeros(n, device="cuda")
    out = torch.zeros(W * n, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            comm.all_reduce(x, "sum")
            comm.all_gather(out, x)
    torch.cuda.current_stream().wait_stream(s)
    for it in range(3):
        x.fill_(float(r + it))
        g.replay()
        tot = float(sum(k + it for k in range(W)))
        assert torch.equal(x, torch.full_like(x, tot)), (it, float(x[0]))
        assert torch.equal(out, torch.full_like(out, tot)), it
    rt.barrier()
    tdp.destroy_process_group()


def captured_ddp_parity(rank, out_dir, kind="sgd", factor=True, replicate=None, steps=6, backend="peer"):
    """The multi-rank DDP step captured into a hipGraph and replayed with real peers (bucket
    collectives / factored gathers on the side stream, deferred forks, join) == the same step
    run eagerly, BITWISE, on every rank; both match the fp32 torch oracle; replicas identical."""
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    tdp.init_process_group(backend)
    r, W = rt.get_rank(), rt.get_world_size()
    lr = 0.05 if kind == "sgd" else 2e-3

    def build():
        torch.manual_seed(0)
        m = ToyMLP(**DIMS, device="cuda")
        d = tdp.DDP(m, device_ids=[rt.device().index], factor_sync=factor)
        d.factor_replicate = replicate
        o = (tdp.optim.SGD(d.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
             if kind == "sgd" else tdp.optim.Adam(d.parameters(), lr=lr, weight_decay=1e-4))
        assert d.register_fused_optimizer(o)
        return m, d, o

    m1, d1, o1 = build()
    m2, d2, o2 = build()
    ref = _torch_mlp(m1)
    ropt = (torch.optim.SGD(ref.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4)
            if kind == "sgd" else torch.optim.Adam(ref.parameters(), lr=lr, weight_decay=1e-4))
    sx = torch.empty(B, DIMS["in_features"], device="cuda")
    sy = torch.empty(B, dtype=torch.long, device="cuda")

    def step2():
        o2.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(d2(sx), sy))
        o2.step()

    g = None
    for step in range(steps):
        if step == 3:
            for o in (o1, o2, ropt):
                o.param_groups[0]["lr"] *= 0.5
        x, y = _batch(r, step)
        o1.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(d1(x), y))
        o1.step()
        sx.copy_(x)
        sy.copy_(y)
        if g is None:
            g = CapturedStep(step2, warmup=1)  # one real (eager) step on this batch, then record
        else:
            g.replay()
        _oracle_step(ref, ropt, W, step, -1, -1)
    torch.cuda.synchronize()
    plan = d2.sync_plan()
    if factor:
        assert plan["fc1.weight"].startswith("factored"), plan
        if isinstance(replicate, float):
            assert plan["fc1.weight"] == plan["fc2.weight"] == "factored-split", plan
    for i, (a, b) in enumerate(zip(m1.parameters(), m2.parameters())):
        assert torch.equal(a, b), f"rank {r}: captured != eager for param {i} " \
                                  f"(max diff {float((a - b).abs().max())})"
    _close(m2, ref, f"captured W={W} {kind} factor={factor} replicate={replicate}")
    d1.check_replicas()
    d2.check_replicas()
    rt.barrier()
    tdp.destroy_process_group()


def stalled_peer_times_out(rank, out_dir):
    """Rank 1 stalls its next collective 6 s (device-side, bounded) while every wait is bounded
    by TDP_PEER_TIMEOUT_S=1: rank 0's wait expires, its watchdog reports and exits 86."""
    os.environ["TDP_PEER_TIMEOUT_S"] = "1"
    tdp.init_process_group("peer")
    comm = rt.comm()
    if rt.get_rank() == 1:
        comm.inject_stall_ms(6000)
    t = torch.ones(1024, device="cuda")
    comm.all_reduce(t, "sum")
    time.sleep(30)  # the watchdog ends this process first (exit 86); never reached in time
    raise SystemExit(0)


def rccl_watchdog_child():
    """One rank on RCCL: a bounded 8 s stall ahead of a watched collective, 2 s timeout -> the
    watchdog aborts the communicator and exits 86 (run in a child process by the test)."""
    os.environ["TDP_TIMEOUT_S"] = "2"
    tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    comm = rt.comm()
    assert comm.native_rccl and comm.timeout == 2.0
    comm.set_watch_single_rank(True)
    native().debug_spin_ms(8000)
    t = torch.ones(16, device="cuda")
    comm.all_reduce(t, "sum")
    comm.watch_current("stalled collective")
    time.sleep(30)
    raise SystemExit(0)


def capture_beside_pending_watch_child():
    """One rank on RCCL with a watch pending (a 1.5 s device spin on a side stream) while the main
    thread records a hipGraph in global capture mode for 0.35 s: the watchdog thread polls the
    pending event meanwhile (every 100 ms). Its queries must not invalidate the capture (they did
    before the watchdog thread switched itself to relaxed capture mode)."""
    os.environ["TDP_TIMEOUT_S"] = "30"
    tdp.init_process_group("nccl", rank=0, world_size=1, local_rank=0)
    comm = rt.comm()
    comm.set_watch_single_rank(True)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        native().debug_spin_ms(1500)
        comm.watch_current("pending spin")
    assert comm.pending_watches() == 1
    x = torch.ones(1 << 16, device="cuda")
    torch.cuda.current_stream().synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = x * 2.0
        time.sleep(0.35)  # the watchdog wakes at least three times during the capture
        y += 1.0
    g.replay()
    torch.cuda.synchronize()
    assert float(y.sum()) == 3.0 * x.numel()
    print("capture-ok", flush=True)
    raise SystemExit(0)


if __name__ == "__main__":
    if sys.argv[1:] == ["capture_beside_pending_watch"]:
        capture_beside_pending_watch_child()
    rccl_watchdog_child()


def _eager_vs_captured(step1, step2, batches, sx, sy, fill=None):
    """Run step1 eagerly on each batch and step2 as a captured graph (one real warm-up step on
    the first batch, then replays) on the same batches, fed through the static buffers."""
    from tutorial_torch_distributed_data_parallel_amd.train.graph import CapturedStep

    g = None
    for x, y in batches:
        step1(x, y)
        if fill is not None:
            fill(x, y)
        else:
            sx.copy_(x)
            sy.copy_(y)
        if g is None:
            g = CapturedStep(step2, warmup=1)
        else:
            g.replay()
    torch.cuda.synchronize()
    return g


def _assert_bitwise(m1, m2, tag):
    r = rt.get_rank()
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(a, b), f"rank {r} {tag}: captured != eager for {n} " \
                                  f"(max diff {float((a - b).abs().max())})"
    for (n, a), b in zip(m1.named_buffers(), m2.buffers()):
        if a.is_floating_point():
            assert torch.equal(a, b), f"rank {r} {tag}: captured != eager for buffer {n}"


def captured_syncbn_parity(rank, out_dir, steps=5, backend="peer", sync1d=False):
    """BASELINE config 3 (toy MLP + SyncBatchNorm) as a CAPTURED multi-rank step with real peers:
    the forward statistics all-gather and the backward all-reduce of every BN layer are recorded
    inline on the compute stream, the bucket / factored collectives on the side stream. Captured
    == eager bitwise (parameters and running stats) on every rank; both == BN over the global
    batch (the fp32 torch oracle); replicas identical."""
    import torch.nn as nn
    import torch.nn.functional as F

    from tutorial_torch_distributed_data_parallel_amd.ops import norm as norm_mod

    norm_mod.set_sync1d(sync1d)  # the whole-column SyncBN halves (csrc/norm.hip) or the split ones
    tdp.init_process_group(backend)
    r, W = rt.get_rank(), rt.get_world_size()

    def build():
        torch.manual_seed(0)
        m = tdp.nn.convert_sync_batchnorm(ToyMLP(**DIMS, batchnorm=True, device="cuda"))
        d = tdp.DDP(m, device_ids=[rt.device().index])
        o = tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9)
        assert d.register_fused_optimizer(o)
        return m, d, o

    m1, d1, o1 = build()
    m2, d2, o2 = build()
    ref = _torch_mlp(m1)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    sx = torch.empty(B, DIMS["in_features"], device="cuda")
    sy = torch.empty(B, dtype=torch.long, device="cuda")

    def step1(x, y):
        o1.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(d1(x), y))
        o1.step()

    def step2():
        o2.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(d2(sx), sy))
        o2.step()

    batches = [_batch(r, s) for s in range(steps)]
    _eager_vs_captured(step1, step2, batches, sx, sy)
    for s in range(steps):
        ropt.zero_grad(set_to_none=True)
        xs, ys = zip(*[_batch(k, s) for k in range(W)])
        out = ref(torch.cat(xs))
        sum(F.cross_entropy(o, t) for o, t in zip(out.split(B), ys)).div(W).backward()
        ropt.step()
    _assert_bitwise(m1, m2, f"SyncBN W={W}")
    _close(m2, ref, f"captured SyncBN W={W}", atol=1e-4, rtol=1e-3)
    bns = [m for m in m2.modules() if hasattr(m, "running_mean")]
    rbns = [m for m in ref.modules() if isinstance(m, nn.BatchNorm1d)]
    assert len(bns) == len(rbns) > 0
    for a, b in zip(bns, rbns):
        torch.testing.assert_close(a.running_mean, b.running_mean, atol=1e-5, rtol=1e-4)
        torch.testing.assert_close(a.running_var, b.running_var, atol=1e-4, rtol=1e-4)
    d1.check_replicas()
    d2.check_replicas()
    rt.barrier()
    tdp.destroy_process_group()


def captured_accelerate_parity(rank, out_dir, steps=5, backend="peer"):
    """BASELINE config 4: the step through the Accelerate-style facade (prepare -> DDP, fused
    optimizer, accelerator.backward) CAPTURED with real peers == eager bitwise; both == the fp32
    torch oracle (mean over ranks of each rank's mean-loss gradient)."""
    from tutorial_torch_distributed_data_parallel_amd.accelerate import Accelerator

    tdp.init_process_group(backend)
    r, W = rt.get_rank(), rt.get_world_size()
    accel = Accelerator()
    assert accel.num_processes == W

    def build():
        torch.manual_seed(0)
        m = ToyMLP(**DIMS, device="cuda")
        o = tdp.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
        pm, po = accel.prepare(m, o)
        assert accel.fuse_optimizer(pm, po)
        return m, pm, po

    m1, p1, o1 = build()
    m2, p2, o2 = build()
    ref = _torch_mlp(m1)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    sx = torch.empty(B, DIMS["in_features"], device="cuda")
    sy = torch.empty(B, dtype=torch.long, device="cuda")

    def step1(x, y):  # REF/multi-GPU-training-accelerate.py:45-55
        o1.zero_grad()
        accel.backward(tdp.ops.cross_entropy(p1(x), y))
        o1.step()

    def step2():
        o2.zero_grad()
        accel.backward(tdp.ops.cross_entropy(p2(sx), sy))
        o2.step()

    _eager_vs_captured(step1, step2, [_batch(r, s) for s in range(steps)], sx, sy)
    for s in range(steps):
        _oracle_step(ref, ropt, W, s, -1, -1)
    _assert_bitwise(m1, m2, f"Accelerate W={W}")
    _close(m2, ref, f"captured Accelerate W={W}")
    accel.ddp_of(p2).check_replicas()
    rt.barrier()
    tdp.destroy_process_group()


class SmallCNN(torch.nn.Module):
    """conv -> SyncBN -> ReLU -> pool, twice, -> Linear: the ResNet-style CNN path (implicit-GEMM
    convolutions, BN, pooling, several gradient buckets) at a size a unit test can run."""

    def __init__(self):
        super().__init__()
        nn = tdp.nn
        self.conv1 = nn.Conv2d(4, 32, 3, padding=1, device="cuda")
        self.bn1 = nn.BatchNorm2d(32, device="cuda")
        self.pool1 = nn.MaxPool2d(2)
        self.conv2 = nn.Conv2d(32, 64, 3, padding=1, device="cuda")
        self.bn2 = nn.BatchNorm2d(64, device="cuda")
        self.pool2 = nn.MaxPool2d(2)
        self.fc = nn.Linear(64 * 4 * 4, 10, device="cuda")

    def forward(self, x):
        from tutorial_torch_distributed_data_parallel_amd import ops

        x = self.pool1(torch.relu(self.bn1(self.conv1(x))))
        x = self.pool2(torch.relu(self.bn2(self.conv2(x))))
        return self.fc(ops.flatten(x))


def _torch_cnn(m):
    import torch.nn as nn

    ref = nn.Sequential(nn.Conv2d(4, 32, 3, padding=1), nn.BatchNorm2d(32), nn.ReLU(),
                        nn.MaxPool2d(2), nn.Conv2d(32, 64, 3, padding=1), nn.BatchNorm2d(64),
                        nn.ReLU(), nn.MaxPool2d(2), nn.Flatten(), nn.Linear(64 * 4 * 4, 10))
    ref = ref.cuda()
    src = [m.conv1, m.bn1, m.conv2, m.bn2, m.fc]
    dst = [ref[0], ref[1], ref[4], ref[5], ref[9]]
    with torch.no_grad():
        for a, b in zip(src, dst):
            for (n, p) in a.named_parameters():
                getattr(b, n).copy_(p.contiguous())
    return ref


def _cnn_batch(r, step, n=8):
    g = torch.Generator(device="cuda").manual_seed(100 * step + r)
    x = torch.randn(n, 4, 16, 16, device="cuda", generator=g)
    return x.contiguous(memory_format=torch.channels_last), \
        torch.randint(0, 10, (n,), device="cuda", generator=g)


def captured_cnn_parity(rank, out_dir, steps=4, backend="peer"):
    """BASELINE config 5 in miniature: a conv + SyncBN + pool + Linear CNN whose gradients go
    through several buckets (small caps, split parameters) with the sharded fused update,
    CAPTURED with real peers == eager bitwise (parameters, running stats); both == the global-
    batch fp32 torch oracle."""
    import torch.nn as nn
    import torch.nn.functional as F

    tdp.init_process_group(backend)
    r, W = rt.get_rank(), rt.get_world_size()

    def build():
        torch.manual_seed(0)
        m = tdp.nn.convert_sync_batchnorm(SmallCNN())
        d = tdp.DDP(m, device_ids=[rt.device().index], bucket_cap_mb=0.02,
                    first_bucket_cap_mb=0.004, split_bucket_mb=0.01)
        o = tdp.optim.SGD(d.parameters(), lr=0.05, momentum=0.9)
        assert d.register_fused_optimizer(o)
        return m, d, o

    m1, d1, o1 = build()
    m2, d2, o2 = build()
    assert len(d2._bounds) - 1 >= 4, d2._bounds  # several buckets, split parameters
    ref = _torch_cnn(m1)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    sx = torch.empty(8, 4, 16, 16, device="cuda").contiguous(memory_format=torch.channels_last)
    sy = torch.empty(8, dtype=torch.long, device="cuda")

    def step1(x, y):
        o1.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(d1(x), y))
        o1.step()

    def step2():
        o2.zero_grad(set_to_none=True)
        tdp.ops.backward(tdp.ops.cross_entropy(d2(sx), sy))
        o2.step()

    _eager_vs_captured(step1, step2, [_cnn_batch(r, s) for s in range(steps)], sx, sy)
    for s in range(steps):
        ropt.zero_grad(set_to_none=True)
        xs, ys = zip(*[_cnn_batch(k, s) for k in range(W)])
        out = ref(torch.cat(xs))
        sum(F.cross_entropy(o, t) for o, t in zip(out.split(8), ys)).div(W).backward()
        ropt.step()
    _assert_bitwise(m1, m2, f"CNN W={W}")
    for (n, p), q in zip(m2.named_parameters(),
                         [ref[0].weight, ref[0].bias, ref[1].weight, ref[1].bias, ref[4].weight,
                          ref[4].bias, ref[5].weight, ref[5].bias, ref[9].weight, ref[9].bias]):
        torch.testing.assert_close(p.detach().contiguous(), q.detach().contiguous(), atol=1e-4,
                                   rtol=1e-3, msg=lambda s: f"CNN W={W} {n}: {s}")
    for a, b in ((m2.bn1, ref[1]), (m2.bn2, ref[5])):
        torch.testing.assert_close(a.running_mean, b.running_mean, atol=1e-5, rtol=1e-4)
        torch.testing.assert_close(a.running_var, b.running_var, atol=1e-4, rtol=1e-4)
    d1.check_replicas()
    d2.check_replicas()
    rt.barrier()
    tdp.destroy_process_group()
