"""Single-node launcher: 1-8 ranks, one process per MI355X, fail-fast.

Replaces the reference's ``mp.spawn`` (REF/multi-GPU-training-torch.py:269-279,
TORCH/multiprocessing/spawn.py:79-211) and its HTCondor submitter (REF/submit_job.py), which on
one 8xMI355X node has nothing to submit to (SURVEY.md §7.1 layer 3). Differences by design:
  * a free TCP port on 127.0.0.1 instead of the hard-coded localhost:12355 (two jobs on one node
    no longer collide);
  * every rank gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in its
    environment, so both entry points (native DDP and the Accelerate-style facade) become
    multi-rank under the same launcher (the reference's Accelerate script silently runs one
    process under plain python);
  * fail-fast is kept: the first rank that fails makes the launcher terminate the others
    (SIGTERM, then SIGKILL after a grace period) and re-raise the failing rank's traceback.

Two forms:
  ``spawn(fn, nprocs, args)``        -- call ``fn(rank, *args)`` in N spawned processes;
  ``python -m tutorial_torch_distributed_data_parallel_amd.parallel.launcher --nproc N
     script.py [args...]``           -- run a script N times (torchrun-like).
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import signal
import socket
import subprocess
import sys
import time
import traceback


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def _launcher_store(addr: str, nprocs: int):
    """The rendezvous store, hosted by the launcher itself on a port the OS picks at bind time
    (torchrun's agent store): no window between choosing a free port and rank 0 binding it, in
    which another socket can take it (seen as EADDRINUSE on a shared GPU box). Ranks connect as
    clients (TORCHELASTIC_USE_AGENT_STORE, torch/distributed/rendezvous.py). Returns
    (store or None, port, extra env)."""
    if nprocs <= 1:
        return None, free_port(addr), {}
    try:
        import datetime

        from torch.distributed import TCPStore

        store = TCPStore(addr, 0, nprocs, True, timeout=datetime.timedelta(minutes=30),
                         wait_for_workers=False)
        return store, int(store.port), {"TORCHELASTIC_USE_AGENT_STORE": "True"}
    except Exception:  # noqa: BLE001 - no torch store here: fall back to a probed free port
        return None, free_port(addr), {}


class ProcessRaisedException(RuntimeError):
    def __init__(self, msg, rank, pid):
        super().__init__(msg)
        self.rank, self.pid = rank, pid


class ProcessExitedException(RuntimeError):
    def __init__(self, msg, rank, pid, exit_code):
        super().__init__(msg)
        self.rank, self.pid, self.exit_code = rank, pid, exit_code


def _one_gpu_vehicle() -> bool:
    """Several ranks share one GPU through the peer / relay vehicles (parallel/peer.py,
    parallel/relay.py): they exchange device memory through IPC handles."""
    return os.environ.get("TDP_GPU_PEER", "0") == "1" or \
        os.environ.get("TDP_GPU_RELAY", "0") == "1"


def _rank_env(rank, nprocs, addr, port, local_offset=0):
    env = {"RANK": str(rank), "LOCAL_RANK": str(rank + local_offset),
           "WORLD_SIZE": str(nprocs), "LOCAL_WORLD_SIZE": str(nprocs), "MASTER_ADDR": addr,
           "MASTER_PORT": str(port)}
    # HSA_ENABLE_IPC_MODE_LEGACY: the ranks inherit whatever the node's environment says (the
    # MI355X pool this was built on exports 0 for every process: its host driver shares device
    # memory between processes by dmabuf only, for RCCL's intra-node buffers as for tensors).
    # The launcher sets it itself only for the one-GPU vehicles, whose cross-process device
    # memory is the whole mechanism, and never overrides an operator's explicit value.
    if _one_gpu_vehicle() and "HSA_ENABLE_IPC_MODE_LEGACY" not in os.environ:
        env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    return env


def _child(fn, rank, args, env, err_q):
    os.environ.update(env)
    try:
        fn(rank, *args)
    except KeyboardInterrupt:
        sys.exit(130)
    except BaseException:  # noqa: BLE001 - forward everything, like torch's _wrap
        err_q.put((rank, traceback.format_exc()))
        sys.exit(1)


def _terminate(procs, grace: float):
    for p in procs:
        if p.is_alive():
            p.terminate()
    deadline = time.time() + grace
    for p in procs:
        p.join(max(0.0, deadline - time.time()))
        if p.is_alive():
            p.kill()
            p.join()


def spawn(fn, nprocs: int, args=(), master_addr: str = "127.0.0.1",
          master_port: int | None = None, grace: float = 30.0, poll: float = 0.1):
    """Run ``fn(rank, *args)`` on ``nprocs`` spawned ranks; re-raise the first failure."""
    if not 1 <= nprocs:
        raise ValueError("nprocs must be >= 1")
    store, port, extra = (None, master_port, {}) if master_port else \
        _launcher_store(master_addr, nprocs)
    ctx = mp.get_context("spawn")
    err_q = ctx.SimpleQueue()
    procs = []
    for r in range(nprocs):
        env = dict(_rank_env(r, nprocs, master_addr, port), **extra)
        p = ctx.Process(target=_child, args=(fn, r, args, env, err_q), daemon=False)
        p.start()
        procs.append(p)
    try:
        while True:
            alive = False
            for r, p in enumerate(procs):
                if p.is_alive():
                    alive = True
                    continue
                if p.exitcode not in (0, None):
                    _terminate(procs, grace)
                    errs = []
                    while not err_q.empty():
                        errs.append(err_q.get())
                    if errs:
                        er, tb = errs[0]
                        raise ProcessRaisedException(
                            f"\n-- Process {er} terminated with the following error:\n{tb}", er,
                            procs[er].pid)
                    raise ProcessExitedException(
                        f"process {r} terminated with exit code {p.exitcode}", r, p.pid,
                        p.exitcode)
            if not alive:
                return
            time.sleep(poll)
    except KeyboardInterrupt:
        _terminate(procs, grace)
        raise


def run_script(nproc: int, argv, master_addr: str = "127.0.0.1", master_port: int | None = None,
               grace: float = 30.0, env_extra: dict | None = None, rank0_stdout=None) -> int:
    """torchrun-style: run ``python argv...`` nproc times with rank env; fail-fast.
    ``env_extra`` is added to every rank's environment; ``rank0_stdout`` (a file object)
    receives rank 0's stdout instead of the launcher's (bench.py relays it)."""
    store, port, extra = (None, master_port, {}) if master_port else \
        _launcher_store(master_addr, nproc)
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update(_rank_env(r, nproc, master_addr, port), **extra)
        if env_extra:
            env.update({k: str(v) for k, v in env_extra.items()})
        out = rank0_stdout if r == 0 and rank0_stdout is not None else None
        procs.append(subprocess.Popen([sys.executable, *argv], env=env, start_new_session=True,
                                      stdout=out))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0:
                    rc = code
                    for q in procs:  # fail-fast: stop the survivors
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
                    deadline = time.time() + grace
                    for q in procs:
                        try:
                            q.wait(max(0.1, deadline - time.time()))
                        except subprocess.TimeoutExpired:
                            os.killpg(q.pid, signal.SIGKILL)
                            q.wait()
                    procs = []
                    break
            time.sleep(0.1)
    except KeyboardInterrupt:
        for q in procs:
            os.killpg(q.pid, signal.SIGTERM)
        raise
    return rc


def main(argv=None):
    ap = argparse.ArgumentParser(description="launch N ranks of a training script on one node")
    ap.add_argument("--nproc", "--nproc-per-node", type=int, default=1, dest="nproc")
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if not 1 <= a.nproc <= 64:
        ap.error("--nproc must be in [1, 64]")
    return run_script(a.nproc, [a.script, *a.args], a.master_addr, a.master_port)


if __name__ == "__main__":
    sys.exit(main())
