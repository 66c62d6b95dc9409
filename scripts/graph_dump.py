"""Run bench.py with every captured hipGraph described: node count by kind, edges, fork nodes
(> 1 successor) and join nodes (> 1 predecessor), read through the HIP graph API (ctypes) -- for
comparing the dp1 step's graph with its multi-GPU rehearsal's. Also tries hipGraphDebugDotPrint
into $DUMP_DIR/graph_<n>.dot.

    python scripts/graph_dump.py -- --steps 20 --warmup 5
"""
import ctypes
import json
import os
import runpy
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.abspath(os.environ.get("DUMP_DIR", os.path.join(ROOT, "gpurun_out", "graphs")))
os.makedirs(OUT, exist_ok=True)
_Base = torch.cuda.CUDAGraph
_n = [0]
KINDS = {0: "kernel", 1: "memcpy", 2: "memset", 3: "host", 4: "child", 5: "empty",
         6: "wait_event", 7: "event_record", 10: "mem_alloc", 11: "mem_free"}


def _hip():
    for name in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    raise OSError("libamdhip64 not found")


def describe(g):
    hip = _hip()
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(ctypes.c_void_p(g), None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(ctypes.c_void_p(g), nodes, ctypes.byref(n)) == 0
    kinds = {}
    for nd in nodes:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        k = KINDS.get(t.value, str(t.value))
        kinds[k] = kinds.get(k, 0) + 1
    e = ctypes.c_size_t(0)
    assert hip.hipGraphGetEdges(ctypes.c_void_p(g), None, None, ctypes.byref(e)) == 0
    src = (ctypes.c_void_p * e.value)()
    dst = (ctypes.c_void_p * e.value)()
    assert hip.hipGraphGetEdges(ctypes.c_void_p(g), src, dst, ctypes.byref(e)) == 0
    outd, ind = {}, {}
    for s, d in zip(src, dst):
        outd[s] = outd.get(s, 0) + 1
        ind[d] = ind.get(d, 0) + 1
    return {"nodes": n.value, "kinds": kinds, "edges": e.value,
            "forks": sum(1 for v in outd.values() if v > 1),
            "joins": sum(1 for v in ind.values() if v > 1),
            "roots": sum(1 for nd in nodes if nd not in ind),
            "sinks": sum(1 for nd in nodes if nd not in outd)}


class DumpingGraph(_Base):
    def __new__(cls, *args, **kwargs):
        return _Base.__new__(cls, True)

    def __init__(self, *args, **kwargs):
        super().__init__(keep_graph=True)

    def capture_end(self):
        super().capture_end()
        i = _n[0]
        _n[0] += 1
        try:
            info = describe(self.raw_cuda_graph())
        except Exception as ex:  # noqa: BLE001 -- diagnostics only
            info = {"error": repr(ex)}
        try:
            path = os.path.join(OUT, f"graph_{i}.dot")
            rc = _hip().hipGraphDebugDotPrint(ctypes.c_void_p(self.raw_cuda_graph()),
                                              path.encode(), ctypes.c_uint(1))
            info["dot_rc"] = rc
        except Exception as ex:  # noqa: BLE001
            info["dot_error"] = repr(ex)
        print(f"[graph_dump] graph {i}: {json.dumps(info)}", file=sys.stderr, flush=True)


torch.cuda.CUDAGraph = DumpingGraph
args = sys.argv[1:]
if args[:1] == ["--"]:
    args = args[1:]
sys.argv = [os.path.join(ROOT, "bench.py")] + args
runpy.run_path(sys.argv[0], run_name="__main__")
