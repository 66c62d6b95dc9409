#!/bin/bash
# Round 6 first look: changed GPU tests (TP accumulation with a late aux stream, bench labels),
# driver-shaped dp1 bench, the peer-vehicle N=2 default (DDP) record.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r10a; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 500 python -u -m pytest tests/test_tensor_parallel_gpu.py tests/test_bench_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r10a/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r10a/tests.log; grep -E "FAILED|Error" gpurun_out/r10a/tests.log | head -5; fatal $rc tests
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r10a/d1.json 2> gpurun_out/r10a/d1.err; fatal $? bench
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); g=d.get("diagnostics",{}); print(d["ms_per_step"], {k: g.get(k) for k in ("rehearsal_ms","rehearsal_over_dp1","rehearsal_schedule_over_dp1")})' gpurun_out/r10a/d1.json
TDP_GPU_PEER=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r10a/peer2.json 2> gpurun_out/r10a/peer2.err; fatal $? peer2
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); c=d["config"]; print(d["ms_per_step"], c["parallelism"], c["rung"], c["sync"]["replicas_identical"])' gpurun_out/r10a/peer2.json
echo done
