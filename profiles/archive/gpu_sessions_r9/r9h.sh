#!/bin/bash
# peer vehicle: bench fallback ladder rungs + captured W>1 parity for BASELINE configs 3/4/5
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9h; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
export TDP_PEER_TIMEOUT_S=15
timeout -k 10 900 python -u -m pytest tests/test_peer_gpu.py tests/test_multigpu_rccl.py -v --timeout 300 --timeout-method thread -k "ladder or captured_syncbn or captured_accelerate or captured_cnn or rccl" > gpurun_out/r9h/pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|SKIP|ERROR" gpurun_out/r9h/pytest.log | tail -30; fatal $rc pytest

timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r9h/d.json 2>gpurun_out/r9h/d.err; fatal $? bench
python3 -c 'import json; d=json.load(open("gpurun_out/r9h/d.json")); print(d["ms_per_step"], d["config"]["rung"], d["config"]["fallbacks"], {k:v for k,v in d["diagnostics"].items() if "rehearsal" in k})'
echo done
