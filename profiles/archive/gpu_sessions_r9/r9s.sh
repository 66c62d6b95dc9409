#!/bin/bash
# Tensor-sharded N > 1 diagnostics on the peer vehicle.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9s; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_tensor_parallel_gpu.py -x -v --timeout 300 --timeout-method thread -k "diagnostics or bench" > gpurun_out/r9s/pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/r9s/pytest.log | tail -8; fatal $rc pytest
TDP_GPU_PEER=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --parallel tensor > gpurun_out/r9s/peer_tp.json 2> gpurun_out/r9s/peer_tp.err; rc=$?; fatal $rc peer_tp
python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(d["ms_per_step"], d["config"]["rung"], d["config"]["selection"], d["diagnostics"])' gpurun_out/r9s/peer_tp.json
echo done
