#!/bin/bash
# Tensor-sharded step after the native bias+ReLU backward / node-batch input: GPU tests, the
# per-rank proxy, its kernel table at W = 8.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r9o; export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_tensor_parallel_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r9o/pytest.log 2>&1; rc=$?; grep -E "passed|failed" gpurun_out/r9o/pytest.log | tail -3; fatal $rc pytest
timeout -k 10 300 python -u scripts/tp_rank_proxy.py > gpurun_out/r9o/proxy.jsonl 2> gpurun_out/r9o/proxy.err; rc=$?; grep W gpurun_out/r9o/proxy.jsonl; fatal $rc proxy
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r9o/kt -o kt -- python3 scripts/tp_rank_proxy.py --no-dp1 8 > gpurun_out/r9o/kt.log 2>&1; fatal $? kt
T=$(find gpurun_out/r9o/kt -name '*kernel_trace.csv' | head -1)
python3 scripts/step_timeline.py $T ce_fwd 2 > gpurun_out/r9o/tp8_timeline.md; cat gpurun_out/r9o/tp8_timeline.md
echo done
